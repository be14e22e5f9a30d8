set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r01_gpu_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/bench.json 2> gpurun_out/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_prof.json 2> gpurun_out/prof.err
echo EXIT $?
