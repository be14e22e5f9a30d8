# One GPU call: all GPU tests, the C2 bench (BASELINE metric) + C3 (with LBA), rocprof kernel stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-run}
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err && \
timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 2 > gpurun_out/${TAG}_bench_c3.json 2> gpurun_out/${TAG}_bench_c3.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_bench_prof.json 2> gpurun_out/${TAG}_prof.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof_c3 -o run -- python3 bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_bench_prof_c3.json 2> gpurun_out/${TAG}_prof_c3.err
echo EXIT $?
