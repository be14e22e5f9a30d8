# One GPU call: LBA parity tests, C3 bench, C3 rocprof kernel stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-lba}
timeout -k 10 300 python -u -m pytest tests/test_gpu_lba.py -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_bench_c3.json 2> gpurun_out/${TAG}_bench_c3.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof_c3 -o run -- python3 bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_bench_prof_c3.json 2> gpurun_out/${TAG}_prof_c3.err
echo EXIT $?
