# One GPU call: every GPU test, C2 (BASELINE metric) bench with CPU baseline + ATE, C3 and C5 benches,
# rocprof kernel stats of C2, then the FETCH_SIZE / WRITE_SIZE PMC passes of C2 (separate runs).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-final}
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/${TAG}_c2.json 2> gpurun_out/${TAG}_c2.err && \
timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 2 > gpurun_out/${TAG}_c3.json 2> gpurun_out/${TAG}_c3.err && \
timeout -k 10 300 python bench.py --config c5 --steps 5 --warmup 2 --batch 64 > gpurun_out/${TAG}_c5.json 2> gpurun_out/${TAG}_c5.err && \
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_prof.json 2> gpurun_out/${TAG}_prof.err && \
GPU_MAX_HW_QUEUES=8 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/${TAG}_pmc_fetch -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_pmc_fetch.log 2>&1 && \
GPU_MAX_HW_QUEUES=8 timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/${TAG}_pmc_write -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_pmc_write.log 2>&1
echo EXIT $?
