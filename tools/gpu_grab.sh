# One GPU call: grab + e2e step tests, C2 bench (CPU baseline + ATE), rocprof kernel stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-grab}
timeout -k 10 400 python -u -m pytest tests/test_gpu_grab.py tests/test_gpu_pipeline.py -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/${TAG}_c2.json 2> gpurun_out/${TAG}_c2.err && \
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_prof.json 2> gpurun_out/${TAG}_prof.err
echo EXIT $?
