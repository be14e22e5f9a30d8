# One GPU call: ORB parity, ORB alone (per-kind times), the C2 bench without ATE.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8
TAG=${TAG:-orb}
timeout -k 10 600 python -u -m pytest tests/test_gpu_orb.py tests/test_gpu_pipeline.py -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/${TAG}_tests.log 2>&1 && \
timeout -k 10 120 python tools/orb_bench.py > gpurun_out/${TAG}_orb.txt 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --ate-frames 0 > gpurun_out/${TAG}_bench_c2.json 2> gpurun_out/${TAG}_bench_c2.err
echo EXIT $?
