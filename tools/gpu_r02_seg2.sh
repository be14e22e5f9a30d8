# One GPU call: plane parity, segmentation phases, C2 bench, stages alone.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8
TAG=${TAG:-seg2}
timeout -k 10 600 python -u -m pytest tests/test_gpu_planes.py tests/test_gpu_supposed.py -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/${TAG}_tests.log 2>&1 && \
timeout -k 10 200 python tools/seg_phases.py > gpurun_out/${TAG}_phases.txt 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --ate-frames 0 > gpurun_out/${TAG}_bench_c2.json 2> gpurun_out/${TAG}_bench_c2.err && \
timeout -k 10 300 python tools/stage_bench.py > gpurun_out/${TAG}_stages.txt 2>&1
echo EXIT $?
