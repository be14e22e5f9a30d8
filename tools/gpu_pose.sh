# One GPU call: pose / LBA / e2e parity, pose scaling study, C2 bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-pose}
timeout -k 10 400 python -u -m pytest tests/test_gpu_pose.py tests/test_gpu_pipeline.py tests/test_gpu_lba.py -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 && \
timeout -k 10 240 python tools/pose_scaling.py > gpurun_out/${TAG}_scaling.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_c2.json 2> gpurun_out/${TAG}_c2.err
echo EXIT $?
