# One GPU call: pose parity (incl. bit-exact device-order), then the pose phase profile and stages alone.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8
TAG=${TAG:-pose}
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_pose.py > gpurun_out/${TAG}_tests.log 2>&1 && \
SPSLAM_GPU_LIB=sp-slam_amd/libspslam_gpu_prof.so timeout -k 10 300 python tools/pose_phases.py > gpurun_out/${TAG}_pose_phases.txt 2>&1 && \
for s in 1 2; do SPSLAM_POSE_SPEC=$s SPSLAM_GPU_LIB=sp-slam_amd/libspslam_gpu_prof.so timeout -k 10 300 python tools/pose_phases.py > gpurun_out/${TAG}_pose_phases_spec$s.txt 2>&1 || exit 1; done && \
timeout -k 10 300 python tools/stage_bench.py > gpurun_out/${TAG}_stages.txt 2>&1
echo EXIT $?
