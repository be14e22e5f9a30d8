# One GPU call: PoseOptimization phase profile (diagnostic build) and every stage timed alone.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8
TAG=${TAG:-ph}
CFG=${CFG:-c2}
SPSLAM_GPU_LIB=sp-slam_amd/libspslam_gpu_prof.so timeout -k 10 300 python tools/pose_phases.py --config $CFG > gpurun_out/${TAG}_pose_phases.txt 2>&1 && \
timeout -k 10 300 python tools/stage_bench.py --config $CFG > gpurun_out/${TAG}_stages.txt 2>&1
echo EXIT $?
