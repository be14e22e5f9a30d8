set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-.}
export GPU_MAX_HW_QUEUES=8
B="python3 bench.py --config c2 --steps 10 --warmup 3 --no-cpu-baseline --ate-frames 0 --closed-loop-steps 0 --single-sequence-frames 0"
SPSLAM_GPU_LIB=sp-slam_amd/libspslam_gpu.so timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tl_new -o run -- $B > gpurun_out/tl_new.log 2>&1 &&
SPSLAM_GPU_LIB=sp-slam_amd/libspslam_gpu_base.so timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tl_base -o run -- $B > gpurun_out/tl_base.log 2>&1
