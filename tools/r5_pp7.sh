set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd ${GRAFT_REPO_ROOT:-.}
SPSLAM_GPU_LIB=sp-slam_amd/libspslam_gpu_prof.so timeout -k 10 200 python tools/pose_phases.py --batch 1 > gpurun_out/pp7_b1.txt 2>&1 || exit 1
SPSLAM_GPU_LIB=sp-slam_amd/libspslam_gpu_prof.so timeout -k 10 200 python tools/pose_phases.py --batch 256 > gpurun_out/pp7_b256.txt 2>&1 || exit 1
