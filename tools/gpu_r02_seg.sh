# One GPU call: segmentation phase stamps (1024 and 512 threads) and the ORB stage alone.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 python tools/seg_phases.py > gpurun_out/seg_phases_1024.txt 2>&1 && \
SPSLAM_GPU_LIB=sp-slam_amd/libspslam_gpu_seg512.so timeout -k 10 200 python tools/seg_phases.py > gpurun_out/seg_phases_512.txt 2>&1
echo EXIT $?
