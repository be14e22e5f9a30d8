set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-.}
SPSLAM_GPU_LIB=sp-slam_amd/libspslam_gpu_ladiag.so timeout -k 10 200 python tools/b1_prof.py --frames 100 --serial > gpurun_out/madiag.txt 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/b1tl_pipe2 -o run -- python3 tools/b1_prof.py --frames 150 --lookahead 2 --max-inflight 1 > gpurun_out/b1tl_pipe2.log 2>&1
