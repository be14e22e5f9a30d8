set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd ${GRAFT_REPO_ROOT:-.}
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_bow.py tests/test_gpu_sequence.py > gpurun_out/b1b_tests.log 2>&1 || exit 1
P="python tools/b1_prof.py --frames 300 --lookahead 2 --max-inflight 1"
for r in 1 2; do
  timeout -k 10 200 $P > gpurun_out/b1b_new_$r.txt 2>&1 || exit 1
  SPSLAM_GPU_LIB=sp-slam_amd/libspslam_gpu_old.so timeout -k 10 200 $P > gpurun_out/b1b_old_$r.txt 2>&1 || exit 1
done
timeout -k 10 200 python tools/b1_prof.py --frames 200 --serial > gpurun_out/b1b_new_serial.txt 2>&1 || exit 1
SPSLAM_GPU_LIB=sp-slam_amd/libspslam_gpu_ladiag.so timeout -k 10 200 python tools/b1_prof.py --frames 100 --serial > gpurun_out/b1b_ladiag.txt 2>&1 || exit 1
