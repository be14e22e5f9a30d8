set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd ${GRAFT_REPO_ROOT:-.}
W=sp-slam_amd/libspslam_gpu_posew7.so
SPSLAM_GPU_LIB=$W timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_pose.py tests/test_gpu_sequence.py > gpurun_out/pw_tests.log 2>&1 || exit 1
P="python tools/b1_prof.py --frames 300 --lookahead 2 --max-inflight 1"
for r in 1 2; do
  SPSLAM_GPU_LIB=$W timeout -k 10 200 $P > gpurun_out/pw_w7_$r.txt 2>&1 || exit 1
  timeout -k 10 200 $P > gpurun_out/pw_w4_$r.txt 2>&1 || exit 1
done
SPSLAM_GPU_LIB=$W timeout -k 10 200 python tools/b1_prof.py --frames 200 --serial > gpurun_out/pw_w7_serial.txt 2>&1 || exit 1
timeout -k 10 200 python tools/b1_prof.py --frames 200 --serial > gpurun_out/pw_w4_serial.txt 2>&1 || exit 1
B="python bench.py --config c2 --steps 60 --warmup 5 --no-cpu-baseline --ate-frames 0 --closed-loop-steps 0 --single-sequence-frames 0"
for r in 1 2; do
  SPSLAM_GPU_LIB=$W timeout -k 10 300 $B > gpurun_out/pw_c2_w7_$r.json 2>/dev/null || exit 1
  timeout -k 10 300 $B > gpurun_out/pw_c2_w4_$r.json 2>/dev/null || exit 1
done
