set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-.}
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_frame.py tests/test_gpu_sequence.py > gpurun_out/fr_tests.log 2>&1 || exit 1
P="python tools/b1_prof.py --frames 300 --lookahead 2 --max-inflight 1"
B="python bench.py --config c2 --steps 60 --warmup 5 --no-cpu-baseline --ate-frames 0 --closed-loop-steps 0 --single-sequence-frames 0"
for r in 1 2; do
  timeout -k 10 200 $P > gpurun_out/fr_new_$r.txt 2>&1 || exit 1
  SPSLAM_GPU_LIB=sp-slam_amd/libspslam_gpu_prev.so timeout -k 10 200 $P > gpurun_out/fr_prev_$r.txt 2>&1 || exit 1
done
timeout -k 10 300 $B > gpurun_out/fr_c2_new.json 2>/dev/null || exit 1
SPSLAM_GPU_LIB=sp-slam_amd/libspslam_gpu_prev.so timeout -k 10 300 $B > gpurun_out/fr_c2_prev.json 2>/dev/null || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/fr_ser -o run -- python3 tools/b1_prof.py --frames 60 --serial > gpurun_out/fr_ser.log 2>&1
