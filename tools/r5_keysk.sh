set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd ${GRAFT_REPO_ROOT:-.}
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_match.py tests/test_gpu_sequence.py tests/test_gpu_pipeline.py > gpurun_out/kk_tests.log 2>&1 || exit 1
P="python tools/b1_prof.py --frames 300 --lookahead 2 --max-inflight 1"
B="python bench.py --config c2 --steps 60 --warmup 5 --no-cpu-baseline --ate-frames 0 --closed-loop-steps 0 --single-sequence-frames 0"
for r in 1 2; do
  timeout -k 10 200 $P > gpurun_out/kk_new_$r.txt 2>&1 || exit 1
  SPSLAM_GPU_LIB=sp-slam_amd/libspslam_gpu_prev.so timeout -k 10 200 $P > gpurun_out/kk_prev_$r.txt 2>&1 || exit 1
  timeout -k 10 300 $B > gpurun_out/kk_c2_new_$r.json 2>/dev/null || exit 1
  SPSLAM_GPU_LIB=sp-slam_amd/libspslam_gpu_prev.so timeout -k 10 300 $B > gpurun_out/kk_c2_prev_$r.json 2>/dev/null || exit 1
done
