set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd ${GRAFT_REPO_ROOT:-.}
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_planes.py tests/test_gpu_supposed.py tests/test_gpu_sequence.py > gpurun_out/cf_tests.log 2>&1 || exit 1
B="python bench.py --config c2 --steps 60 --warmup 5 --no-cpu-baseline --ate-frames 0 --closed-loop-steps 0 --single-sequence-frames 0"
for r in 1 2; do
  timeout -k 10 300 $B > gpurun_out/cf_new_$r.json 2>/dev/null || exit 1
  SPSLAM_GPU_LIB=sp-slam_amd/libspslam_gpu_old.so timeout -k 10 300 $B > gpurun_out/cf_old_$r.json 2>/dev/null || exit 1
done
