set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd ${GRAFT_REPO_ROOT:-.}
for v in seg512 seg768; do
  SPSLAM_GPU_LIB=sp-slam_amd/libspslam_gpu_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_planes.py > gpurun_out/seg_tests_$v.log 2>&1 || exit 1
done
B="python bench.py --config c2 --steps 60 --warmup 5 --no-cpu-baseline --ate-frames 0 --closed-loop-steps 0 --single-sequence-frames 0"
for r in 1 2; do
  for v in "" seg512 seg768; do
    SPSLAM_GPU_LIB=sp-slam_amd/libspslam_gpu${v:+_$v}.so timeout -k 10 300 $B > gpurun_out/seg_c2_${v:-def}_$r.json 2>/dev/null || exit 1
  done
done
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sequence.py -k c3_local > gpurun_out/seg_c3lm.log 2>&1
