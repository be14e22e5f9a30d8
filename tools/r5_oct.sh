# octree A/B: parity of the default library, then ORB alone and the pipelined C2 step per library variant
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd ${GRAFT_REPO_ROOT:-.}
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_orb.py > gpurun_out/oct_tests.log 2>&1 || exit 1
for r in 1 2; do
  for v in "" octold octk32 octk0; do
    L=sp-slam_amd/libspslam_gpu${v:+_$v}.so
    SPSLAM_GPU_LIB=$L timeout -k 10 120 python tools/orb_bench.py 256 2>/dev/null | sed "s/^/${v:-new} /" >> gpurun_out/oct_orb.txt || exit 1
  done
done
B="python bench.py --config c2 --steps 40 --warmup 5 --no-cpu-baseline --ate-frames 0 --closed-loop-steps 0 --single-sequence-frames 0"
for r in 1 2; do
  for v in "" octold; do
    L=sp-slam_amd/libspslam_gpu${v:+_$v}.so
    SPSLAM_GPU_LIB=$L timeout -k 10 300 $B > gpurun_out/oct_c2_${v:-new}_$r.json 2>/dev/null || exit 1
  done
done
