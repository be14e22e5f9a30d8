set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd ${GRAFT_REPO_ROOT:-.}
B="python bench.py --config c2 --steps 60 --warmup 5 --no-cpu-baseline --ate-frames 0 --closed-loop-steps 0 --single-sequence-frames 0"
for r in 1 2 3; do
  for v in "" base oldoct oldplane; do
    L=sp-slam_amd/libspslam_gpu${v:+_$v}.so
    SPSLAM_GPU_LIB=$L timeout -k 10 300 $B > gpurun_out/iso_c2_${v:-new}_$r.json 2>/dev/null || exit 1
  done
done
