set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd ${GRAFT_REPO_ROOT:-.}
B="python bench.py --config c2 --steps 60 --warmup 5 --no-cpu-baseline --ate-frames 0 --closed-loop-steps 0 --single-sequence-frames 0"
P="python tools/b1_prof.py --frames 300 --lookahead 2 --max-inflight 1"
for r in 1 2; do
  for S in 4 2; do
    SPSLAM_POSE_SPEC=$S timeout -k 10 300 $B > gpurun_out/spec${S}_c2_$r.json 2>/dev/null || exit 1
    SPSLAM_POSE_SPEC=$S timeout -k 10 200 $P > gpurun_out/spec${S}_b1_$r.txt 2>&1 || exit 1
  done
done
