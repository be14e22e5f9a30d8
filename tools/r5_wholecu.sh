set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd ${GRAFT_REPO_ROOT:-.}
B="python bench.py --config c2 --steps 60 --warmup 5 --no-cpu-baseline --ate-frames 0 --closed-loop-steps 0 --single-sequence-frames 0"
for r in 1 2 3; do
  timeout -k 10 300 $B > gpurun_out/wcu_def_$r.json 2>/dev/null || exit 1
  SPSLAM_POSE_WHOLE_CU=1 timeout -k 10 300 $B > gpurun_out/wcu_pad_$r.json 2>/dev/null || exit 1
done
