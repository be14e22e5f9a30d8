set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd ${GRAFT_REPO_ROOT:-.}
B="python bench.py --config c2 --steps 40 --warmup 5 --no-cpu-baseline --ate-frames 0 --closed-loop-steps 0 --single-sequence-frames 0"
for r in 1 2; do
  for b in 256 320 384 512; do
    timeout -k 10 300 $B --batch $b > gpurun_out/batch_${b}_$r.json 2>/dev/null || exit 1
  done
done
