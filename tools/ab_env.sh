# Interleaved A/B of step variants selected by bench flags / environment on the pipelined C2 step (AB_CONFIG,
# AB_STEPS: another config / step count):
#   bash tools/ab_env.sh TAG ROUNDS "VARIANT_A" "VARIANT_B" ["VARIANT_C" ...]
# each VARIANT is "ENV=VAL ... -- bench flags" (either part may be empty); gpurun_out/ab_TAG_<i>_<r>.json
cd ${GRAFT_REPO_ROOT:-.}
TAG=$1; R=$2; shift 2
B="python bench.py --config ${AB_CONFIG:-c2} --steps ${AB_STEPS:-40} --warmup 5 --no-cpu-baseline --ate-frames 0 --closed-loop-steps 0 --single-sequence-frames 0"
for r in $(seq 1 $R); do
  i=0
  for v in "$@"; do
    envs="${v%%--*}"; flags="${v#*--}"; [ "$flags" = "$v" ] && flags=""
    env $envs timeout -k 10 300 $B $flags > gpurun_out/ab_${TAG}_${i}_$r.json 2>/dev/null || exit 1
    i=$((i+1))
  done
done
for f in gpurun_out/ab_${TAG}_*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', round(d['ms_per_step'],3), round(d['value']))"; done
