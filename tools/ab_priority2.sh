# Interleaved A/B/C of stream priorities at the current HEAD (3 rounds; gpurun_out/ab_prio2_*.json)
cd ${GRAFT_REPO_ROOT:-.}
B="python bench.py --config c2 --steps 40 --warmup 5 --no-cpu-baseline --ate-frames 0 --closed-loop-steps 0"
for r in 1 2 3; do
  timeout -k 10 300 $B > gpurun_out/ab_prio2_base_$r.json 2>/dev/null || exit 1
  timeout -k 10 300 $B --orb-priority > gpurun_out/ab_prio2_orb_$r.json 2>/dev/null || exit 1
  timeout -k 10 300 $B --orb-priority --no-tail-priority > gpurun_out/ab_prio2_orbnotail_$r.json 2>/dev/null || exit 1
done
for f in gpurun_out/ab_prio2_*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', round(d['ms_per_step'],3))"; done
