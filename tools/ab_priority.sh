# Interleaved A/B of stream-priority layouts of the pipelined C2 step (3 rounds; gpurun_out/ab_prio_*.json).
cd ${GRAFT_REPO_ROOT:-.}
B="python bench.py --config c2 --steps 40 --warmup 5 --no-cpu-baseline --ate-frames 0 --closed-loop-steps 0"
for r in 1 2 3; do
  timeout -k 10 300 $B > gpurun_out/ab_prio_base_$r.json 2>/dev/null || exit 1
  timeout -k 10 300 $B --planes-priority > gpurun_out/ab_prio_planes_$r.json 2>/dev/null || exit 1
  timeout -k 10 300 $B --planes-priority --no-tail-priority > gpurun_out/ab_prio_planesonly_$r.json 2>/dev/null || exit 1
  timeout -k 10 300 $B --planes-priority --orb-priority > gpurun_out/ab_prio_all_$r.json 2>/dev/null || exit 1
done
for f in gpurun_out/ab_prio_*.json; do python3 -c "import json,sys; d=json.load(open('$f')); print('$f', round(d['ms_per_step'],3))"; done
