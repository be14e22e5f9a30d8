#!/bin/bash
# C3 step time against the LocalBundleAdjustment team size (workgroups per local map), interleaved.
# usage: tools/ab_c3_team.sh "1 3 4 5" [rounds] [depths]
set -o pipefail
teams=${1:-"1 4 5"}; rounds=${2:-2}; depths=${3:-0}
mkdir -p gpurun_out
for r in $(seq 1 $rounds); do
  for d in $depths; do
  for t in $teams; do
    f=gpurun_out/c3_team${t}_d${d}_$r
    timeout -k 10 240 python bench.py --config c3 --steps 20 --lba-team $t --lba-depth $d --no-cpu-baseline --ate-frames 0 \
      --single-sequence-frames 0 --closed-loop-steps 0 > $f.json 2> $f.err || exit $?
    python3 -c "import json,sys; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); print('team $t depth $d round $r', round(d['value']), d['ms_per_step'], d['parity_ok'])"
  done
  done
done
