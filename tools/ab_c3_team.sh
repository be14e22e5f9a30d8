#!/bin/bash
# C3 step time against the LocalBundleAdjustment team size (workgroups per local map), interleaved.
# usage: tools/ab_c3_team.sh "1 3 4 5" [rounds]
set -o pipefail
teams=${1:-"1 4 5"}; rounds=${2:-2}
mkdir -p gpurun_out
for r in $(seq 1 $rounds); do
  for t in $teams; do
    SPSLAM_LBA_TEAM=$t timeout -k 10 240 python bench.py --config c3 --steps 20 --no-cpu-baseline --ate-frames 0 \
      --single-sequence-frames 0 --closed-loop-steps 0 > gpurun_out/c3_team${t}_$r.json 2> gpurun_out/c3_team${t}_$r.err || exit $?
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/c3_team${t}_$r.json').read().strip().splitlines()[-1]); print('team $t round $r', round(d['value']), d['ms_per_step'])"
  done
done
