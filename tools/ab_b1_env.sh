#!/bin/bash
# Interleaved A/B of B = 1 serial latency (tools/b1_prof.py --serial) under environment variants:
#   bash tools/ab_b1_env.sh TAG ROUNDS "ENV=VAL ..." "ENV=VAL ..." [...]
# B1_ARGS replaces the b1_prof arguments (default "--serial --frames 80"; e.g. "--lookahead 2 --max-inflight 1
# --frames 120" for bench.py's pipelined single_sequence line).
# gpurun_out/TAG_b1_<i>_<r>.txt, a summary line per run on stdout.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
TAG=$1; R=$2; shift 2
mkdir -p gpurun_out
for r in $(seq 1 $R); do
  i=0
  for v in "$@"; do
    env $v timeout -k 10 300 python tools/b1_prof.py ${B1_ARGS:---serial --frames 80} > gpurun_out/${TAG}_b1_${i}_$r.txt 2>/dev/null || exit 1
    echo "[$v] round $r: $(tail -1 gpurun_out/${TAG}_b1_${i}_$r.txt)"
    i=$((i+1))
  done
done
