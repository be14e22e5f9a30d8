#!/bin/bash
# Interleaved A/B of library variants on LocalBundleAdjustment:
#   bash tools/ab_lba_lib.sh TAG ROUNDS LIB_A LIB_B ...
# per round and library: tools/lba_bench.py (51 maps of 12 keyframes, teams 5 / 1 / 16) and tools/lba_single.py
# (one map at a time, teams 1 / 5 / 16, one CPU timing) -> gpurun_out/TAG_{bench,single}_<i>_<r>.txt
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
TAG=$1; R=$2; shift 2
mkdir -p gpurun_out
for r in $(seq 1 $R); do
  i=0
  for L in "$@"; do
    SPSLAM_GPU_LIB=$L timeout -k 10 300 python tools/lba_bench.py --config c3s --reps 3 --team 5 1 16 \
        > gpurun_out/${TAG}_bench_${i}_$r.txt 2>&1 || exit 1
    SPSLAM_GPU_LIB=$L timeout -k 10 300 python tools/lba_single.py --reps 5 --cpu-reps 1 \
        > gpurun_out/${TAG}_single_${i}_$r.txt 2>&1 || exit 1
    echo "[$L] round $r"; grep "team" gpurun_out/${TAG}_bench_${i}_$r.txt | cut -c1-60
    i=$((i+1))
  done
done
