#!/bin/bash
# Round-6 closing measurements, in two GPU calls (each step under its own limit, the first failure ends the call):
#   bash tools/gpu_r6_final.sh A   GPU test suite, smoke, the driver's default bench line (C2), its rocprofv3
#                                  kernel stats and the PMC traffic passes of the same library
#   bash tools/gpu_r6_final.sh B   the other configs' bench lines (C3 room window, C1 proxy, C4, C5; CONFIGS=... a subset)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
case $1 in
  A)
    bash tools/gpu_run.sh ${TAG:-r6f} tests smoke || exit 1
    timeout -k 10 600 python bench.py > gpurun_out/${TAG:-r6f}_bench_c2.json 2> gpurun_out/${TAG:-r6f}_bench_c2.err || exit 1
    cut -c1-300 gpurun_out/${TAG:-r6f}_bench_c2.json
    bash tools/gpu_run.sh ${TAG:-r6f} prof:c2 pmc:c2 || exit 1 ;;
  B)
    for c in ${CONFIGS:-c3 c1 c4 c5}; do
      # (a heartbeat line a minute: C5's CPU baseline and ATE legs run minutes without output)
      timeout -k 10 900 python bench.py --config $c > gpurun_out/${TAG:-r6f}_bench_$c.json 2> gpurun_out/${TAG:-r6f}_bench_$c.err &
      pid=$!
      while kill -0 $pid 2> /dev/null; do sleep 60; echo "   $c running $(date +%T)"; done
      wait $pid || exit 1
      cut -c1-200 gpurun_out/${TAG:-r6f}_bench_$c.json
    done ;;
esac
echo "== done $(date +%T)"
