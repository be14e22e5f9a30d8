#!/bin/bash
# Round 6: the barrier-free plane wavefront (plane_wave_kernel, default) against round 5's barrier wavefront
# (SPSLAM_PLANE_WAVE_BARRIER=1): B = 1 serial latency, interleaved, then a kernel trace of the serial B = 1 step.
#   bash tools/ab_plane_wave.sh TAG
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
TAG=${1:-pw}
mkdir -p gpurun_out
for r in 1 2; do
  for v in 0 1; do
    SPSLAM_PLANE_WAVE_BARRIER=$v timeout -k 10 300 python tools/b1_prof.py --serial --frames 80 \
      > gpurun_out/${TAG}_b1_barrier${v}_$r.txt 2>/dev/null || exit 1
    echo "barrier=$v round $r: $(tail -1 gpurun_out/${TAG}_b1_barrier${v}_$r.txt)"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_b1trace -o run -- \
  python3 tools/b1_prof.py --serial --frames 20 > gpurun_out/${TAG}_b1trace.log 2>&1 || exit 1
