#!/bin/bash
# B = 1 serial step under rocprofv3 --kernel-trace (tools/b1_prof.py --serial), for tools/timeline.py:
#   bash tools/b1_timeline.sh TAG   -> gpurun_out/TAG_b1_prof/run_results.db, gpurun_out/TAG_b1_timeline.txt
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
TAG=$1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_b1_prof -o run -- \
    python3 tools/b1_prof.py --serial --frames 30 > gpurun_out/${TAG}_b1_prof.txt 2>&1 || exit 1
python3 tools/timeline.py gpurun_out/${TAG}_b1_prof/run_results.db 3 > gpurun_out/${TAG}_b1_timeline.txt || exit 1
tail -3 gpurun_out/${TAG}_b1_timeline.txt
