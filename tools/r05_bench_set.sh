#!/bin/bash
# Round-5 measurement set: the driver's default line (C2), C3 with its defaults, and a C3 kernel trace (rocprofv3)
# showing the in-flight LocalBundleAdjustment calls beside the tracking streams.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/bench_c2_r05.json 2> gpurun_out/bench_c2_r05.err || exit $?
timeout -k 10 400 python bench.py --config c3 > gpurun_out/bench_c3_r05.json 2> gpurun_out/bench_c3_r05.err || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
GPU_MAX_HW_QUEUES=16 SPSLAM_BENCH_CHILD=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o c3 -- \
  python bench.py --config c3 --steps 10 --no-cpu-baseline --ate-frames 0 --single-sequence-frames 0 \
  --closed-loop-steps 0 > gpurun_out/prof_c3.json 2> gpurun_out/prof_c3.err || exit $?
