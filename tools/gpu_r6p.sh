#!/bin/bash
# One GPU call (round 6): the LBA layout rule and the refinement scan change under test, B = 1 phases, a C2 kernel
# trace, the C3 in-flight depth sweep and the C2 stream-priority A/B.  Steps chained: the first failure ends the call.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
bash tools/gpu_run.sh r6p tests:tests/test_gpu_planes.py,tests/test_gpu_lba_large.py,tests/test_gpu_lba.py \
    py:tools/lba_single.py py:tools/seg_phases.py:--batch_1 prof:c2 || exit 1
timeout -k 10 200 python tools/b1_prof.py --serial --frames 80 > gpurun_out/r6p_b1_serial.txt 2>&1 || exit 1
AB_CONFIG=c3 AB_STEPS=20 bash tools/ab_env.sh r6p_c3 1 "-- --lba-depth 2" "-- --lba-depth 3" "-- --lba-depth 4" \
    > gpurun_out/r6p_ab_c3.txt 2>&1 || exit 1
bash tools/ab_env.sh r6p_prio 2 "--" "-- --orb-priority" "-- --planes-priority" > gpurun_out/r6p_ab_prio.txt 2>&1 || exit 1
echo done
