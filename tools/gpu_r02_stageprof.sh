# One GPU call: every stage alone (tools/stage_bench.py) under a rocprof kernel trace: per-kernel durations
# without the other streams' contention.   TAG=<name> CFG=c2 bash tools/gpu_r02_stageprof.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8
TAG=${TAG:-sp}
CFG=${CFG:-c2}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run -- python3 tools/stage_bench.py --config $CFG > gpurun_out/${TAG}_stages.txt 2>&1 && \
timeout -k 10 120 python3 tools/orb_bench.py > gpurun_out/${TAG}_orb.txt 2>&1
echo EXIT $?
