# One GPU call: C2 rocprof kernel trace (pipelined, 8 HW queues) for the per-queue busy analysis.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8
TAG=${1:-prof}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --ate-frames 0 > gpurun_out/${TAG}_prof.json 2> gpurun_out/${TAG}_prof.err
echo EXIT $?
