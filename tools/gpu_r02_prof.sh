# One GPU call: stages alone (tools/stage_bench.py) and a rocprof kernel trace of the pipelined C2 bench.
#   TAG=<name> CFG=c2 bash tools/gpu_r02_prof.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8
TAG=${TAG:-prof}
CFG=${CFG:-c2}
timeout -k 10 300 python tools/stage_bench.py --config $CFG > gpurun_out/${TAG}_stages.txt 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --config $CFG --steps 10 --warmup 2 --no-cpu-baseline --ate-frames 0 > gpurun_out/${TAG}_prof.json 2> gpurun_out/${TAG}_prof.err
echo EXIT $?
