# One GPU call: plane parity tests, then a rocprofv3 kernel trace + stats of the pipelined C2 bench.
#   TAG=<name> bash tools/gpu_prof_c2.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8
TAG=${TAG:-prof}
CFG=${CFG:-c2}
timeout -k 10 400 python -u -m pytest tests/test_gpu_planes.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --config $CFG --steps 10 --warmup 2 --no-cpu-baseline --ate-frames 0 > gpurun_out/${TAG}_prof.json 2> gpurun_out/${TAG}_prof.err
echo EXIT $?
