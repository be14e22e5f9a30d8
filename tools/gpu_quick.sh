# One GPU call: selected tests, then the C2 bench and its rocprof kernel stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-quick}
timeout -k 10 500 python -u -m pytest "$@" -x -v --timeout 400 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_c2.json 2> gpurun_out/${TAG}_c2.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > /dev/null 2> gpurun_out/${TAG}_prof.err
echo EXIT $?
