# One GPU call (round 2): GPU tests, then the C2 bench (BASELINE metric) and the C4 (ICL) bench.
#   TAG=<name> bash tools/gpu_r02.sh [pytest selection...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8
TAG=${TAG:-r02}
SEL=${@:-tests -m gpu}
timeout -k 10 900 python -u -m pytest $SEL -x -v --timeout 400 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/${TAG}_bench_c2.json 2> gpurun_out/${TAG}_bench_c2.err && \
timeout -k 10 300 python bench.py --config c4 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_bench_c4.json 2> gpurun_out/${TAG}_bench_c4.err
echo EXIT $?
