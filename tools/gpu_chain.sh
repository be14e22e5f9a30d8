# One GPU call: the benchmarked step's e2e parity + tracking-graph tests, then a C2 bench with CPU baseline + ATE.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-chain}
timeout -k 10 400 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_match.py tests/test_gpu_pose.py -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/${TAG}_c2.json 2> gpurun_out/${TAG}_c2.err
echo EXIT $?
