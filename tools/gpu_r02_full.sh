# One GPU call: every GPU test, the default bench (driver command) with its wall time, then C3 / C4 / C5.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-full}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1 && \
S=$SECONDS && timeout -k 10 600 python bench.py > gpurun_out/${TAG}_c2.json 2> gpurun_out/${TAG}_c2.err && echo "c2 wall $((SECONDS - S)) s" > gpurun_out/${TAG}_c2_wall.txt && \
timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 3 --ate-frames 0 --no-cpu-baseline > gpurun_out/${TAG}_c3.json 2> gpurun_out/${TAG}_c3.err && \
timeout -k 10 300 python bench.py --config c4 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_c4.json 2> gpurun_out/${TAG}_c4.err && \
timeout -k 10 300 python bench.py --config c5 --batch 64 --steps 10 --warmup 3 --ate-frames 0 --no-cpu-baseline > gpurun_out/${TAG}_c5.json 2> gpurun_out/${TAG}_c5.err
echo EXIT $?
