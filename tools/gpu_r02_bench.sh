# One GPU call: the default bench (driver command) with its wall time, then C3 and C5.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-bench}
S=$SECONDS; timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_c2.json 2> gpurun_out/${TAG}_c2.err && echo "c2 wall $((SECONDS - S)) s" && \
timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 3 --ate-frames 0 --no-cpu-baseline > gpurun_out/${TAG}_c3.json 2> gpurun_out/${TAG}_c3.err && \
timeout -k 10 300 python bench.py --config c5 --batch 64 --steps 10 --warmup 3 --ate-frames 0 --no-cpu-baseline > gpurun_out/${TAG}_c5.json 2> gpurun_out/${TAG}_c5.err
echo EXIT $?
