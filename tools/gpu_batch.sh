# One GPU call: C2 bench at several batch sizes (pipelined).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-batch}
for B in 128 384 512; do
timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --batch $B > gpurun_out/${TAG}_c2_b$B.json 2> gpurun_out/${TAG}_c2_b$B.err || exit 1
done
echo EXIT $?
