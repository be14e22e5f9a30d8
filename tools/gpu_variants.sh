# One GPU call: the C2 bench under several stream-priority variants (no CPU baseline), one JSON per variant.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-var}
i=0
for v in "$@"; do
  timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline $v > gpurun_out/${TAG}_$i.json 2> gpurun_out/${TAG}_$i.err || exit $?
  i=$((i+1))
done
echo EXIT 0
