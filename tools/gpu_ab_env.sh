# Same-box A/B of an environment knob on the C2 bench:  VAR=NAME VALUES="a b c" TAG=t bash tools/gpu_ab_env.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8
TAG=${TAG:-ab}
CFG=${CFG:-c2}
for v in $VALUES; do
  env $VAR=$v timeout -k 10 300 python bench.py --config $CFG --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_${v}.json 2> gpurun_out/${TAG}_${v}.err || exit $?
done
echo EXIT 0
