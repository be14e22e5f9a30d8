# One GPU call: interleaved A/B of library variants on the C2 bench (no ATE, no CPU baseline), REPS rounds.
#   TAG=<name> REPS=2 bash tools/gpu_ab.sh <lib.so>...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8
TAG=${TAG:-ab}
CFG=${CFG:-c2}
for rep in $(seq 1 ${REPS:-2}); do
  for lib in "$@"; do
    v=$(basename $lib .so)
    SPSLAM_GPU_LIB=$lib timeout -k 10 300 python bench.py --config $CFG --steps 20 --warmup 5 --no-cpu-baseline --ate-frames 0 > gpurun_out/${TAG}_${v}_${rep}.json 2> gpurun_out/${TAG}_${v}_${rep}.err || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], round(d['value']), round(d['ms_per_step'],3))" gpurun_out/${TAG}_${v}_${rep}.json $v $rep
  done
done
echo EXIT 0
