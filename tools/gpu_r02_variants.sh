# One GPU call: the C2 bench (no ATE) for each library variant given, SPSLAM_GPU_LIB per run.
#   TAG=<name> bash tools/gpu_r02_variants.sh <lib.so>...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8
TAG=${TAG:-vars}
for lib in "$@"; do
  v=$(basename $lib .so)
  SPSLAM_GPU_LIB=$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --ate-frames 0 > gpurun_out/${TAG}_${v}.json 2> gpurun_out/${TAG}_${v}.err || exit 1
done
echo EXIT 0
