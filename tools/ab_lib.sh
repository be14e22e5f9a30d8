# Interleaved A/B of library variants on the pipelined C2 step: bash tools/ab_lib.sh TAG LIB_B [EXTRA_B]
# (A = the default library; 3 rounds; gpurun_out/ab_TAG_{a,b}_R.json)
cd ${GRAFT_REPO_ROOT:-.}
TAG=$1; LIBB=$2; EXTRA=$3
B="python bench.py --config c2 --steps 40 --warmup 5 --no-cpu-baseline --ate-frames 0 --closed-loop-steps 0"
for r in 1 2 3; do
  timeout -k 10 300 $B > gpurun_out/ab_${TAG}_a_$r.json 2>/dev/null || exit 1
  SPSLAM_GPU_LIB=$LIBB timeout -k 10 300 $B $EXTRA > gpurun_out/ab_${TAG}_b_$r.json 2>/dev/null || exit 1
done
for f in gpurun_out/ab_${TAG}_*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', round(d['ms_per_step'],3), round(d['kernels_ms_per_step']['pose_kernel'],3))"; done
