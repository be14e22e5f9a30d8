# Interleaved A/B/C of library variants on the pipelined C2 step: bash tools/ab_libs3.sh TAG LIB_B LIB_C
cd ${GRAFT_REPO_ROOT:-.}
TAG=$1; LIBB=$2; LIBC=$3
B="python bench.py --config c2 --steps 40 --warmup 5 --no-cpu-baseline --ate-frames 0 --closed-loop-steps 0"
for r in 1 2 3; do
  timeout -k 10 300 $B > gpurun_out/ab_${TAG}_a_$r.json 2>/dev/null || exit 1
  SPSLAM_GPU_LIB=$LIBB timeout -k 10 300 $B > gpurun_out/ab_${TAG}_b_$r.json 2>/dev/null || exit 1
  SPSLAM_GPU_LIB=$LIBC timeout -k 10 300 $B > gpurun_out/ab_${TAG}_c_$r.json 2>/dev/null || exit 1
done
for f in gpurun_out/ab_${TAG}_*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', round(d['ms_per_step'],3), round(d['kernels_ms_per_step']['pose_kernel'],3))"; done
