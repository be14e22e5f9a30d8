# One GPU call: match parity with the prefetch variant, then an interleaved A/B of the C2 bench over library
# variants and the plane-stream priority knob (SPSLAM_PLANES_STREAM_PRIO).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8
SPSLAM_GPU_LIB=sp-slam_amd/libspslam_gpu_pf.so timeout -k 10 400 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_sequence.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab2_tests.log 2>&1 || exit 1
run() {  # tag lib streamprio rep
  SPSLAM_PLANES_STREAM_PRIO=$3 SPSLAM_GPU_LIB=$2 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --ate-frames 0 > gpurun_out/ab2_$1_$4.json 2> gpurun_out/ab2_$1_$4.err || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], round(d['value']), round(d['ms_per_step'],3))" gpurun_out/ab2_$1_$4.json $1 $4
}
for rep in 1 2 3; do
  run base sp-slam_amd/libspslam_gpu.so 0 $rep
  run pf sp-slam_amd/libspslam_gpu_pf.so 0 $rep
  run pfprio sp-slam_amd/libspslam_gpu_pfprio.so 0 $rep
  run pfstream sp-slam_amd/libspslam_gpu_pf.so 1 $rep
done
echo EXIT 0
