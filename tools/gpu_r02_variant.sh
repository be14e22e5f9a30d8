# One GPU call: a library variant (SPSLAM_GPU_LIB=$LIB) -- selected tests, the C2 bench and stages alone.
#   TAG=<name> LIB=sp-slam_amd/libspslam_gpu_<v>.so bash tools/gpu_r02_variant.sh <pytest selection...>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8
export SPSLAM_GPU_LIB=$LIB
TAG=${TAG:-var}
timeout -k 10 600 python -u -m pytest "$@" -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/${TAG}_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --ate-frames 0 > gpurun_out/${TAG}_bench_c2.json 2> gpurun_out/${TAG}_bench_c2.err && \
timeout -k 10 300 python tools/stage_bench.py > gpurun_out/${TAG}_stages.txt 2>&1
echo EXIT $?
