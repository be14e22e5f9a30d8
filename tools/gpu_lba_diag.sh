set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in 1 2; do
SPSLAM_GPU_LIB=sp-slam_amd/libspslam_gpu_lbad$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/lbad$v -o run -- python3 tools/lba_bench.py --reps 2 > gpurun_out/lbad$v.txt 2>&1 || exit 1
done
echo EXIT 0
