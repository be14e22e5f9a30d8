set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd ${GRAFT_REPO_ROOT:-.}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_lba.py tests/test_gpu_lba_large.py > gpurun_out/lba1_tests.log 2>&1 || exit 1
timeout -k 10 200 python tools/lba_bench.py --team 1 5 --reps 2 > gpurun_out/lba1_bench.txt 2>&1 || exit 1
SPSLAM_GPU_LIB=sp-slam_amd/libspslam_gpu_dbuild.so timeout -k 10 200 python tools/lba_bench.py --team 1 --reps 1 >> gpurun_out/lba1_bench.txt 2>&1
