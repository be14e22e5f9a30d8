set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
bash tools/gpu_run.sh r6n tests:tests/test_gpu_planes.py,tests/test_gpu_supposed.py,tests/test_gpu_sequence.py,tests/test_gpu_pipeline.py || exit 1
bash tools/ab_b1_env.sh r6n 2 "SPSLAM_SEG_ROW_SCAN=0" "SPSLAM_SEG_ROW_SCAN=1" > gpurun_out/r6n_ab_b1.txt 2>&1 || exit 1
SPSLAM_LBG_ROWS_MAX_TEAM=16 timeout -k 10 300 python tools/lba_single.py > gpurun_out/r6n_lba_single_rows16.log 2>&1 || exit 1
SPSLAM_LBG_ROWS_MAX_TEAM=16 timeout -k 10 300 python tools/lba_bench.py --config c3s --team 5 8 --reps 2 > gpurun_out/r6n_lba_bench_rows16.txt 2>&1 || exit 1
SPSLAM_GPU_LIB=sp-slam_amd/libspslam_gpu_diagbuild.so timeout -k 10 300 python tools/lba_bench.py --config c3 --team 1 --reps 2 > gpurun_out/r6n_diagbuild.txt 2>&1 || exit 1
echo done
