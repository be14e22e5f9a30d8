set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd ${GRAFT_REPO_ROOT:-.}
SPSLAM_GPU_LIB=sp-slam_amd/libspslam_gpu_prof.so timeout -k 10 200 python tools/pose_phases.py --batch 1 > gpurun_out/pose_phases_b1.txt 2>&1 || exit 1
SPSLAM_GPU_LIB=sp-slam_amd/libspslam_gpu_prof.so timeout -k 10 200 python tools/pose_phases.py --batch 256 > gpurun_out/pose_phases_b256.txt 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sequence.py -k "pipelined_equals or lookahead or frame1" > gpurun_out/pp_tests.log 2>&1 || exit 1
timeout -k 10 200 python tools/b1_prof.py --frames 200 --serial > gpurun_out/pp_b1_serial.txt 2>&1
