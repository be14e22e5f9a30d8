set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd ${GRAFT_REPO_ROOT:-.}
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_sequence.py > gpurun_out/refkf_tests.log 2>&1 || exit 1
timeout -k 10 200 env GPU_MAX_HW_QUEUES=8 python tools/b1_prof.py --frames 300 --lookahead 2 --max-inflight 1 > gpurun_out/refkf_b1.txt 2>&1
