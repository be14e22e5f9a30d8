set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_sequence.py -k "pipelined_equals or lookahead" tests/test_gpu_lba.py -k "pipelined_equals or lookahead or two_streams" > gpurun_out/b1_tests.log 2>&1 &&
for L in 1 2 3; do timeout -k 10 200 env GPU_MAX_HW_QUEUES=8 python -u tools/b1_prof.py --frames 200 --lookahead $L >> gpurun_out/b1_look.txt 2>&1 || exit 1; done
