set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd ${GRAFT_REPO_ROOT:-.}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sequence.py > gpurun_out/lmh2_tests.log 2>&1 || exit 1
timeout -k 10 500 python bench.py --config c3 --no-cpu-baseline --single-sequence-frames 0 > gpurun_out/lmh2_bench_c3.json 2> gpurun_out/lmh2_bench_c3.err || exit 1
GPU_MAX_HW_QUEUES=16 timeout -k 10 400 python -m cProfile -o gpurun_out/c3cl2.prof bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline --single-sequence-frames 0 --ate-frames 0 > gpurun_out/c3cl2.json 2> gpurun_out/c3cl2.err
