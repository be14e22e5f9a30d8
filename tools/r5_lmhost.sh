set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd ${GRAFT_REPO_ROOT:-.}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sequence.py tests/test_gpu_pipeline.py > gpurun_out/lmh_tests.log 2>&1 || exit 1
timeout -k 10 500 python bench.py --config c3 --no-cpu-baseline --single-sequence-frames 0 > gpurun_out/lmh_bench_c3.json 2> gpurun_out/lmh_bench_c3.err
