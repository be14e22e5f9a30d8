set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd ${GRAFT_REPO_ROOT:-.}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/r5_gpu_tests2.log 2>&1 || exit 1
timeout -k 10 600 python bench.py --config c3 --no-cpu-baseline --single-sequence-frames 0 > gpurun_out/r5i_bench_c3.json 2> gpurun_out/r5i_bench_c3.err
