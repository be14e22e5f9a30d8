set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd ${GRAFT_REPO_ROOT:-.}
timeout -k 10 900 python bench.py --config c3 --no-cpu-baseline --single-sequence-frames 0 > gpurun_out/r5g_bench_c3.json 2> gpurun_out/r5g_bench_c3.err || exit 1
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-.}
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5g_b1 -o run -- python3 tools/b1_prof.py --frames 120 --lookahead 2 --max-inflight 1 > gpurun_out/r5g_b1.log 2>&1
