set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd ${GRAFT_REPO_ROOT:-.}
timeout -k 10 500 python bench.py --config c4 --no-cpu-baseline --single-sequence-frames 0 --closed-loop-steps 0 > gpurun_out/${TAG:-r5j}_bench_c4.json 2> gpurun_out/${TAG:-r5j}_bench_c4.err || exit 1
timeout -k 10 500 python bench.py --config c5 --no-cpu-baseline --single-sequence-frames 0 --closed-loop-steps 0 --ate-frames 0 > gpurun_out/${TAG:-r5j}_bench_c5.json 2> gpurun_out/${TAG:-r5j}_bench_c5.err
