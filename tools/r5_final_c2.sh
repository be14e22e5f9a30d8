# final C2 evidence at the committed library: PMC passes, the bench line (reading that PMC file), kernel stats
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd ${GRAFT_REPO_ROOT:-.}
TAG=${1:-r5f}
bash tools/pmc_round.sh c2 $TAG || exit 1
cp gpurun_out/${TAG}_pmc_c2.json profiles/pmc_c2_b256.json
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench_c2.json 2> gpurun_out/${TAG}_bench_c2.err || exit 1
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-.}
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof_c2 -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --ate-frames 0 --closed-loop-steps 0 --single-sequence-frames 0 > gpurun_out/${TAG}_prof_c2.log 2>&1
