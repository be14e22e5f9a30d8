# final evidence at the committed library: C2 (PMC passes, the full bench line, kernel stats) and the C3 line
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd ${GRAFT_REPO_ROOT:-.}
TAG=${1:-r5k}
bash tools/r5_final_c2.sh $TAG || exit 1
timeout -k 10 500 python bench.py --config c3 --no-cpu-baseline --single-sequence-frames 0 > gpurun_out/${TAG}_bench_c3.json 2> gpurun_out/${TAG}_bench_c3.err
