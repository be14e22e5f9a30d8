# One GPU call at the end of a work block: every GPU test + the benches (tools/gpu_r02_full.sh), then the two
# PMC passes of the C2 bench with their summary, then a rocprof kernel trace of the pipelined C2 bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-final}
TAG=$TAG bash tools/gpu_r02_full.sh | grep -q "EXIT 0" && \
bash tools/pmc_round.sh c2 | grep -q "EXIT 0" && \
SPSLAM_PMC_CMD="tools/gpu_r02_final.sh (tools/pmc_round.sh c2 + tools/pmc_summary.py)" python tools/pmc_summary.py gpurun_out/pmc_fetch_c2 gpurun_out/pmc_write_c2 gpurun_out/pmc_c2_b256.json > gpurun_out/${TAG}_pmc_summary.txt 2>&1 && \
bash tools/gpu_prof.sh ${TAG} | grep -q "EXIT 0"
echo EXIT $?
