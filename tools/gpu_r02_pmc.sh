# One GPU call: the local-mapping-beside-tracking test, then the two PMC passes for c2 and their summary.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
    "tests/test_gpu_pipeline.py::test_c3_local_mapping_beside_tracking" > gpurun_out/c3_lm_test.log 2>&1 && \
bash tools/pmc_round.sh c2 && \
SPSLAM_PMC_CMD="tools/gpu_r02_pmc.sh" python tools/pmc_summary.py gpurun_out/pmc_fetch_c2 gpurun_out/pmc_write_c2 gpurun_out/pmc_c2_b256.json
echo EXIT $?
