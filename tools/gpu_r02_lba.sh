# One GPU call: LBA parity incl. the stop-flag tests, and the C3 pipeline test.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread -m gpu tests/test_gpu_lba.py \
    "tests/test_gpu_pipeline.py::test_c3_local_mapping_beside_tracking" > gpurun_out/lba_tests.log 2>&1
echo EXIT $?
