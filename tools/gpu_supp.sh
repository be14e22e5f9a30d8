cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_supposed.py tests/test_gpu_planes.py -x -v --timeout 300 --timeout-method thread > gpurun_out/supp_tests.log 2>&1
echo EXIT $?
