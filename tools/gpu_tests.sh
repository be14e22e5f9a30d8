# GPU call: selected test files (args), verbose, bounded.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-sel}
timeout -k 10 500 python -u -m pytest "$@" -x -v --timeout 400 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
echo EXIT $?
