# One GPU call: supposed-plane parity tests, then an interleaved C2 A/B of the library variants given.
#   TAG=<name> bash tools/gpu_supp_ab.sh <lib.so>...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-supp}
timeout -k 10 400 python -u -m pytest tests/test_gpu_supposed.py tests/test_gpu_pipeline.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 && \
TAG=${TAG} bash tools/gpu_ab.sh "$@"
