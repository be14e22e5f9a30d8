# One GPU call: plane parity tests, segmentation phase stamps (C2, C5), then an interleaved C2 A/B of the
# library variants given.
#   TAG=<name> bash tools/gpu_seg_ab.sh <lib.so>...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-seg}
timeout -k 10 400 python -u -m pytest tests/test_gpu_planes.py tests/test_gpu_supposed.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 && \
timeout -k 10 200 python tools/seg_phases.py --config c2 > gpurun_out/${TAG}_seg_c2.txt 2>&1 && \
timeout -k 10 200 python tools/seg_phases.py --config c5 --batch 64 > gpurun_out/${TAG}_seg_c5.txt 2>&1 && \
TAG=${TAG} bash tools/gpu_ab.sh "$@"
