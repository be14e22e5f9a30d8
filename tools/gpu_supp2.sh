# One GPU call: supposed-plane / pipeline parity tests, supp_lines phase clocks, then a C2 A/B of the libraries given.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-supp}
timeout -k 10 400 python -u -m pytest tests/test_gpu_supposed.py tests/test_gpu_pipeline.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 && \
SPSLAM_GPU_LIB=sp-slam_amd/libspslam_gpu_suppprof.so timeout -k 10 200 python tools/supp_phases.py > gpurun_out/${TAG}_phases.txt 2>&1 && \
TAG=${TAG} bash tools/gpu_ab.sh "$@"
