# One GPU call: ORB + e2e parity, ORB alone timing, C2 bench (pipelined and serial).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-orb}
timeout -k 10 400 python -u -m pytest tests/test_gpu_orb.py tests/test_gpu_pipeline.py tests/test_gpu_frame.py -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 && \
timeout -k 10 200 python tools/orb_bench.py 256 th > gpurun_out/${TAG}_orbb.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_c2.json 2> gpurun_out/${TAG}_c2.err && \
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pipeline > gpurun_out/${TAG}_c2_serial.json 2> gpurun_out/${TAG}_c2_serial.err
echo EXIT $?
