# One GPU call: C2 bench variants (pipelined with / without tracking priority, serial), 8 HW queues via bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-pipe}
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_c2.json 2> gpurun_out/${TAG}_c2.err && \
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-tail-priority > gpurun_out/${TAG}_c2_noprio.json 2> gpurun_out/${TAG}_c2_noprio.err && \
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pipeline > gpurun_out/${TAG}_c2_serial.json 2> gpurun_out/${TAG}_c2_serial.err && \
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --config c3 > gpurun_out/${TAG}_c3.json 2> gpurun_out/${TAG}_c3.err
echo EXIT $?
