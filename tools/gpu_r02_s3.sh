# One GPU call: C2 stages alone, rocprof kernel trace + stats of the pipelined C2 bench, C5 segmentation phases.
#   TAG=<name> bash tools/gpu_r02_s3.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8
TAG=${TAG:-s3}
timeout -k 10 300 python tools/stage_bench.py --config c2 > gpurun_out/${TAG}_stages_c2.txt 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --config c2 --steps 10 --warmup 2 --no-cpu-baseline --ate-frames 0 > gpurun_out/${TAG}_prof.json 2> gpurun_out/${TAG}_prof.err && \
timeout -k 10 200 python tools/seg_phases.py --config c5 --batch 64 > gpurun_out/${TAG}_seg_c5.txt 2>&1 && \
timeout -k 10 200 python tools/seg_phases.py --config c2 > gpurun_out/${TAG}_seg_c2.txt 2>&1 && \
timeout -k 10 200 python tools/stage_bench.py --config c5 --batch 64 > gpurun_out/${TAG}_stages_c5.txt 2>&1
echo EXIT $?
