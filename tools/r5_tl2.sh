set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-.}
export GPU_MAX_HW_QUEUES=8
B="python3 bench.py --config c2 --steps 10 --warmup 3 --no-cpu-baseline --ate-frames 0 --closed-loop-steps 0 --single-sequence-frames 0"
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tl2 -o run -- $B > gpurun_out/tl2.log 2>&1
