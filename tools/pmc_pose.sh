# SQ counters of the PoseOptimization kernel alone (tools/pose_phases.py --no-prof), two passes of <= 8 SQ
# counters, kernel trace only beside them.   bash tools/pmc_pose.sh TAG
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8
TAG=${1:-pmcpose}
timeout -s KILL 120 rocprofv3 -L > gpurun_out/${TAG}_avail.txt 2>&1
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-trace --output-format csv -d gpurun_out/${TAG}_p1 -o run -- python3 tools/pose_phases.py --no-prof > gpurun_out/${TAG}_p1.log 2>&1 && \
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS --kernel-trace --output-format csv -d gpurun_out/${TAG}_p2 -o run -- python3 tools/pose_phases.py --no-prof > gpurun_out/${TAG}_p2.log 2>&1
