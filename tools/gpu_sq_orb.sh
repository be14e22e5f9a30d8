# One GPU call: SQ counters of the ORB kernels alone (tools/orb_bench.py), two passes.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_INST_ANY --kernel-trace --output-format csv -d gpurun_out/sq1 -o run -- python3 tools/orb_bench.py > gpurun_out/sq1.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY --kernel-trace --output-format csv -d gpurun_out/sq2 -o run -- python3 tools/orb_bench.py > gpurun_out/sq2.log 2>&1
echo EXIT $?
