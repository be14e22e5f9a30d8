# SQ counters of the LBA phase kernels (tools/lba_bench.py alone), one pass of <= 8 SQ counters, kernel trace
# only beside them.   bash tools/pmc_lba.sh TAG
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
TAG=${1:-pmclba}
timeout -s KILL 180 rocprofv3 --pmc ${PMC:-SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_VMEM} --kernel-include-regex "lba::" --kernel-trace --output-format csv -d gpurun_out/${TAG}_p1 -o run -- python3 tools/lba_bench.py --reps 2 > gpurun_out/${TAG}_p1.log 2>&1
