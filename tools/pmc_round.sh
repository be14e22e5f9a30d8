# HBM traffic per kernel (MI355X_MICROARCH.md "HBM"): FETCH_SIZE and WRITE_SIZE in separate passes,
# kernel trace only beside the counters.  Results under gpurun_out/pmc_*/.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
# bench.py itself is the profiled process (no re-run child for the hardware-queue count)
export GPU_MAX_HW_QUEUES=8
CFG=${1:-c2}
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch_${CFG} -o run -- python3 bench.py --config ${CFG} --steps 3 --warmup 1 --no-cpu-baseline --ate-frames 0 > gpurun_out/pmc_fetch_${CFG}.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write_${CFG} -o run -- python3 bench.py --config ${CFG} --steps 3 --warmup 1 --no-cpu-baseline --ate-frames 0 > gpurun_out/pmc_write_${CFG}.log 2>&1
echo EXIT $?
