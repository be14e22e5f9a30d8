# HBM traffic per kernel (MI355X_MICROARCH.md "HBM"): FETCH_SIZE, WRITE_SIZE and the size-resolved read requests
# (TCC_EA0_RDREQ_{32B,64B,128B}: the read bytes without FETCH_SIZE's uncalibrated width factor) in separate passes,
# kernel trace only beside the counters.  Then tools/pmc_summary.py -> gpurun_out/TAG_pmc_CFG.json, whose
# provenance (git commit + sha256 of the profiled library) bench.py checks before reporting it as
# roofline.traffic (copy it to profiles/pmc_CFG_b256.json).
#   bash tools/pmc_round.sh CFG TAG
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
# bench.py itself is the profiled process (no re-run child for the hardware-queue count)
export GPU_MAX_HW_QUEUES=8
CFG=${1:-c2}
TAG=${2:-pmc}
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/${TAG}_pmc_fetch_${CFG} -o run -- python3 bench.py --config ${CFG} --steps 3 --warmup 1 --no-cpu-baseline --ate-frames 0 --closed-loop-steps 0 --single-sequence-frames 0 > gpurun_out/${TAG}_pmc_fetch_${CFG}.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/${TAG}_pmc_write_${CFG} -o run -- python3 bench.py --config ${CFG} --steps 3 --warmup 1 --no-cpu-baseline --ate-frames 0 --closed-loop-steps 0 --single-sequence-frames 0 > gpurun_out/${TAG}_pmc_write_${CFG}.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --kernel-trace --output-format csv -d gpurun_out/${TAG}_pmc_sized_${CFG} -o run -- python3 bench.py --config ${CFG} --steps 3 --warmup 1 --no-cpu-baseline --ate-frames 0 --closed-loop-steps 0 --single-sequence-frames 0 > gpurun_out/${TAG}_pmc_sized_${CFG}.log 2>&1 && \
python3 tools/pmc_summary.py gpurun_out/${TAG}_pmc_fetch_${CFG} gpurun_out/${TAG}_pmc_write_${CFG} gpurun_out/${TAG}_pmc_${CFG}.json gpurun_out/${TAG}_pmc_sized_${CFG}
