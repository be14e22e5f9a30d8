# level_kernel traffic per pyramid level and the FETCH_SIZE scale of 16 / 4 / 1-byte loads
# (tools/fetch_probe.hip, built beforehand: hipcc --offload-arch=gfx950 -O3 -o tools/fetch_probe.bin
# tools/fetch_probe.hip).  One counter per pass, kernel trace beside it only.
#   bash tools/pmc_levels.sh TAG
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
TAG=${1:-lv}
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/${TAG}_probe_fetch -o run -- ./tools/fetch_probe.bin > gpurun_out/${TAG}_probe.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/${TAG}_fetch -o run -- python3 tools/orb_bench.py 256 > gpurun_out/${TAG}_fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/${TAG}_write -o run -- python3 tools/orb_bench.py 256 > gpurun_out/${TAG}_write.log 2>&1 && \
python3 tools/pmc_levels.py gpurun_out/${TAG}_probe_fetch gpurun_out/${TAG}_fetch gpurun_out/${TAG}_write 256 gpurun_out/${TAG}_pmc_levels.json > gpurun_out/${TAG}_pmc_levels.txt 2>&1
