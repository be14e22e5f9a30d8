set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT:-.}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/b1n_pipe -o run -- python3 tools/b1_prof.py --frames 150 --lookahead 2 --max-inflight 1 > gpurun_out/b1n_pipe.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/b1n_ser -o run -- python3 tools/b1_prof.py --frames 100 --serial > gpurun_out/b1n_ser.log 2>&1
