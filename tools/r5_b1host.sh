set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd ${GRAFT_REPO_ROOT:-.}
timeout -k 10 200 python tools/b1_prof.py --frames 300 --lookahead 2 --max-inflight 1 > gpurun_out/b1h_plain.txt 2>&1 || exit 1
timeout -k 10 200 python tools/b1_prof.py --frames 300 --lookahead 2 --max-inflight 1 --cprofile gpurun_out/b1h_cprofile.txt > gpurun_out/b1h_prof.txt 2>&1 || exit 1
