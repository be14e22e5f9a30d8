set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd ${GRAFT_REPO_ROOT:-.}
for r in 1 2 3; do
  for o in "" "--no-refkf"; do
    timeout -k 10 200 env GPU_MAX_HW_QUEUES=8 python tools/b1_prof.py --frames 300 --lookahead 2 --max-inflight 1 $o 2>/dev/null >> gpurun_out/b1ab.txt || exit 1
  done
done
timeout -k 10 200 python tools/b1_prof.py --frames 200 --serial 2>/dev/null >> gpurun_out/b1ab.txt
