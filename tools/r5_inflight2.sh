set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd ${GRAFT_REPO_ROOT:-.}
for q in 8 16; do
  for la in 1 2 3 4; do
    for m in 0 1; do
      SPSLAM_MAX_INFLIGHT=$m timeout -k 10 200 env GPU_MAX_HW_QUEUES=$q python tools/b1_prof.py --frames 300 --lookahead $la 2>/dev/null | sed "s/^/hwq=$q inflight=$m /" >> gpurun_out/inflight2_b1.txt || exit 1
    done
  done
done
