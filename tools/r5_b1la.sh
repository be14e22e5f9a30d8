set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd ${GRAFT_REPO_ROOT:-.}
for r in 1 2; do
  for L in 2 3 4; do
    timeout -k 10 200 python tools/b1_prof.py --frames 300 --lookahead $L --max-inflight 1 > gpurun_out/la_${L}_$r.txt 2>&1 || exit 1
  done
  timeout -k 10 200 python tools/b1_prof.py --frames 300 --lookahead 3 --max-inflight 2 > gpurun_out/la_3i2_$r.txt 2>&1 || exit 1
done
