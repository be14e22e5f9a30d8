# One GPU call: pipeline parity with SPSLAM_ORB_AFTER_SUPP=1, then an interleaved A/B of the C2 bench with and without it.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8
SPSLAM_ORB_AFTER_SUPP=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_pipeline.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ow_tests.log 2>&1 || exit 1
for rep in 1 2 3; do
  for v in 0 1; do
    SPSLAM_ORB_AFTER_SUPP=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --ate-frames 0 > gpurun_out/ow_${v}_$rep.json 2> gpurun_out/ow_${v}_$rep.err || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('orb_after_supp', sys.argv[2], sys.argv[3], round(d['value']), round(d['ms_per_step'],3))" gpurun_out/ow_${v}_$rep.json $v $rep
  done
done
echo EXIT 0
