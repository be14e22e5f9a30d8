# One GPU call: pipeline / sequence / supposed parity with the supposed-plane stage moved to the tracking stream,
# then an interleaved A/B against the previous layout (new = SPSLAM_SUPP_ON_TAIL=1).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8
timeout -k 10 500 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_sequence.py tests/test_gpu_supposed.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/split_tests.log 2>&1 || exit 1
for rep in 1 2 3; do
  for v in new old; do
    if [ $v = old ]; then
      timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --ate-frames 0 > gpurun_out/split_${v}_$rep.json 2> gpurun_out/split_${v}_$rep.err || exit 1
    else
      SPSLAM_SUPP_ON_TAIL=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --ate-frames 0 > gpurun_out/split_${v}_$rep.json 2> gpurun_out/split_${v}_$rep.err || exit 1
    fi
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], round(d['value']), round(d['ms_per_step'],3))" gpurun_out/split_${v}_$rep.json $v $rep
  done
done
echo EXIT 0
