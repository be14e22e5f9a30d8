# One GPU call: LBA parity, the C3 local-mapping test, the LBA wall time tool and the C3 bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8
TAG=${TAG:-lba2}
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_lba.py \
    "tests/test_gpu_pipeline.py::test_c3_local_mapping_beside_tracking" > gpurun_out/${TAG}_tests.log 2>&1 && \
timeout -k 10 120 python tools/lba_bench.py > gpurun_out/${TAG}_lba_bench.txt 2>&1 && \
timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 3 --ate-frames 0 --no-cpu-baseline > gpurun_out/${TAG}_bench_c3.json 2> gpurun_out/${TAG}_bench_c3.err
echo EXIT $?
