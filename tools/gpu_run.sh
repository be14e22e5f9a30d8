#!/bin/bash
# One GPU-box call, parameterised (replaces the round-1/2 one-shot lease scripts):
#   gpurun -- 'bash tools/gpu_run.sh TAG STEP [STEP ...]'
# Steps run in order, each under its own time limit; the first failing step ends the call.
#   tests                 pytest -m gpu over tests/ (verbose, thread timeout per test)
#   tests:F1,F2           pytest over the given test files only
#   testsk:F1,F2:EXPR     pytest over the files with -k EXPR (_ for spaces); failing tests do not end the call
#   smoke                 __graft_entry__.smoke()
#   bench:CFG[:EXTRA]     python bench.py --config CFG --steps 20 --warmup 3 EXTRA (EXTRA: '_' for spaces)
#   prof:CFG              rocprofv3 --kernel-trace --stats over a short bench of CFG (no CPU baseline / ATE)
#   pmc:CFG               tools/pmc_round.sh CFG (HBM FETCH/WRITE passes, provenance = git HEAD)
#   py:SCRIPT[:ARGS]      python SCRIPT ARGS (ARGS: '_' for spaces)
# Outputs: gpurun_out/TAG_*.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
TAG=$1
shift
mkdir -p gpurun_out
for step in "$@"; do
    kind=${step%%:*}
    arg=${step#*:}
    [ "$arg" = "$step" ] && arg=""
    echo "== $step $(date +%T)"
    case $kind in
        tests)
            files=tests
            [ -n "$arg" ] && files=$(echo "$arg" | tr ',' ' ')
            timeout -k 10 900 python -u -m pytest $files -m gpu -x -v --timeout 300 --timeout-method thread \
                > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
            tail -3 gpurun_out/${TAG}_tests.log ;;
        testsk)  # testsk:F1,F2:EXPR -- the given files, -k EXPR ('_' for spaces), no -x
            files=$(echo "${arg%%:*}" | tr ',' ' ')
            expr=$(echo "${arg#*:}" | tr '_' ' ')
            timeout -k 10 900 python -u -m pytest $files -m gpu -v --timeout 300 --timeout-method thread -k "$expr" \
                > gpurun_out/${TAG}_testsk.log 2>&1
            rc=$?
            tail -3 gpurun_out/${TAG}_testsk.log
            [ $rc -le 1 ] || exit 1 ;;  # test failures go on; a time limit, crash or usage error ends the call
        smoke)
            timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 \
                || { tail -30 gpurun_out/${TAG}_smoke.log; exit 1; }
            tail -3 gpurun_out/${TAG}_smoke.log ;;
        bench)
            cfg=${arg%%:*}; extra=""
            [ "$cfg" != "$arg" ] && extra=$(echo "${arg#*:}" | tr '_' ' ')
            timeout -k 10 600 python bench.py --config $cfg --steps 20 --warmup 3 $extra \
                > gpurun_out/${TAG}_bench_${cfg}.json 2> gpurun_out/${TAG}_bench_${cfg}.err \
                || { tail -30 gpurun_out/${TAG}_bench_${cfg}.err; exit 1; }
            cut -c1-400 gpurun_out/${TAG}_bench_${cfg}.json ;;
        prof)
            timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof_${arg} -o run -- \
                python3 bench.py --config $arg --steps 10 --warmup 2 --no-cpu-baseline --ate-frames 0 \
                > gpurun_out/${TAG}_prof_${arg}.json 2> gpurun_out/${TAG}_prof_${arg}.err \
                || { tail -30 gpurun_out/${TAG}_prof_${arg}.err; exit 1; } ;;
        pmc)
            timeout -k 10 600 bash tools/pmc_round.sh $arg ${TAG} > gpurun_out/${TAG}_pmc_${arg}.log 2>&1 \
                || { tail -30 gpurun_out/${TAG}_pmc_${arg}.log; exit 1; } ;;
        py)
            scr=${arg%%:*}; extra=""
            [ "$scr" != "$arg" ] && extra=$(echo "${arg#*:}" | tr '_' ' ')
            timeout -k 10 900 python -u $scr $extra > gpurun_out/${TAG}_$(basename $scr .py).log 2>&1 \
                || { tail -30 gpurun_out/${TAG}_$(basename $scr .py).log; exit 1; }
            tail -5 gpurun_out/${TAG}_$(basename $scr .py).log ;;
        *) echo "unknown step $step"; exit 2 ;;
    esac
done
echo "== done $(date +%T)"
