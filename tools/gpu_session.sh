#!/bin/bash
# One GPU-box session, parametrised (replaces round 3's one-off tools/gpu_r03*.sh).
#
#   bash tools/gpu_session.sh TAG STEP [STEP ...]
#
# Steps run in order, outputs under gpurun_out/TAG/, each under its own time
# limit.  A test failure (pytest rc 1) is reported and the session goes on;
# any other non-zero status (fault, abort, time limit) ends the session there.
#   smoke               __graft_entry__.smoke()
#   tests[=EXPR]        pytest -m gpu (-k EXPR; "all" or empty: everything)
#   bench[=ARGS]        python bench.py ARGS       -> bench_<i>.json
#   ab=ARGS             python tools/cg_ab.py ARGS -> ab_<i>.jsonl (fixed CG counts)
#   stats=ARGS          rocprofv3 --kernel-trace --stats over bench.py ARGS
#   pmc=CTRS@ARGS       rocprofv3 --pmc CTRS (space-separated) over bench.py ARGS
#   ktrace=SCRIPT ARGS  rocprofv3 --kernel-trace over python SCRIPT ARGS (tools/trace_gaps.py)
#   py=SCRIPT ARGS      python SCRIPT ARGS         -> py_<i>.log
#   setenv=VAR=VALUE    export VAR for the following steps (e.g. MR_LIB_PATH=...)
#   unsetenv=VAR        unset it
# ARGS are split on spaces.  MR_LIB_PATH in the environment selects a variant
# library (movie_recommender_amd/_lib.py).
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
i=0
stop() { echo "[$TAG] step $i ($1) rc=$2: stop"; exit $2; }
for step in "$@"; do
  i=$((i + 1))
  name=${step%%=*}
  arg=""
  [ "$name" != "$step" ] && arg=${step#*=}
  echo "[$TAG] step $i: $step"
  case $name in
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
      rc=$?; tail -3 $OUT/smoke.log; [ $rc -ne 0 ] && stop smoke $rc ;;
    tests)
      K=()
      [ -n "$arg" ] && [ "$arg" != all ] && K=(-k "$arg")
      timeout -k 10 1500 python -u -m pytest tests -m gpu -v --timeout 300 \
        --timeout-method thread "${K[@]}" > $OUT/tests_$i.log 2>&1
      rc=$?
      grep -E "FAILED|ERROR" $OUT/tests_$i.log | head -40; tail -2 $OUT/tests_$i.log
      [ $rc -ne 0 ] && [ $rc -ne 1 ] && stop tests $rc ;;
    bench)
      timeout -k 10 900 python -u bench.py $arg > $OUT/bench_$i.json 2> $OUT/bench_$i.err
      rc=$?; tail -c 1500 $OUT/bench_$i.json; tail -2 $OUT/bench_$i.err
      [ $rc -ne 0 ] && stop bench $rc ;;
    ab)
      timeout -k 10 600 python -u tools/cg_ab.py $arg >> $OUT/ab_$i.jsonl 2> $OUT/ab_$i.err
      rc=$?; tail -c 800 $OUT/ab_$i.jsonl; [ $rc -ne 0 ] && stop ab $rc ;;
    stats)
      timeout -k 10 900 rocprofv3 --kernel-trace --stats -f csv rocpd -d $OUT/stats_$i -o run -- \
        python3 bench.py $arg > $OUT/stats_$i.json 2> $OUT/stats_$i.err
      rc=$?; find $OUT/stats_$i -name "*kernel_stats.csv" | head -3
      [ $rc -ne 0 ] && stop stats $rc ;;
    ktrace)
      timeout -k 10 600 rocprofv3 --kernel-trace -d $OUT/ktrace_$i -o run -- \
        python3 $arg > $OUT/ktrace_$i.log 2>&1
      rc=$?; tail -3 $OUT/ktrace_$i.log; [ $rc -ne 0 ] && stop ktrace $rc ;;
    pmc)
      ctrs=${arg%%@*}; bargs=${arg#*@}
      timeout -s KILL 300 rocprofv3 --pmc $ctrs -f csv -d $OUT/pmc_$i -o run -- \
        python3 bench.py $bargs > $OUT/pmc_$i.json 2> $OUT/pmc_$i.err
      rc=$?; [ $rc -ne 0 ] && stop pmc $rc ;;
    py)
      timeout -k 10 900 python -u $arg > $OUT/py_$i.log 2>&1
      rc=$?; tail -5 $OUT/py_$i.log; [ $rc -ne 0 ] && stop py $rc ;;
    setenv) export "$arg" ;;
    unsetenv) unset "$arg" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "[$TAG] DONE"
