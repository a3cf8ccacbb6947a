#!/bin/bash
# round 3 session n: the full GPU suite and smoke on the current build, the
# profile set again (bench with CPU baseline, rocprof stats, PMC traffic),
# C1 (ML-100K shape, k = 10) on the GPU and the general-CG bench.
set -o pipefail
OUT=gpurun_out/r03n; mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@"
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$name rc=$rc: stop"; exit $rc; fi
}
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $OUT/gpu_tests.log | tail -10
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "TESTS rc=$rc: stop"; exit $rc; fi
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
tail -3 $OUT/smoke.log
step bench 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
cut -c1-300 $OUT/bench.json
step trace 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --no-cpu --steps 20 --warmup 5 > $OUT/bench_under_rocprof.json 2> $OUT/trace.err
step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/pmc_fetch -o run --output-format csv -- python3 bench.py --no-cpu --no-kernel-events --steps 3 --warmup 1 > /dev/null 2> $OUT/pmc_fetch.err
step pmc_write 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/pmc_write -o run --output-format csv -- python3 bench.py --no-cpu --no-kernel-events --steps 3 --warmup 1 > /dev/null 2> $OUT/pmc_write.err
step c1 300 python -u bench.py --shape ml-100k --k 10 --steps 50 > $OUT/bench_c1.json 2> $OUT/bench_c1.err
cut -c1-300 $OUT/bench_c1.json
step k128 600 python -u bench.py --no-cpu --k 128 --steps 20 --warmup 3 > $OUT/bench_k128.json 2> $OUT/bench_k128.err
step bench_cg 600 python -u bench_cg.py --no-cpu > $OUT/bench_cg.json 2> $OUT/bench_cg.err
echo DONE
