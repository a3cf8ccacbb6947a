#!/bin/bash
# round 3 session m: user-side rhs / row sums on the MFMA: Gram and parity
# tests, fixed-count A/B (option on / off) at k = 64 and 128, bench.
set -o pipefail
OUT=gpurun_out/r03m; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -m gpu -v --timeout 400 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $OUT/tests.log | tail -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "TESTS rc=$rc: stop"; exit $rc; fi
ab() { timeout -k 10 300 python -u tools/cg_ab.py "$@" >> $OUT/cg_ab.jsonl 2>> $OUT/cg_ab.err; }
for k in 64 128; do
  ab --k $k --m 5 --tag rhs-mfma || exit $?
  ab --k $k --m 5 --opt gram_rhs_mfma=0 --tag rhs-valu || exit $?
  ab --k $k --m 5 --tag rhs-mfma-2 || exit $?
done
cut -c1-420 $OUT/cg_ab.jsonl
timeout -k 10 300 python -u bench.py --no-cpu > $OUT/bench.json 2> $OUT/bench.err; rc=$?
cut -c1-400 $OUT/bench.json; exit $rc
