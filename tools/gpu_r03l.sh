#!/bin/bash
# round 3 session l: serving tests after the score-kernel layout change,
# top-N and factor-similarity benches.
set -o pipefail
OUT=gpurun_out/r03l; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_serving.py tests/test_gpu_factor_similar.py -m gpu -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $OUT/tests.log | tail -10
if [ $rc -ne 0 ]; then echo "TESTS rc=$rc: stop"; exit $rc; fi
timeout -k 10 300 python -u bench_serving.py --what topn,fsim > $OUT/bench_serving.json 2> $OUT/bench_serving.err; rc=$?
cut -c1-700 $OUT/bench_serving.json; exit $rc
