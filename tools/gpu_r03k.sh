#!/bin/bash
# round 3 session k: score-kernel probe, tests of the changed paths (one-pass
# per side, opaque tiles, CSR exclusions), fixed-count A/B and bench.
set -o pipefail
OUT=gpurun_out/r03k; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 ./tools/probes/score_probe2 > $OUT/score_probe2.txt 2>&1; rc=$?; cat $OUT/score_probe2.txt
if [ $rc -ne 0 ]; then echo "probe rc=$rc: stop"; exit $rc; fi
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_serving.py tests/test_distributed.py -m gpu -v --timeout 400 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $OUT/tests.log | tail -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "TESTS rc=$rc: stop"; exit $rc; fi
ab() { timeout -k 10 300 python -u tools/cg_ab.py "$@" >> $OUT/cg_ab.jsonl 2>> $OUT/cg_ab.err; }
ab --k 64 --tag default || exit $?
ab --k 128 --tag default || exit $?
cut -c1-500 $OUT/cg_ab.jsonl
timeout -k 10 300 python -u bench_serving.py --what topn --no-cpu > $OUT/bench_topn.json 2> $OUT/bench_topn.err || exit $?
cut -c1-900 $OUT/bench_topn.json
timeout -k 10 300 python -u bench.py --no-cpu > $OUT/bench.json 2> $OUT/bench.err; rc=$?
cut -c1-400 $OUT/bench.json; exit $rc
