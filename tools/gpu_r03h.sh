#!/bin/bash
# round 3 session h: C4 (direct r.r in the one-pass CG), the CG oracle tests,
# the matvec grid-size sweep (one-pass, k = 64) and the general-CG bench
# after the first-column row sort.
set -o pipefail
OUT=gpurun_out/r03h; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_scale.py "tests/test_gpu_parity.py::test_cg_iterations_vs_oracle" "tests/test_gpu_parity.py::test_headline_paths_golden" -m gpu -v --timeout 400 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $OUT/tests.log | tail -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "TESTS rc=$rc: stop"; exit $rc; fi
for parts in 768 1024 1536 2048; do
  MR_MV_PARTS=$parts timeout -k 10 300 python -u tools/cg_ab.py --k 64 --tag parts$parts >> $OUT/cg_ab.jsonl 2>> $OUT/cg_ab.err || exit $?
done
MR_MV_PARTS=2048 timeout -k 10 300 python -u tools/cg_ab.py --k 64 --onepass 0 --tag twokernel2048 >> $OUT/cg_ab.jsonl 2>> $OUT/cg_ab.err || exit $?
MR_MV_PARTS=1024 timeout -k 10 300 python -u tools/cg_ab.py --k 64 --onepass 0 --tag twokernel1024 >> $OUT/cg_ab.jsonl 2>> $OUT/cg_ab.err || exit $?
cat $OUT/cg_ab.jsonl | cut -c1-400
timeout -k 10 400 python -u bench_cg.py --no-cpu > $OUT/bench_cg.json 2> $OUT/bench_cg.err; rc=$?
cat $OUT/bench_cg.json | cut -c1-1500; exit $rc
