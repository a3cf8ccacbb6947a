#!/bin/bash
# round 3 session i: full GPU suite on the peeled Gram loop + resident-grid
# one-pass CG, then the A/B (peel vs HEAD~ build; one-pass grid sweep) and
# the default bench.
set -o pipefail
OUT=gpurun_out/r03i; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $OUT/gpu_tests.log | tail -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "TESTS rc=$rc: stop"; exit $rc; fi
ab() { timeout -k 10 300 python -u tools/cg_ab.py "$@" >> $OUT/cg_ab.jsonl 2>> $OUT/cg_ab.err; }
ab --k 64 --tag peel-default || exit $?
MR_LIB_PATH=$PWD/var_libs/nopeel/cpp_ls_lib.so ab --k 64 --tag nopeel-2048 || exit $?
for parts in 512 640 896; do MR_MV_PARTS=$parts ab --k 64 --tag parts$parts || exit $?; done
ab --k 128 --tag peel-default || exit $?
MR_LIB_PATH=$PWD/var_libs/nopeel/cpp_ls_lib.so ab --k 128 --tag nopeel-2048 || exit $?
cut -c1-600 $OUT/cg_ab.jsonl
timeout -k 10 300 python -u bench.py --steps 30 --no-cpu > $OUT/bench.json 2> $OUT/bench.err; rc=$?
cut -c1-800 $OUT/bench.json; exit $rc
