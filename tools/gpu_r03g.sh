#!/bin/bash
# round 3 session g: C4/C5 + layout tests on the new build, one-pass A/B at a
# fixed CG iteration count (k = 64, 128), then the default bench.
set -o pipefail
OUT=gpurun_out/r03g; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_scale.py "tests/test_gpu_parity.py::test_full_size_context_build_exact" "tests/test_gpu_parity.py::test_headline_paths_golden" -m gpu -v --timeout 400 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $OUT/tests.log | tail -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "TESTS rc=$rc: stop"; exit $rc; fi
for k in 64 128; do
  for v in op3 op4; do
    MR_LIB_PATH=$PWD/var_libs/$v/cpp_ls_lib.so timeout -k 10 300 python -u tools/cg_ab.py --k $k --tag $v-onepass >> $OUT/cg_ab.jsonl 2>> $OUT/cg_ab.err || exit $?
  done
  MR_LIB_PATH=$PWD/var_libs/op3/cpp_ls_lib.so timeout -k 10 300 python -u tools/cg_ab.py --k $k --onepass 0 --tag twokernel >> $OUT/cg_ab.jsonl 2>> $OUT/cg_ab.err || exit $?
done
cat $OUT/cg_ab.jsonl
timeout -k 10 300 python -u bench.py --steps 30 --no-cpu > $OUT/bench.json 2> $OUT/bench.err; rc=$?
cat $OUT/bench.json; exit $rc
