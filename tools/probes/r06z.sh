# General-CG SpMV: the CG output pass loading its rows' (r, p) pairs beside the gathers (MR_SP_PRELOAD,
# base) against loading them after the row sums (nopre); tests first
set -o pipefail
OUT=gpurun_out/r06z; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_cgls.py -m gpu > $OUT/tests.log 2>&1 || { echo "tests rc=$?"; tail -20 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for v in base nopre base nopre; do
  if [ $v = base ]; then unset MR_LIB_PATH; else export MR_LIB_PATH=$PWD/var_libs/$v/cpp_ls_lib.so; fi
  timeout -k 10 240 python -u bench_cg.py --no-cpu > $OUT/cg_$v.json 2> $OUT/cg_$v.err || { echo "bench_cg $v rc=$?"; tail -3 $OUT/cg_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/cg_$v.json')); print('$v', d['value'], d['iterations'], {k: (v['avg_us'], v['launches']) for k, v in d['kernels'].items()})"
done
