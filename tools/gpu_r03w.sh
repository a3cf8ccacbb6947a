#!/bin/bash
# round 3 session w: CSR-stream SpMV (general CG) -- parity + A/B of variants
set -o pipefail
OUT=gpurun_out/r03w; mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@"
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$name rc=$rc: stop"; exit $rc; fi
}
step test 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_cgls.py > $OUT/test.log 2>&1
tail -2 $OUT/test.log
for v in ${VARIANTS:-new}; do
  if [ $v = new ]; then unset MR_LIB_PATH; else export MR_LIB_PATH=$PWD/var_libs/$v/cpp_ls_lib.so; fi
  step cg_$v 300 python -u bench_cg.py --no-cpu > $OUT/bench_cg_$v.json 2> $OUT/bench_cg_$v.err
  python3 -c "
import json; d=json.load(open('$OUT/bench_cg_$v.json')); k=d['kernels']
print('$v', d['value'], d['iterations'], {c: v['avg_us'] for c, v in k.items()})"
done
unset MR_LIB_PATH
echo DONE
