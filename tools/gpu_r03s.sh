#!/bin/bash
# round 3 session s: chunk size of the order-independent sums per side --
# GPU tests of the default (users 4, items 1), then a fixed-count A/B of the
# CG iteration over the chunk variants and the committed build.
set -o pipefail
OUT=gpurun_out/r03s; mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@"
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$name rc=$rc: stop"; exit $rc; fi
}
timeout -k 10 700 python -u -m pytest tests/test_gpu_cgls.py tests/test_gpu_parity.py tests/test_distributed.py -m gpu -v --timeout 400 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $OUT/gpu_tests.log | tail -12
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "TESTS rc=$rc: stop"; exit $rc; fi
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
tail -1 $OUT/smoke.log
for v in new head u4i2 u2i2 u4i4 u2i1; do
  if [ $v = new ]; then LP=""; else LP=var_libs/$v/cpp_ls_lib.so; fi
  MR_LIB_PATH=$LP step ab_$v 300 python -u tools/cg_ab.py --k 64 --tag $v > $OUT/ab_${v}_k64.json 2> $OUT/ab_${v}_k64.err
done
for v in new head; do
  if [ $v = new ]; then LP=""; else LP=var_libs/$v/cpp_ls_lib.so; fi
  MR_LIB_PATH=$LP step ab128_$v 300 python -u tools/cg_ab.py --k 128 --tag $v > $OUT/ab_${v}_k128.json 2> $OUT/ab_${v}_k128.err
done
python3 - <<'PY'
import glob, json
for f in sorted(glob.glob("gpurun_out/r03s/ab_*.json")):
    d = json.load(open(f))
    print(f.split("/")[-1], "users", d["users"]["ms_per_cg_iteration"], d["users"]["kernels"].get("matvec_users"),
          "items", d["items"]["ms_per_cg_iteration"], d["items"]["kernels"].get("matvec_items"))
PY
echo DONE
