#!/bin/bash
# round 3 session ae: write-through publish (no L2 write-back per published
# CG state) -- parity with the variant, then fixed-count A/B and bench
set -o pipefail
OUT=gpurun_out/r03ae; mkdir -p $OUT
export TMPDIR=/tmp
V=$PWD/var_libs/pubwt/cpp_ls_lib.so
MR_LIB_PATH=$V timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "headline or sweep or peer or sharded or replay or cgls or mlshape or dense" > $OUT/tests.log 2>&1
rc=$?; tail -1 $OUT/tests.log
if [ $rc -ne 0 ]; then echo "tests rc=$rc: stop"; exit $rc; fi
for v in base wt base wt; do
  if [ $v = wt ]; then export MR_LIB_PATH=$V; else unset MR_LIB_PATH; fi
  timeout -k 10 300 python -u tools/cg_ab.py --k 64 --m 20 --reps 3 --tag $v >> $OUT/ab_k64.jsonl 2>> $OUT/ab.err || { echo "$v failed"; exit 1; }
done
python3 - <<'PY'
import json
for l in open("gpurun_out/r03ae/ab_k64.jsonl"):
    d=json.loads(l); print(d["tag"], d["users"]["ms_per_cg_iteration"], d["items"]["ms_per_cg_iteration"], d["users"]["kernels"].get("matvec_users"), d["items"]["kernels"].get("matvec_items"), d["users"]["gram_ms"], d["items"]["gram_ms"])
PY
for v in base wt; do
  if [ $v = wt ]; then export MR_LIB_PATH=$V; else unset MR_LIB_PATH; fi
  timeout -k 10 600 python -u bench.py --no-cpu > $OUT/bench_$v.json 2> $OUT/bench_$v.err || exit 1
  python3 -c "
import json; d=json.load(open('$OUT/bench_$v.json')); print('$v', d['value']/1e9, d['ms_per_step'], d['ms_per_step_with_kernel_events'], {k:v['avg_us'] for k,v in d['kernels'].items()})"
done
echo DONE
