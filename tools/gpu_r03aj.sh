#!/bin/bash
# round 3 session aj: the batched bin collection (tools/patches) as a variant
# library: parity subset, then a same-box A/B at fixed CG counts and bench
set -o pipefail
OUT=gpurun_out/r03aj; mkdir -p $OUT
export TMPDIR=/tmp
V=$PWD/var_libs/new/cpp_ls_lib.so
MR_LIB_PATH=$V timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "xsum or headline or sweep or peer or sharded or replay or mlshape or dense or cg_iterations" > $OUT/tests.log 2>&1
rc=$?; tail -1 $OUT/tests.log
if [ $rc -ne 0 ]; then echo "tests rc=$rc: stop"; exit $rc; fi
for v in old new old new; do
  if [ $v = new ]; then export MR_LIB_PATH=$V; else unset MR_LIB_PATH; fi
  timeout -k 10 300 python -u tools/cg_ab.py --k 64 --m 20 --reps 3 --tag $v >> $OUT/ab_k64.jsonl 2>> $OUT/ab.err || { echo "$v failed"; exit 1; }
done
python3 - <<'PY'
import json
for l in open("gpurun_out/r03aj/ab_k64.jsonl"):
    d=json.loads(l); print(d["tag"], d["users"]["ms_per_cg_iteration"], d["items"]["ms_per_cg_iteration"], d["users"]["kernels"].get("matvec_users"), d["items"]["kernels"].get("matvec_items"), d["users"]["gram_ms"], d["items"]["gram_ms"])
PY
MR_LIB_PATH=$V timeout -k 10 600 python -u bench.py --no-cpu > $OUT/bench_new.json 2> $OUT/bench.err || { echo bench failed; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/bench_new.json')); print(d['value']/1e9, d['ms_per_step'], d['cg_iterations']['users_total'], d['cg_iterations']['items_total'], {k:v['avg_us'] for k,v in d['kernels'].items()})"
echo DONE
