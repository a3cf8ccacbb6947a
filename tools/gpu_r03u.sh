#!/bin/bash
# round 3 session u: sweep-direction (Infinity-Cache reuse) A/B of the one-pass
# CG at fixed CG counts, plain vs non-temporal G loads, bitwise-neutrality test.
set -o pipefail
OUT=gpurun_out/r03u; mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@"
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$name rc=$rc: stop"; exit $rc; fi
}
step test 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "sweep or replay" > $OUT/test.log 2>&1
tail -2 $OUT/test.log
for v in 0 1 2 0 1 2; do
  step ab_$v 300 python -u tools/cg_ab.py --k 64 --m 20 --reps 3 --tag sweep$v --opt cg_sweep=$v >> $OUT/ab_k64.jsonl 2> $OUT/ab.err
done
for v in 0 1; do
  MR_LIB_PATH=$PWD/var_libs/gnt0/cpp_ls_lib.so step abg_$v 300 python -u tools/cg_ab.py --k 64 --m 20 --reps 3 --tag gnt0_sweep$v --opt cg_sweep=$v >> $OUT/ab_k64.jsonl 2> $OUT/ab.err
done
python3 - <<'PY'
import json
for l in open("gpurun_out/r03u/ab_k64.jsonl"):
    d=json.loads(l); print(d["tag"], d["users"]["ms_per_cg_iteration"], d["items"]["ms_per_cg_iteration"], d["users"]["kernels"].get("matvec_users"), d["items"]["kernels"].get("matvec_items"))
PY
for v in 0 1; do
  step bench_$v 300 python -u bench.py --no-cpu --opt cg_sweep=$v > $OUT/bench_sweep$v.json 2> $OUT/bench_$v.err
  cut -c1-200 $OUT/bench_sweep$v.json
done
echo DONE
