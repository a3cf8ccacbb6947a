#!/bin/bash
# round 3 session v: cached-tail experiment on the alternating sweep
set -o pipefail
OUT=gpurun_out/r03v; mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@"
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$name rc=$rc: stop"; exit $rc; fi
}
for mb in 0 64 128 192 256 0 96 160; do
  MR_SWEEP_TAIL_MB=$mb step ab_$mb 300 python -u tools/cg_ab.py --k 64 --m 20 --reps 3 --tag tail$mb --opt cg_sweep=1 >> $OUT/ab_k64.jsonl 2> $OUT/ab.err
done
python3 - <<'PY'
import json
for l in open("gpurun_out/r03v/ab_k64.jsonl"):
    d=json.loads(l); print(d["tag"], d["users"]["ms_per_cg_iteration"], d["items"]["ms_per_cg_iteration"], d["users"]["kernels"].get("matvec_users"), d["items"]["kernels"].get("matvec_items"), d["users"]["gram_ms"], d["items"]["gram_ms"])
PY
echo DONE
