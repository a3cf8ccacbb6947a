#!/bin/bash
# round 3 session aa: one-pass grid sized so every wave runs the same number
# of entity chunks (no partial last round), fixed CG counts, k = 64
set -o pipefail
OUT=gpurun_out/r03aa; mkdir -p $OUT
export TMPDIR=/tmp
for np in 0 920 900 880 0 920 E; do
  unset MR_MV_PARTS MR_EVEN_ROUNDS; if [ $np = E ]; then export MR_EVEN_ROUNDS=1; elif [ $np != 0 ]; then export MR_MV_PARTS=$np; fi
  timeout -k 10 300 python -u tools/cg_ab.py --k 64 --m 20 --reps 3 --tag parts$np >> $OUT/ab_k64.jsonl 2>> $OUT/ab.err || { echo "$np failed"; exit 1; }
done
unset MR_MV_PARTS
python3 - <<'PY'
import json
for l in open("gpurun_out/r03aa/ab_k64.jsonl"):
    d=json.loads(l); print(d["tag"], d["users"]["ms_per_cg_iteration"], d["items"]["ms_per_cg_iteration"], d["users"]["kernels"].get("matvec_users"), d["items"]["kernels"].get("matvec_items"))
PY
echo DONE
