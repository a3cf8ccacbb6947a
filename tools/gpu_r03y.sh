#!/bin/bash
# round 3 session y: users one-pass CG at k = 128 (fixed CG counts) vs matvec + update
set -o pipefail
OUT=gpurun_out/r03y; mkdir -p $OUT
export TMPDIR=/tmp
for v in new:1 new:2 updlast:2 w1:2 new:1 new:2 w1:2; do
  lib=${v%%:*}; op=${v##*:}
  if [ $lib = new ]; then unset MR_LIB_PATH; else export MR_LIB_PATH=$PWD/var_libs/$lib/cpp_ls_lib.so; fi
  timeout -k 10 300 python -u tools/cg_ab.py --k 128 --m 20 --reps 3 --tag ${lib}_op$op --opt cg_onepass=$op >> $OUT/ab_k128.jsonl 2>> $OUT/ab.err || { echo "$v failed"; exit 1; }
done
python3 - <<'PY'
import json
for l in open("gpurun_out/r03y/ab_k128.jsonl"):
    d=json.loads(l); print(d["tag"], d["users"]["ms_per_cg_iteration"], d["items"]["ms_per_cg_iteration"], d["users"]["kernels"])
PY
echo DONE
