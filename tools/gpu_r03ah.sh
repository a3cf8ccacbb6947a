#!/bin/bash
# round 3 session ah: fused-start GEMV without per-tile sched barriers (Gram
# epilogue), same-box A/B at fixed CG counts; C5 one-rank slice and C1 on HEAD
set -o pipefail
OUT=gpurun_out/r03ah; mkdir -p $OUT
export TMPDIR=/tmp
V=$PWD/var_libs/nosb/cpp_ls_lib.so
for v in base nosb base nosb; do
  if [ $v = nosb ]; then export MR_LIB_PATH=$V; else unset MR_LIB_PATH; fi
  timeout -k 10 300 python -u tools/cg_ab.py --k 64 --m 4 --reps 3 --tag $v >> $OUT/ab_k64.jsonl 2>> $OUT/ab.err || { echo "$v failed"; exit 1; }
done
unset MR_LIB_PATH
python3 - <<'PY'
import json
for l in open("gpurun_out/r03ah/ab_k64.jsonl"):
    d=json.loads(l); print(d["tag"], "gram ms users/items", d["users"]["gram_ms"], d["items"]["gram_ms"], d["users"]["kernels"].get("gram_users"), d["items"]["kernels"].get("gram_items"))
PY
timeout -k 10 900 python -u bench.py --no-cpu --shape c5 --scale 0.125 --k 128 --steps 3 --warmup 1 > $OUT/bench_c5_slice_k128.json 2> $OUT/bench_c5.err || { echo c5 failed; exit 1; }
cut -c1-250 $OUT/bench_c5_slice_k128.json
timeout -k 10 600 python -u bench.py --shape ml-100k --k 10 --steps 50 --warmup 3 > $OUT/bench_c1_ml100k_k10.json 2> $OUT/bench_c1.err || { echo c1 failed; exit 1; }
cut -c1-250 $OUT/bench_c1_ml100k_k10.json
echo DONE
