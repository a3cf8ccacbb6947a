#!/bin/bash
# Same-box A/B of library variants on the C5 one-rank slice (k = 128):
# bash tools/ab_c5.sh TAG "A B A B" [bench args]
set -o pipefail
TAG=$1; ORDER=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
n=0
for v in $ORDER; do
  n=$((n+1))
  MR_LIB_PATH=$PWD/var_libs/$v/cpp_ls_lib.so timeout -k 10 300 python -u bench.py --no-cpu --shape c5 --scale 0.125 --k 128 --steps 2 --warmup 1 "$@" > $OUT/${n}_$v.json 2> $OUT/${n}_$v.err
  rc=$?; if [ $rc -ne 0 ]; then echo "$v rc=$rc: stop"; tail -5 $OUT/${n}_$v.err; exit $rc; fi
  python3 -c "
import json; d=json.load(open('$OUT/${n}_$v.json'))
k=d['kernels']; print('$v', round(d['value']/1e9,3), d['ms_per_step'], d['cg_iterations']['users_total'], d['cg_iterations']['items_total'], ' '.join(f'{c}={v[\"avg_us\"]}' for c,v in k.items()))"
done
