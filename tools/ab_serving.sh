#!/bin/bash
# Same-box A/B of library variants on bench_serving: bash tools/ab_serving.sh TAG "A B" WHAT
set -o pipefail
TAG=$1; ORDER=$2; WHAT=$3
OUT=gpurun_out/$TAG; mkdir -p $OUT
n=0
for v in $ORDER; do
  n=$((n+1))
  MR_LIB_PATH=$PWD/var_libs/$v/cpp_ls_lib.so timeout -k 10 300 python -u bench_serving.py --no-cpu --what $WHAT > $OUT/${n}_$v.json 2> $OUT/${n}_$v.err
  rc=$?; if [ $rc -ne 0 ]; then echo "$v rc=$rc: stop"; tail -5 $OUT/${n}_$v.err; exit $rc; fi
  echo "== $v"; cut -c1-600 $OUT/${n}_$v.json
done
