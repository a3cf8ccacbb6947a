#!/bin/bash
# Gram bound analysis: the f32 Gram kernel vs its probes (1: gathers from a
# 1024-row cache-resident slice; 2: no MFMA), then PMC passes on the default.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/gprobe; mkdir -p $OUT
for v in default probe1 probe2; do
  L=movie_recommender_amd/lib/cpp_ls_lib.so; [ $v != default ] && L=var_libs/$v/cpp_ls_lib.so
  MR_LIB_PATH=$PWD/$L timeout -k 10 300 python tools/gram_bench.py "$@" > $OUT/$v.json 2> $OUT/$v.err || { tail -5 $OUT/$v.err; exit 1; }
  echo $v; cat $OUT/$v.json
done
bash tools/pmc_session.sh gprobe/pmc "$@"
