#!/bin/bash
# A/B timing of engine variants on one GPU box (tuning experiments).
# Usage: bash tools/ab_variants.sh "BENCH ARGS" NAME:ENVSPEC ...
# (ENVSPEC = comma-separated VAR=VAL, may be empty;
# MR_LIB_PATH=var_libs/X/cpp_ls_lib.so picks a variant build).
set -o pipefail
mkdir -p gpurun_out/var
export TMPDIR=/tmp
BARGS=$1; shift
for spec in "$@"; do
  v=${spec%%:*}; envs=${spec#*:}
  E=$(echo "$envs" | tr ',' ' ')
  env $E timeout -k 10 300 python bench.py --no-cpu $BARGS > gpurun_out/var/bench_$v.json 2> gpurun_out/var/bench_$v.err || { tail -5 gpurun_out/var/bench_$v.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/var/bench_$v.json')); k=d['kernels']
print('$v', d['ms_per_step'], d['ms_per_step_without_kernel_events'], d['cg_iterations'], {n: round(v['avg_us'],1) for n, v in k.items()})"
done
