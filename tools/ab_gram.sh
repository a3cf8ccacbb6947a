#!/bin/bash
# A/B of the Gram kernel alone (tools/gram_bench.py) over engine variants.
# Usage: bash tools/ab_gram.sh "GRAM_BENCH ARGS" NAME:ENVSPEC ...
set -o pipefail
mkdir -p gpurun_out/abg
export TMPDIR=/tmp
BARGS=$1; shift
for spec in "$@"; do
  v=${spec%%:*}; envs=${spec#*:}
  E=$(echo "$envs" | tr ',' ' ')
  env $E timeout -k 10 300 python tools/gram_bench.py $BARGS > gpurun_out/abg/$v.json 2> gpurun_out/abg/$v.err || { tail -5 gpurun_out/abg/$v.err; exit 1; }
  echo "$v $(cat gpurun_out/abg/$v.json)"
done
