#!/bin/bash
# GPU-box session (round 3): selected GPU tests (failures reported, not
# fatal), then one benchmark command.  Any fault / abort / timeout (exit
# status other than 0 or 1 from pytest) ends the session before the bench.
# Usage (via gpurun): bash tools/gpu_r03.sh TAG "pytest selection" "bench command"
set -o pipefail
TAG=$1; SEL=$2; BENCH=$3
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$SEL" ]; then
  timeout -k 10 1000 python -u -m pytest $SEL -m gpu -v --timeout 400 --timeout-method thread > $OUT/tests.log 2>&1
  rc=$?
  grep -E "FAILED|ERROR|passed|failed" $OUT/tests.log | tail -30
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "TESTS rc=$rc: stop"; exit $rc; fi
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 900 $BENCH > $OUT/bench.json 2> $OUT/bench.err
  rc=$?
  cat $OUT/bench.json; tail -8 $OUT/bench.err
  exit $rc
fi
