#!/bin/bash
# Quick GPU iteration: parity tests (optional filter), then the bench.
# Usage (via gpurun): bash tools/gpu_quick.sh TAG [pytest -k expr] [-- bench args...]
set -o pipefail
TAG=${1:-quick}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
KEXPR=""
if [ $# -gt 0 ] && [ "$1" != "--" ]; then KEXPR=$1; shift; fi
[ "$1" == "--" ] && shift
if [ -n "$KEXPR" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$KEXPR" > $OUT/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $OUT/tests.log; exit 1; }
else
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $OUT/tests.log; exit 1; }
fi
tail -2 $OUT/tests.log
timeout -k 10 600 python bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err || { echo "BENCH FAILED"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
