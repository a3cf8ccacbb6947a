#!/bin/bash
# GPU-box session: smoke, all GPU tests (failures reported, not fatal), bench.
# Any fault / abort / timeout (exit status other than 0 or 1) ends the session.
# Usage (via gpurun): bash tools/gpu_check.sh TAG [pytest -k expr] [-- bench args...]
set -o pipefail
TAG=${1:-check}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
KEXPR=""
if [ $# -gt 0 ] && [ "$1" != "--" ]; then KEXPR=$1; shift; fi
[ "$1" == "--" ] && shift
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; tail -3 $OUT/smoke.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "SMOKE rc=$rc: stop"; exit $rc; fi
if [ -n "$KEXPR" ]; then
  timeout -k 10 1200 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "$KEXPR" > $OUT/tests.log 2>&1
else
  timeout -k 10 1200 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
fi
rc=$?
grep -E "FAILED|ERROR" $OUT/tests.log | head -40; tail -2 $OUT/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "TESTS rc=$rc: stop"; exit $rc; fi
timeout -k 10 600 python -u bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err
rc=$?
cat $OUT/bench.json; tail -3 $OUT/bench.err
exit $rc
