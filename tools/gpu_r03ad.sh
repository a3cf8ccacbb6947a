#!/bin/bash
# round 3 session ad: CG_START control folded into cg_start_split -- parity
# (headline paths incl. split starts, sharded peer tests, sweep), then bench
set -o pipefail
OUT=gpurun_out/r03ad; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "headline or sweep or peer or sharded or replay or scale or band or mlshape or dense" > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log
if [ $rc -ne 0 ]; then echo "tests rc=$rc: stop"; exit $rc; fi
timeout -k 10 600 python -u bench.py --no-cpu > $OUT/bench.json 2> $OUT/bench.err || exit 1
python3 -c "
import json; d=json.load(open('$OUT/bench.json')); print(d['value']/1e9, d['ms_per_step'], d['ms_per_step_with_kernel_events'], d['cg_iterations']['users_total'], d['cg_iterations']['items_total'], {k:(v['avg_us'],v['launches']) for k,v in d['kernels'].items()})"
echo DONE
