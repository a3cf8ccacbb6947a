#!/bin/bash
# round 3 session q: the order-independent CG sums -- full GPU suite (device
# xsum vs restatement, sharded == single bitwise), smoke, fixed-count A/B of
# the CG iteration against the committed build, default bench.
set -o pipefail
OUT=gpurun_out/r03q; mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@"
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$name rc=$rc: stop"; exit $rc; fi
}
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
tail -1 $OUT/smoke.log
for k in 64 128; do
  step ab_new_$k 300 python -u tools/cg_ab.py --k $k --tag new > $OUT/ab_new_k$k.json 2> $OUT/ab_new_k$k.err
  MR_LIB_PATH=var_libs/head/cpp_ls_lib.so step ab_head_$k 300 python -u tools/cg_ab.py --k $k --tag head > $OUT/ab_head_k$k.json 2> $OUT/ab_head_k$k.err
  cut -c1-400 $OUT/ab_new_k$k.json $OUT/ab_head_k$k.json
done
step bench 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
cut -c1-300 $OUT/bench.json
echo DONE
