#!/bin/bash
# End-of-round measurement session: the default bench line, a rocprofv3
# kernel-trace + stats pass of the same command, the two PMC traffic passes
# (FETCH_SIZE and WRITE_SIZE in separate runs) at k = 64 and at k = 128.
# Usage (via gpurun): bash tools/gpu_profile_final.sh TAG
set -o pipefail
TAG=${1:-final}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "[$TAG] $name" >&2
  timeout -k 10 $secs "$@"
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$name rc=$rc: stop"; exit $rc; fi
}
step bench 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
tail -c 400 $OUT/bench.json
step trace 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --no-cpu --steps 20 --warmup 5 > $OUT/bench_under_rocprof.json 2> $OUT/trace.err
python tools/rocprof_agree.py $OUT/trace $OUT/bench_under_rocprof.json --out $OUT/rocprof_vs_events.json > /dev/null
for K in 64 128; do
  # counters per CG iteration: the launch-per-iteration path (the resident
  # solve makes the same accesses per iteration, bench.py scales by its
  # iterations per launch)
  step pmc_fetch_k$K 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/pmc_fetch_k$K -o run --output-format csv -- python3 bench.py --no-cpu --no-kernel-events --k $K --steps 3 --warmup 1 --opt cg_resident=0 > /dev/null 2> $OUT/pmc_fetch_k$K.err
  step pmc_write_k$K 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/pmc_write_k$K -o run --output-format csv -- python3 bench.py --no-cpu --no-kernel-events --k $K --steps 3 --warmup 1 --opt cg_resident=0 > /dev/null 2> $OUT/pmc_write_k$K.err
  python tools/pmc_summary.py --fetch $OUT/pmc_fetch_k$K --write $OUT/pmc_write_k$K --out $OUT/pmc_k$K.json --k $K
done
echo DONE
