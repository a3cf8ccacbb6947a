#!/bin/bash
# GPU-box profiling session (after tools/gpu_check.sh is green): the default
# bench line, a rocprofv3 kernel-trace + stats pass of the same command, the
# two PMC traffic passes (FETCH_SIZE and WRITE_SIZE in separate runs), a
# k = 128 line and a single-rank RCCL (sharded path) line.
# Usage (via gpurun): bash tools/gpu_profile.sh TAG
set -o pipefail
TAG=${1:-prof}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@"
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$name rc=$rc: stop"; exit $rc; fi
}
step bench 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
step trace 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --no-cpu --steps 20 --warmup 5 > $OUT/bench_under_rocprof.json 2> $OUT/trace.err
step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/pmc_fetch -o run --output-format csv -- python3 bench.py --no-cpu --no-kernel-events --steps 3 --warmup 1 > /dev/null 2> $OUT/pmc_fetch.err
step pmc_write 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/pmc_write -o run --output-format csv -- python3 bench.py --no-cpu --no-kernel-events --steps 3 --warmup 1 > /dev/null 2> $OUT/pmc_write.err
python tools/pmc_summary.py --fetch $OUT/pmc_fetch --write $OUT/pmc_write --out $OUT/pmc.json
step k128 600 python -u bench.py --no-cpu --k 128 --steps 20 --warmup 3 > $OUT/bench_k128.json 2> $OUT/bench_k128.err
echo K128; cat $OUT/bench_k128.json
step shard1 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --no-cpu --steps 10 --warmup 2 --force-shard > $OUT/bench_shard1.json 2> $OUT/bench_shard1.err
echo SHARD1; cat $OUT/bench_shard1.json
echo DONE
