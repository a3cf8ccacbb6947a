#!/bin/bash
# round 3 final profile set (HEAD): smoke, default bench (CPU baseline),
# rocprof stats, PMC traffic, k = 128, single-rank sharded peer run
set -o pipefail
OUT=gpurun_out/r03af; mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@"
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$name rc=$rc: stop"; exit $rc; fi
}
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
tail -1 $OUT/smoke.log
step bench 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
cut -c1-300 $OUT/bench.json
step trace 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --no-cpu --steps 20 --warmup 5 > $OUT/bench_under_rocprof.json 2> $OUT/trace.err
step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/pmc_fetch -o run --output-format csv -- python3 bench.py --no-cpu --no-kernel-events --steps 3 --warmup 1 > /dev/null 2> $OUT/pmc_fetch.err
step pmc_write 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/pmc_write -o run --output-format csv -- python3 bench.py --no-cpu --no-kernel-events --steps 3 --warmup 1 > /dev/null 2> $OUT/pmc_write.err
python tools/pmc_summary.py --fetch $OUT/pmc_fetch --write $OUT/pmc_write --out $OUT/pmc.json
step k128 600 python -u bench.py --no-cpu --k 128 --steps 20 --warmup 3 > $OUT/bench_k128.json 2> $OUT/bench_k128.err
step shard_peer 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --no-cpu --steps 20 --warmup 3 --force-shard --scalars peer > $OUT/bench_shard1_peer.json 2> $OUT/bench_shard1_peer.err
echo DONE
