#!/bin/bash
# round 3 session j: opaque-tile one-pass A/B, then the round's profile set:
# default bench (CPU baseline), rocprofv3 stats, the two PMC traffic passes,
# k = 128, single-rank sharded (peer / collective scalars), full-C3 CPU
# baseline once, and the general-CG bench with its CPU leg.
set -o pipefail
OUT=gpurun_out/r03j; mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@"
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$name rc=$rc: stop"; exit $rc; fi
}
ab() { timeout -k 10 300 python -u tools/cg_ab.py "$@" >> $OUT/cg_ab.jsonl 2>> $OUT/cg_ab.err; }
ab --k 64 --tag default || exit $?
MR_LIB_PATH=$PWD/var_libs/opq4/cpp_ls_lib.so ab --k 64 --tag opq4 || exit $?
MR_LIB_PATH=$PWD/var_libs/opq3/cpp_ls_lib.so ab --k 64 --tag opq3 || exit $?
ab --k 64 --onepass 0 --tag twokernel || exit $?
cut -c1-400 $OUT/cg_ab.jsonl
step bench 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
cut -c1-300 $OUT/bench.json
step trace 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --no-cpu --steps 20 --warmup 5 > $OUT/bench_under_rocprof.json 2> $OUT/trace.err
step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/pmc_fetch -o run --output-format csv -- python3 bench.py --no-cpu --no-kernel-events --steps 3 --warmup 1 > /dev/null 2> $OUT/pmc_fetch.err
step pmc_write 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/pmc_write -o run --output-format csv -- python3 bench.py --no-cpu --no-kernel-events --steps 3 --warmup 1 > /dev/null 2> $OUT/pmc_write.err
python tools/pmc_summary.py --fetch $OUT/pmc_fetch --write $OUT/pmc_write --out $OUT/pmc.json; cat $OUT/pmc.json | head -40
step k128 600 python -u bench.py --no-cpu --k 128 --steps 20 --warmup 3 > $OUT/bench_k128.json 2> $OUT/bench_k128.err
cut -c1-300 $OUT/bench_k128.json
step shard_peer 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --no-cpu --steps 20 --warmup 3 --force-shard --scalars peer > $OUT/bench_shard1_peer.json 2> $OUT/bench_shard1_peer.err
step shard_coll 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29512 bench.py --no-cpu --steps 20 --warmup 3 --force-shard --scalars collective > $OUT/bench_shard1_coll.json 2> $OUT/bench_shard1_coll.err
cut -c1-300 $OUT/bench_shard1_peer.json $OUT/bench_shard1_coll.json
step cpu_full 900 python -u bench.py --steps 5 --cpu-scale 1.0 > $OUT/bench_cpu_full.json 2> $OUT/bench_cpu_full.err
step bench_cg 600 python -u bench_cg.py > $OUT/bench_cg.json 2> $OUT/bench_cg.err
echo DONE
