#!/bin/bash
# One GPU-box session: parity tests, bench, rocprofv3 kernel trace + PMC passes.
# Usage (via gpurun): bash tools/gpu_round.sh TAG [bench args...]
set -o pipefail
TAG=${1:-run}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > $OUT/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 600 python bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err || { echo "BENCH FAILED"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --no-cpu --steps 10 --warmup 2 --force-shard > $OUT/bench_shard1.json 2> $OUT/bench_shard1.err || { echo "SHARD BENCH FAILED"; tail -20 $OUT/bench_shard1.err; exit 1; }
echo SHARD1; cat $OUT/bench_shard1.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --no-cpu --steps 10 --warmup 3 > $OUT/bench_trace.json 2> $OUT/bench_trace.err || { echo "TRACE FAILED"; tail -20 $OUT/bench_trace.err; exit 1; }
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/pmc_fetch -o run --output-format csv -- python3 bench.py --no-cpu --steps 3 --warmup 1 > /dev/null 2> $OUT/pmc_fetch.err || { echo "PMC FETCH FAILED"; tail -20 $OUT/pmc_fetch.err; exit 1; }
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/pmc_write -o run --output-format csv -- python3 bench.py --no-cpu --steps 3 --warmup 1 > /dev/null 2> $OUT/pmc_write.err || { echo "PMC WRITE FAILED"; tail -20 $OUT/pmc_write.err; exit 1; }
python tools/pmc_summary.py --fetch $OUT/pmc_fetch --write $OUT/pmc_write --out $OUT/pmc.json

timeout -k 10 600 python bench.py --no-cpu --k 128 --steps 20 > $OUT/bench_k128.json 2> $OUT/bench_k128.err || { echo "K128 BENCH FAILED"; tail -20 $OUT/bench_k128.err; exit 1; }
echo K128; cat $OUT/bench_k128.json
echo DONE
