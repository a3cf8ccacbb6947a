#!/bin/bash
# round 3 closing check: bench stdout is one JSON line (single and sharded
# launch), then the full GPU suite on HEAD
set -o pipefail
OUT=gpurun_out/r03ag; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --no-cpu --steps 5 --warmup 1 --force-shard > $OUT/shard.out 2> $OUT/shard.err || { echo "shard bench failed"; exit 1; }
timeout -k 10 300 python bench.py --no-cpu --steps 5 --warmup 1 > $OUT/single.out 2> $OUT/single.err || { echo "bench failed"; exit 1; }
wc -l $OUT/shard.out $OUT/single.out
python3 -c "
import json
for f in ('$OUT/shard.out', '$OUT/single.out'):
    json.loads(open(f).read())
print('one JSON line each')"
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR" $OUT/gpu_tests.log | head; tail -1 $OUT/gpu_tests.log
exit $rc
