#!/bin/bash
# SQ counters of the bench kernels (one rocprofv3 --pmc pass, 8 SQ slots).
# Usage (via gpurun): bash tools/pmc_sq.sh TAG "COUNTERS"
set -o pipefail
TAG=${1:-sq}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
timeout -s KILL 240 rocprofv3 --pmc $2 --kernel-trace -d $OUT/pmc -o run --output-format csv -- python3 bench.py --no-cpu --no-kernel-events --steps 3 --warmup 1 > /dev/null 2> $OUT/pmc.err
rc=$?
tail -3 $OUT/pmc.err
python tools/pmc_kernels.py $OUT/pmc > $OUT/sq.txt 2>&1; cat $OUT/sq.txt
exit $rc
