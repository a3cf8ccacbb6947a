# HBM traffic of the resident CG solve measured on its own dispatches
# (rocprofv3 PMC, FETCH_SIZE and WRITE_SIZE in separate passes, k = 64): the
# replay slice's bytes over its CG iterations, against the per-iteration
# counters of the launch-per-iteration path the bench line uses
set -o pipefail
OUT=gpurun_out/r06pmc_res; mkdir -p $OUT; export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/fetch -o run --output-format csv -- python3 bench.py --no-cpu --no-same-window --steps 5 --warmup 2 > $OUT/bench_fetch.json 2> $OUT/fetch.err || { echo "fetch rc=$?"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/write -o run --output-format csv -- python3 bench.py --no-cpu --no-same-window --steps 5 --warmup 2 > $OUT/bench_write.json 2> $OUT/write.err || { echo "write rc=$?"; exit 1; }
echo DONE
