# HBM traffic of the general-CG kernels (rocprofv3 PMC: FETCH_SIZE and
# WRITE_SIZE in separate passes) at the reference harness's 27e6 x 2.8e6
# matrix, 12 CG iterations
set -o pipefail
OUT=gpurun_out/r06pmc_cg; mkdir -p $OUT; export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/fetch -o run --output-format csv -- python3 bench_cg.py --no-cpu --solves 1 --max-iteration 12 > /dev/null 2> $OUT/fetch.err || { echo "fetch rc=$?"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/write -o run --output-format csv -- python3 bench_cg.py --no-cpu --solves 1 --max-iteration 12 > /dev/null 2> $OUT/write.err || { echo "write rc=$?"; exit 1; }
echo DONE
