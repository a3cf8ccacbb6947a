# User-side rhs / row sums on the matrix cores at k = 64 (rhsm4:
# MR_RHSM_MIN_NB=4) against the VALU form: Gram parity on the variant, then
# the Gram time A/B (kernel time only: the rhs bits change, so the CG
# trajectory may too)
set -o pipefail
OUT=gpurun_out/r06l; mkdir -p $OUT; export TMPDIR=/tmp
MR_LIB_PATH=$PWD/var_libs/rhsm4/cpp_ls_lib.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "gram_kernel_vs_numpy or mlshape_golden" -m gpu > $OUT/tests_rhsm4.log 2>&1 || { echo "tests rc=$?"; tail -20 $OUT/tests_rhsm4.log; exit 1; }
tail -2 $OUT/tests_rhsm4.log
for v in base rhsm4 base rhsm4 base rhsm4; do
  if [ $v = base ]; then unset MR_LIB_PATH; else export MR_LIB_PATH=$PWD/var_libs/$v/cpp_ls_lib.so; fi
  timeout -k 10 300 python -u bench.py --no-cpu --no-same-window --steps 10 --warmup 3 > $OUT/bench_$v.json 2> $OUT/bench_$v.err || { echo "bench $v rc=$?"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$v.json')); print('$v', round(d['value']/1e9,3), d['ms_per_step'], d['cg_iterations']['per_step_users'], {k: v['avg_us'] for k, v in d['kernels'].items() if k.startswith('gram')})"
done
