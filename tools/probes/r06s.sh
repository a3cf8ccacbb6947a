# General-CG SpMV output-store policy A/B: default (base), non-temporal
# (spnt), write-through sc1 (spsc1); the K1 knock-out (profiles/r06/r06q)
# put 119 us of its 780 us in the 216 MB of output stores
set -o pipefail
OUT=gpurun_out/r06s; mkdir -p $OUT; export TMPDIR=/tmp
for v in spnt spsc1; do
  MR_LIB_PATH=$PWD/var_libs/$v/cpp_ls_lib.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_cgls.py -m gpu > $OUT/tests_$v.log 2>&1 || { echo "tests $v rc=$?"; tail -20 $OUT/tests_$v.log; exit 1; }
  echo "$v $(tail -1 $OUT/tests_$v.log)"
done
for v in base spnt spsc1 base spnt spsc1; do
  if [ $v = base ]; then unset MR_LIB_PATH; else export MR_LIB_PATH=$PWD/var_libs/$v/cpp_ls_lib.so; fi
  timeout -k 10 240 python -u bench_cg.py --no-cpu > $OUT/cg_$v.json 2> $OUT/cg_$v.err || { echo "bench_cg $v rc=$?"; tail -3 $OUT/cg_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/cg_$v.json')); print('$v', d['value'], d['iterations'], d['roofline']['frac'], {k: (v['avg_us'], v['launches']) for k, v in d['kernels'].items()})"
done
