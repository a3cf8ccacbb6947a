# Score kernel epilogue: the 8 biases and 4 medians loaded together before
# use (base) against round 6's previous kernel (scold: loaded per (user,
# candidate) under the range tests); serving GPU tests first (bit-exact)
set -o pipefail
OUT=gpurun_out/r06u; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_serving.py -m gpu > $OUT/tests.log 2>&1 || { echo "tests rc=$?"; tail -20 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for v in base scold base scold; do
  if [ $v = base ]; then unset MR_LIB_PATH; else export MR_LIB_PATH=$PWD/var_libs/$v/cpp_ls_lib.so; fi
  timeout -k 10 300 python -u bench_serving.py --what topn --no-cpu > $OUT/topn_$v.json 2> $OUT/topn_$v.err || { echo "bench $v rc=$?"; tail -3 $OUT/topn_$v.err; exit 1; }
  python3 -c "
import json
for ln in open('$OUT/topn_$v.json'):
    d=json.loads(ln); r=d.get('roofline',{}); print('$v', d.get('value'), d.get('unit'), r.get('avg_launch_ms'), r.get('frac_of_no_fma_ceiling'), r.get('select_ms'))"
done
