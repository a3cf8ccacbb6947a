# Fold-in staging: 4 entries per thread in flight, branch-free (base)
# against one id per trip (fiold); serving tests first
set -o pipefail
OUT=gpurun_out/r06fi; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_serving.py -m gpu > $OUT/tests.log 2>&1 || { echo "tests rc=$?"; tail -20 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for v in base fiold base fiold; do
  if [ $v = base ]; then unset MR_LIB_PATH; else export MR_LIB_PATH=$PWD/var_libs/$v/cpp_ls_lib.so; fi
  timeout -k 10 300 python -u bench_serving.py --what foldin --no-cpu > $OUT/topn_$v.json 2> $OUT/topn_$v.err || { echo "bench $v rc=$?"; tail -3 $OUT/topn_$v.err; exit 1; }
  python3 -c "
import json
for ln in open('$OUT/topn_$v.json'):
    d=json.loads(ln); r=d.get('roofline',{}); print('$v', d.get('value'), d.get('unit'), r.get('avg_launch_ms'))"
done
