# Top-N exclusion kernel: 4 candidate ids loaded before the stores (base)
# against one id per trip (exold); serving tests first
set -o pipefail
OUT=gpurun_out/r06ex; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_serving.py -m gpu > $OUT/tests.log 2>&1 || { echo "tests rc=$?"; tail -20 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for v in base exold base exold; do
  if [ $v = base ]; then unset MR_LIB_PATH; else export MR_LIB_PATH=$PWD/var_libs/$v/cpp_ls_lib.so; fi
  timeout -k 10 300 python -u bench_serving.py --what topn --no-cpu > $OUT/topn_$v.json 2> $OUT/topn_$v.err || { echo "bench $v rc=$?"; tail -3 $OUT/topn_$v.err; exit 1; }
  python3 -c "
import json
for ln in open('$OUT/topn_$v.json'):
    d=json.loads(ln); r=d.get('roofline',{}); dev=65536/d['value']*1e3
    print('$v', round(d['value']), 'dev_ms', round(dev,3), 'score', r.get('avg_launch_ms'), 'select', r.get('select_ms'), 'exclude~', round(dev - r.get('avg_launch_ms') - r.get('select_ms'),3))"
done
