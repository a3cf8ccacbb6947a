set -o pipefail
mkdir -p gpurun_out/r03x
for v in onegather new onegather; do
  if [ $v = new ]; then unset MR_LIB_PATH; else export MR_LIB_PATH=$PWD/var_libs/$v/cpp_ls_lib.so; fi
  timeout -k 10 300 python -u bench_cg.py --no-cpu --solves 1 > gpurun_out/r03x/$v.json 2> gpurun_out/r03x/$v.err || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/r03x/$v.json')); k=d['kernels']
print('$v', d['value'], d['iterations'], {c: v['avg_us'] for c, v in k.items()})"
done
