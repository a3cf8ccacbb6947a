set -o pipefail
mkdir -p gpurun_out/r05p
n=0
for v in spdef spbig spdef spbig; do
  n=$((n+1))
  MR_LIB_PATH=$PWD/var_libs/$v/cpp_ls_lib.so timeout -k 10 240 python -u bench_cg.py --no-cpu --solves 2 > gpurun_out/r05p/${n}_$v.json 2> gpurun_out/r05p/${n}_$v.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/r05p/${n}_$v.json'));print('$v', d['value'], d['iterations'], {k:v['avg_us'] for k,v in d['kernels'].items()})"
  grep "final rr" gpurun_out/r05p/${n}_$v.err
done
echo DONE
