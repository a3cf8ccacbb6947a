set -o pipefail
mkdir -p gpurun_out/r05o
for v in sp0 sp1 sp2 sp3 sp0; do
  MR_LIB_PATH=$PWD/var_libs/$v/cpp_ls_lib.so timeout -k 10 240 python -u bench_cg.py --no-cpu --solves 1 --max-iteration 30 > gpurun_out/r05o/$v.json 2> gpurun_out/r05o/$v.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/r05o/$v.json'));print('$v', d['ms_per_cg_iteration'], {k:v['avg_us'] for k,v in d['kernels'].items()})"
done
for v in sp0 prio sp0 prio; do
  MR_LIB_PATH=$PWD/var_libs/$v/cpp_ls_lib.so timeout -k 10 300 python -u tools/cg_ab.py --tag $v --k 64 --m 10 --shard 0/8 >> gpurun_out/r05o/shard.jsonl 2>> gpurun_out/r05o/shard.err || exit $?
done
for v in sp0 prio; do
  MR_LIB_PATH=$PWD/var_libs/$v/cpp_ls_lib.so timeout -k 10 300 python -u tools/cg_ab.py --tag $v --k 64 --m 10 >> gpurun_out/r05o/full.jsonl 2>> gpurun_out/r05o/full.err || exit $?
done
echo DONE
