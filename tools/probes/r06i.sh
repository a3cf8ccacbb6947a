# Gram workgroup size (waves per block) A/B, same box, fixed CG counts via the bench's replay
set -o pipefail
OUT=gpurun_out/r06i; mkdir -p $OUT; export TMPDIR=/tmp
for v in base gw1 gw2 base gw1 gw2; do
  if [ $v = base ]; then unset MR_LIB_PATH; else export MR_LIB_PATH=$PWD/var_libs/$v/cpp_ls_lib.so; fi
  timeout -k 10 300 python -u bench.py --no-cpu --no-same-window --steps 10 --warmup 3 > $OUT/bench_$v.json 2> $OUT/bench_$v.err || { echo "bench $v rc=$?"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$v.json')); print('$v', round(d['value']/1e9,3), d['ms_per_step'], {k: v['avg_us'] for k, v in d['kernels'].items() if k.startswith('gram')})"
done
unset MR_LIB_PATH
for k in 128; do
  for v in base gw1; do
    if [ $v = base ]; then unset MR_LIB_PATH; else export MR_LIB_PATH=$PWD/var_libs/$v/cpp_ls_lib.so; fi
    timeout -k 10 300 python -u bench.py --no-cpu --no-same-window --steps 5 --warmup 2 --k $k > $OUT/bench_k${k}_$v.json 2> $OUT/bench_k${k}_$v.err || { echo "bench rc=$?"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/bench_k${k}_$v.json')); print('k$k $v', round(d['value']/1e9,3), d['ms_per_step'], {k: v['avg_us'] for k, v in d['kernels'].items() if k.startswith('gram')})"
  done
done
