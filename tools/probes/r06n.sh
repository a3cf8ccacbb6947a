# Gram G stores write-through (sc1: no dirty G lines left in L2) in the
# 4-byte (gsc1) and 16-byte (gwsc1) forms against the default non-temporal
# 4-byte stores: G hashes first (must be identical), then the Gram A/B
set -o pipefail
OUT=gpurun_out/r06n; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 240 python -u tools/probes/g_hash.py > $OUT/hash_base.json 2> $OUT/hash_base.err || { echo "hash base rc=$?"; exit 1; }
for v in gsc1 gwsc1; do
  MR_LIB_PATH=$PWD/var_libs/$v/cpp_ls_lib.so timeout -k 10 240 python -u tools/probes/g_hash.py > $OUT/hash_$v.json 2> $OUT/hash_$v.err || { echo "hash $v rc=$?"; exit 1; }
  if cmp -s $OUT/hash_base.json $OUT/hash_$v.json; then echo "hash: $v identical"; else echo "hash: $v DIFFERS"; fi
done
for v in base gsc1 gwsc1 base gsc1 gwsc1; do
  if [ $v = base ]; then unset MR_LIB_PATH; else export MR_LIB_PATH=$PWD/var_libs/$v/cpp_ls_lib.so; fi
  timeout -k 10 300 python -u bench.py --no-cpu --no-same-window --steps 10 --warmup 3 > $OUT/bench_$v.json 2> $OUT/bench_$v.err || { echo "bench $v rc=$?"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$v.json')); print('$v', round(d['value']/1e9,3), d['ms_per_step'], {k: v['avg_us'] for k, v in d['kernels'].items() if not k.startswith('slab') and not k.startswith('cg_start')})"
done
for v in base gwsc1; do
  if [ $v = base ]; then unset MR_LIB_PATH; else export MR_LIB_PATH=$PWD/var_libs/$v/cpp_ls_lib.so; fi
  timeout -k 10 300 python -u bench.py --no-cpu --no-same-window --steps 5 --warmup 2 --k 128 > $OUT/bench_k128_$v.json 2> $OUT/bench_k128_$v.err || { echo "bench k128 $v rc=$?"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_k128_$v.json')); print('k128 $v', round(d['value']/1e9,3), d['ms_per_step'], {k: v['avg_us'] for k, v in d['kernels'].items() if k.startswith('gram')})"
done
