# 16-byte write-through G stores (gwsc1: MR_G_WIDE=1 MR_G_SC1=1, with the
# store-data hazard nop) against the default: G / factor hashes, Gram A/B at
# k = 64 and 128, and the C5 slice
set -o pipefail
OUT=gpurun_out/r06o; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 240 python -u tools/probes/g_hash.py > $OUT/hash_base.json 2> $OUT/hash_base.err || { echo "hash base rc=$?"; exit 1; }
MR_LIB_PATH=$PWD/var_libs/gwsc1/cpp_ls_lib.so timeout -k 10 240 python -u tools/probes/g_hash.py > $OUT/hash_gwsc1.json 2> $OUT/hash_gwsc1.err || { echo "hash gwsc1 rc=$?"; exit 1; }
if cmp -s $OUT/hash_base.json $OUT/hash_gwsc1.json; then echo "hash: gwsc1 identical"; else echo "hash: gwsc1 DIFFERS"; exit 1; fi
for v in base gwsc1 base gwsc1 base gwsc1; do
  if [ $v = base ]; then unset MR_LIB_PATH; else export MR_LIB_PATH=$PWD/var_libs/$v/cpp_ls_lib.so; fi
  timeout -k 10 300 python -u bench.py --no-cpu --no-same-window --steps 10 --warmup 3 > $OUT/bench_$v.json 2> $OUT/bench_$v.err || { echo "bench $v rc=$?"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$v.json')); print('$v', round(d['value']/1e9,3), d['ms_per_step'], {k: v['avg_us'] for k, v in d['kernels'].items() if not k.startswith('slab') and not k.startswith('cg_start')})"
done
for v in base gwsc1; do
  if [ $v = base ]; then unset MR_LIB_PATH; else export MR_LIB_PATH=$PWD/var_libs/$v/cpp_ls_lib.so; fi
  timeout -k 10 300 python -u bench.py --no-cpu --no-same-window --steps 5 --warmup 2 --k 128 > $OUT/bench_k128_$v.json 2> $OUT/bench_k128_$v.err || { echo "bench k128 $v rc=$?"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_k128_$v.json')); print('k128 $v', round(d['value']/1e9,3), d['ms_per_step'], {k: v['avg_us'] for k, v in d['kernels'].items() if k.startswith('gram') or k.startswith('resident')})"
done
for v in base gwsc1; do
  if [ $v = base ]; then unset MR_LIB_PATH; else export MR_LIB_PATH=$PWD/var_libs/$v/cpp_ls_lib.so; fi
  timeout -k 10 300 python -u bench.py --no-cpu --shape c5 --scale 0.125 --k 128 --steps 2 --warmup 1 > $OUT/bench_c5_$v.json 2> $OUT/bench_c5_$v.err || { echo "bench c5 $v rc=$?"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_c5_$v.json')); print('c5 $v', d['ms_per_step'], {k: v['avg_us'] for k, v in d['kernels'].items() if k.startswith('gram')})"
done
