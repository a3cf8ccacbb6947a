# Gram epilogue A/B: 16-byte tile stores through a quad transpose (gwidep,
# MR_G_WIDE=1) and waves per Gram block (gw1, gw2) against the default;
# hashes of G / factors first (gwidep must be bitwise the default)
set -o pipefail
OUT=gpurun_out/r06j; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 240 python -u tools/probes/g_hash.py > $OUT/hash_base.json 2> $OUT/hash_base.err || { echo "hash base rc=$?"; exit 1; }
MR_LIB_PATH=$PWD/var_libs/gwidep/cpp_ls_lib.so timeout -k 10 240 python -u tools/probes/g_hash.py > $OUT/hash_gwidep.json 2> $OUT/hash_gwidep.err || { echo "hash gwidep rc=$?"; exit 1; }
if cmp -s $OUT/hash_base.json $OUT/hash_gwidep.json; then echo "hash: gwidep identical"; else echo "hash: gwidep DIFFERS"; fi
for v in base gwidep gw1 gw2 base gwidep gw1; do
  if [ $v = base ]; then unset MR_LIB_PATH; else export MR_LIB_PATH=$PWD/var_libs/$v/cpp_ls_lib.so; fi
  timeout -k 10 300 python -u bench.py --no-cpu --no-same-window --steps 10 --warmup 3 > $OUT/bench_$v.json 2> $OUT/bench_$v.err || { echo "bench $v rc=$?"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$v.json')); print('$v', round(d['value']/1e9,3), d['ms_per_step'], {k: v['avg_us'] for k, v in d['kernels'].items() if k.startswith('gram')})"
done
for v in base gwidep; do
  if [ $v = base ]; then unset MR_LIB_PATH; else export MR_LIB_PATH=$PWD/var_libs/$v/cpp_ls_lib.so; fi
  timeout -k 10 300 python -u bench.py --no-cpu --no-same-window --steps 5 --warmup 2 --k 96 > $OUT/bench_k96_$v.json 2> $OUT/bench_k96_$v.err || { echo "bench k96 $v rc=$?"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_k96_$v.json')); print('k96 $v', round(d['value']/1e9,3), d['ms_per_step'], {k: v['avg_us'] for k, v in d['kernels'].items() if k.startswith('gram')})"
done
for v in base gwidep; do
  if [ $v = base ]; then unset MR_LIB_PATH; else export MR_LIB_PATH=$PWD/var_libs/$v/cpp_ls_lib.so; fi
  timeout -k 10 300 python -u bench.py --no-cpu --no-same-window --steps 5 --warmup 2 --k 128 > $OUT/bench_k128_$v.json 2> $OUT/bench_k128_$v.err || { echo "bench k128 $v rc=$?"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_k128_$v.json')); print('k128 $v', round(d['value']/1e9,3), d['ms_per_step'], {k: v['avg_us'] for k, v in d['kernels'].items() if k.startswith('gram')})"
done
