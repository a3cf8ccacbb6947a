# Gram store-stream probes (timing only, wrong results): pg1 drops the G
# stores, pg3 keeps every store but aims them at 8 entities' G (L2-resident:
# no HBM writes) -- is the exposed store time HBM write bandwidth or the
# store path itself?
set -o pipefail
OUT=gpurun_out/r06k; mkdir -p $OUT; export TMPDIR=/tmp
for v in base pg3 pg1 base pg3 pg1; do
  if [ $v = base ]; then unset MR_LIB_PATH; else export MR_LIB_PATH=$PWD/var_libs/$v/cpp_ls_lib.so; fi
  timeout -k 10 300 python -u bench.py --no-cpu --no-same-window --steps 10 --warmup 3 > $OUT/bench_$v.json 2> $OUT/bench_$v.err || { echo "bench $v rc=$?"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$v.json')); print('$v', round(d['value']/1e9,3), d['ms_per_step'], {k: v['avg_us'] for k, v in d['kernels'].items() if k.startswith('gram')})"
done
