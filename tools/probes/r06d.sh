set -o pipefail
OUT=gpurun_out/r06d; mkdir -p $OUT; export TMPDIR=/tmp
for v in base sl8 sl32 rstouch rsmix; do
  for sh in "" "--shard 0/8"; do
    MR_LIB_PATH=$PWD/var_libs/$v/cpp_ls_lib.so timeout -k 10 300 python -u tools/cg_ab.py --k 64 --wall $sh --tag $v >> $OUT/ab.jsonl 2>> $OUT/ab.err || { echo "ab $v rc=$?"; exit 1; }
  done
  tail -2 $OUT/ab.jsonl | cut -c1-400
done
for v in base pgst pgath; do
  MR_LIB_PATH=$PWD/var_libs/$v/cpp_ls_lib.so timeout -k 10 300 python -u bench.py --no-cpu --steps 3 --warmup 1 --no-same-window > $OUT/probe_$v.json 2> $OUT/probe_$v.err || { echo "probe $v rc=$?"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/probe_$v.json')); print('$v', {k: v['avg_us'] for k, v in d['kernels'].items() if k.startswith('gram')})"
done
