# balanced chunk ranges: bitwise tests, timeline, wall A/B against one launch per iteration
set -o pipefail
OUT=gpurun_out/r06g; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 -k "resident or headline_paths or cg_iterations" > $OUT/tests.log 2>&1; echo "tests rc=$?"; tail -2 $OUT/tests.log
for args in "--shard 0/8 --side users" "--shard 0/8 --side items" "--side users" "--side items"; do
  MR_LIB_PATH=$PWD/var_libs/rsprof/cpp_ls_lib.so timeout -k 10 300 python -u tools/op_timeline.py --resident $args >> $OUT/timeline.jsonl 2>> $OUT/timeline.err || { echo "rc=$?"; exit 1; }
done
for args in "--k 64" "--k 64 --shard 0/8" "--k 128" "--k 128 --shard 0/8"; do
  for o in "cg_resident=0" "cg_resident=1"; do
    timeout -k 10 300 python -u tools/cg_ab.py $args --wall --opt $o --tag "$o" >> $OUT/ab.jsonl 2>> $OUT/ab.err || { echo "ab rc=$?"; exit 1; }
  done
done
for o in "cg_resident=0" "cg_resident=1"; do
  timeout -k 10 300 python -u bench.py --no-cpu --opt $o > $OUT/bench_$o.json 2> $OUT/bench_$o.err || { echo "bench rc=$?"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$o.json')); print('$o', d['value']/1e9, d['ms_per_step'], d['ms_per_step_with_kernel_events'], d['phase_ms_per_step'])"
done
