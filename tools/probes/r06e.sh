# resident vs launch-per-iteration after the load-wait fix (wall clock, fixed CG counts)
set -o pipefail
OUT=gpurun_out/r06e; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 -k "resident or golden or headline_paths or cg_iterations or sweep" > $OUT/tests.log 2>&1; echo "tests rc=$?"; tail -2 $OUT/tests.log
for args in "--k 64" "--k 64 --shard 0/8" "--k 128" "--k 128 --shard 0/8" "--k 64 --shard 0/4"; do
  for o in "cg_resident=0" "cg_resident=1"; do
    timeout -k 10 300 python -u tools/cg_ab.py $args --wall --opt $o --tag "$o" >> $OUT/ab.jsonl 2>> $OUT/ab.err || { echo "ab rc=$?"; exit 1; }
  done
done
MR_LIB_PATH=$PWD/var_libs/rstouch/cpp_ls_lib.so timeout -k 10 300 python -u tools/cg_ab.py --k 64 --shard 0/8 --wall --tag touch >> $OUT/ab.jsonl 2>> $OUT/ab.err
MR_LIB_PATH=$PWD/var_libs/rstouch/cpp_ls_lib.so timeout -k 10 300 python -u tools/cg_ab.py --k 64 --wall --tag touch >> $OUT/ab.jsonl 2>> $OUT/ab.err
for o in "cg_resident=0" "cg_resident=1"; do
  timeout -k 10 300 python -u bench.py --no-cpu --opt $o > $OUT/bench_$o.json 2> $OUT/bench_$o.err || { echo "bench rc=$?"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$o.json')); print('$o', d['value']/1e9, d['ms_per_step'], d['ms_per_step_with_kernel_events'], d['phase_ms_per_step'])"
done
