# full GPU suite + A/B + bench with CPU leg (round-6 build)
set -o pipefail
OUT=gpurun_out/r06h; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 1200 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "FAILED|ERROR" $OUT/tests.log | head; tail -2 $OUT/tests.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for args in "--k 64" "--k 64 --shard 0/8" "--k 64 --shard 0/4" "--k 128" "--k 128 --shard 0/8" "--k 128 --shard 0/4"; do
  for o in "cg_resident=0" "cg_resident=1"; do
    timeout -k 10 300 python -u tools/cg_ab.py $args --wall --opt $o --tag "$o" >> $OUT/ab.jsonl 2>> $OUT/ab.err || { echo "ab rc=$?"; exit 1; }
  done
done
timeout -k 10 900 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench rc=$?"; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value']/1e9, d['ms_per_step'], d['roofline'], d['cpu_baseline']['value'] if d['cpu_baseline'] else None)"
