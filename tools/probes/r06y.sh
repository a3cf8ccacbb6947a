# Round-6 final build at the other BASELINE shapes: ML-full k = 128 (C4's
# per-GPU problem) and one rank's C5 slice (1/8 of 10 M x 1 M, k = 128)
set -o pipefail
OUT=gpurun_out/r06y; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py --k 128 --no-cpu --steps 5 --warmup 2 > $OUT/bench_k128.json 2> $OUT/bench_k128.err || { echo "k128 rc=$?"; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_k128.json')); print('k128', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'])"
timeout -k 10 600 python -u bench.py --shape c5 --scale 0.125 --k 128 --no-cpu --steps 2 --warmup 1 > $OUT/bench_c5_slice_k128.json 2> $OUT/bench_c5.err || { echo "c5 rc=$?"; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_c5_slice_k128.json')); print('c5', d['value'], d['ms_per_step'], {k: v['avg_us'] for k, v in d['kernels'].items()})"
