# General-CG SpMV knock-out probes (timing only, wrong results): which part of
# K1 (t = A p, 27e6 rows x 10 non-zeros) keeps it below the 6.2 TB/s its bare
# stream reaches (tools/probes/stream_probe.hip, profiles/r06/r06p)?
# sp1 no gathers, sp2 no LDS staging / row sums, sp4 no output stores,
# sp8 no row-offset loads, sp14 = 2+4+8, sp15 = all
set -o pipefail
OUT=gpurun_out/r06q; mkdir -p $OUT; export TMPDIR=/tmp
for v in base sp1 sp2 sp4 sp8 sp14 sp15 base; do
  if [ $v = base ]; then unset MR_LIB_PATH; else export MR_LIB_PATH=$PWD/var_libs/$v/cpp_ls_lib.so; fi
  timeout -k 10 240 python -u bench_cg.py --no-cpu --solves 1 --max-iteration 12 > $OUT/cg_$v.json 2> $OUT/cg_$v.err || { echo "bench_cg $v rc=$?"; tail -3 $OUT/cg_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/cg_$v.json')); print('$v', d['iterations'], {k: (v['avg_us'], v['launches']) for k, v in d['kernels'].items()})"
done
