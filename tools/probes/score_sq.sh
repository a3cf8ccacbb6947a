# SQ counters of the top-N score kernel (two --pmc passes, 8 SQ each at most)
set -o pipefail
OUT=gpurun_out/score_sq
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
pick() { local out=""; for c in "$@"; do grep -qw "$c" $OUT/counters.txt && out="$out $c"; done; echo $out; }
P1=$(pick SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS)
P2=$(pick SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_LDS SQ_INST_CYCLES_VALU SQ_WAIT_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM)
echo "P1: $P1"; echo "P2: $P2"
n=0
for P in "$P1" "$P2"; do
  n=$((n+1))
  timeout -s KILL 240 rocprofv3 --pmc $P --kernel-trace -d $OUT/pmc$n -o run --output-format csv -- python3 bench_serving.py --what topn --users 16384 --reps 1 --no-cpu > $OUT/b$n.json 2> $OUT/pmc$n.err || exit $?
  python tools/pmc_kernels.py $OUT/pmc$n > $OUT/sq$n.txt 2>&1; grep -A12 "rec_score" $OUT/sq$n.txt
done
echo DONE
