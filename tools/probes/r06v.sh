# Entities per sum term of the users one-pass / resident CG at k = 64
# (MR_XC_U: 4 default, 2, 1): full size deals 25,746 chunks of 4 over 4,096
# waves (7 vs 6.29 per wave: the last round runs 29 % of the waves); smaller
# chunks even that out.  Fixed CG counts, wall clock per CG iteration.
set -o pipefail
OUT=gpurun_out/r06v; mkdir -p $OUT; export TMPDIR=/tmp
for args in "--k 64" "--k 64 --shard 0/8" "--k 64 --shard 0/4"; do
  for v in base xcu2 xcu1 base xcu2 xcu1; do
    if [ $v = base ]; then unset MR_LIB_PATH; else export MR_LIB_PATH=$PWD/var_libs/$v/cpp_ls_lib.so; fi
    timeout -k 10 300 python -u tools/cg_ab.py $args --wall --tag "$v" >> $OUT/ab.jsonl 2>> $OUT/ab.err || { echo "ab rc=$?"; tail -3 $OUT/ab.err; exit 1; }
  done
done
python3 -c "
import json
for ln in open('$OUT/ab.jsonl'):
    d=json.loads(ln); print(d.get('tag'), d.get('shard'), d.get('k'), round(d['users']['wall_ms_per_cg_iteration']*1e3,1), round(d['items']['wall_ms_per_cg_iteration']*1e3,1))"
