# where the resident iteration's fixed cost goes (MR_OP_PROF build)
set -o pipefail
OUT=gpurun_out/r06f; mkdir -p $OUT; export TMPDIR=/tmp
export MR_LIB_PATH=$PWD/var_libs/rsprof/cpp_ls_lib.so
for args in "--shard 0/8 --side users" "--shard 0/8 --side items" "--side users" "--side items" "--shard 0/8 --side users --k 128"; do
  timeout -k 10 300 python -u tools/op_timeline.py --resident $args >> $OUT/timeline.jsonl 2>> $OUT/timeline.err || { echo "rc=$?"; exit 1; }
  tail -1 $OUT/timeline.jsonl
done
