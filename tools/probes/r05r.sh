set -o pipefail
for v in base gnt base gnt; do
  MR_LIB_PATH=$PWD/var_libs/$v/cpp_ls_lib.so bash tools/gpu_session.sh r05r "ab=--tag $v --k 64 --m 10" "ab=--tag $v --k 128 --m 10" || exit $?
done
bash tools/ab_c5.sh r05r_c5 "base gnt" || exit $?
echo DONE
