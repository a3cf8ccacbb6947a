set -o pipefail
for v in nopers persist nopers persist; do
  MR_LIB_PATH=$PWD/var_libs/$v/cpp_ls_lib.so bash tools/gpu_session.sh r05s "ab=--tag $v --k 128 --m 10" || exit $?
done
bash tools/ab_c5.sh r05s_c5 "nopers persist" || exit $?
echo DONE
