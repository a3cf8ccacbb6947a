set -o pipefail
for v in w3 w4 w3 w4; do
  MR_LIB_PATH=$PWD/var_libs/$v/cpp_ls_lib.so bash tools/gpu_session.sh r05y "ab=--tag $v --k 64 --m 10" || exit $?
done
echo DONE
