set -o pipefail
for v in base xpre base xpre; do
  MR_LIB_PATH=$PWD/var_libs/$v/cpp_ls_lib.so bash tools/gpu_session.sh r05u "ab=--tag $v --k 128 --m 10" || exit $?
done
bash tools/ab_c5.sh r05u_c5 "base xpre" || exit $?
echo DONE
