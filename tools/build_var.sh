#!/bin/bash
# Build a library variant for tools/ab.sh: kernels.hip recompiled with extra
# flags (e.g. -DMR_VAR_X), linked with the product objects of build/obj.
# Usage: bash tools/build_var.sh NAME [hipcc flags...]   (after `make` in csrc)
# SRC=path builds that kernels.hip instead (e.g. a `git show REV:...` copy);
# UNIT=serving (or any csrc/*.hip stem) recompiles that unit instead of kernels
set -e
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/var_libs/$NAME
mkdir -p "$OUT"
OBJ=$ROOT/build/obj
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result \
  -munsafe-fp-atomics $( [ "${UNIT:-kernels}" = kernels ] && echo -fno-slp-vectorize ) "$@" \
  -I"$ROOT/movie_recommender_amd/csrc" -c "${SRC:-$ROOT/movie_recommender_amd/csrc/${UNIT:-kernels}.hip}" \
  -o "$OUT/${UNIT:-kernels}.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC "$OUT/${UNIT:-kernels}.o" \
  $(ls $OBJ/*.o | grep -v "/${UNIT:-kernels}.o$") -o "$OUT/cpp_ls_lib.so" \
  -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib -Wl,-z,defs
echo "$OUT/cpp_ls_lib.so"
