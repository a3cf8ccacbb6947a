#!/bin/bash
# Build an experimental variant of cpp_ls_lib.so with extra compile flags for
# kernels.hip (A/B timing on the GPU box via MR_LIB_PATH); not part of build().
# Usage: bash tools/build_variant.sh NAME "-DMACRO=VAL ..."
set -e
NAME=$1; FLAGS=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
make -s -C $ROOT/movie_recommender_amd/csrc -j8
OBJ=$ROOT/build/obj
OUT=$ROOT/var_libs/$NAME
mkdir -p $OUT
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result \
  -munsafe-fp-atomics $FLAGS -c $ROOT/movie_recommender_amd/csrc/kernels.hip -o $OUT/kernels.o
OBJS=$(ls $OBJ/*.o | grep -v '/kernels.o$')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OUT/kernels.o $OBJS -o $OUT/cpp_ls_lib.so \
  -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo $OUT/cpp_ls_lib.so
