#!/bin/bash
# Build a library variant for tools/ab.sh: kernels.hip recompiled with extra
# flags (e.g. -DMR_VAR_X), linked with the product objects of build/obj.
# Usage: bash tools/build_var.sh NAME [hipcc flags...]   (after `make` in csrc)
# SRC=path builds that file as the rebuilt unit (e.g. a `git show REV:...` copy);
# UNIT=serving (or any csrc/*.hip stem) recompiles that unit instead of kernels;
# UNITS="kernels engine" recompiles several units with the same flags (needed
# when a flag changes a header constant both units use, e.g. MR_GRAM_WAVES)
set -e
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/var_libs/$NAME
mkdir -p "$OUT"
OBJ=$ROOT/build/obj
UNITS=${UNITS:-${UNIT:-kernels}}
OBJS=""
for U in $UNITS; do
  SRCU=$ROOT/movie_recommender_amd/csrc/$U.hip
  [ -n "$SRC" ] && SRCU=$SRC   # SRC: the source of the (single) rebuilt unit
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result \
    -munsafe-fp-atomics $( [ "$U" = kernels ] && echo -fno-slp-vectorize ) "$@" \
    -I"$ROOT/movie_recommender_amd/csrc" -c "$SRCU" -o "$OUT/$U.o"
  OBJS="$OBJS $OUT/$U.o"
done
for O in $OBJ/*.o; do
  case " $UNITS " in *" $(basename "$O" .o) "*) ;; *) OBJS="$OBJS $O" ;; esac
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OBJS -o "$OUT/cpp_ls_lib.so" \
  -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib -Wl,-z,defs
echo "$OUT/cpp_ls_lib.so"
