#!/bin/bash
# Build a probe variant of the library: bash tools/probes/build_probe.sh N
# (N = MR_GRAM_PROBE value, see kernels.hip); output build/probeN/cpp_ls_lib.so
set -e
N=$1
D=build/probe$N
mkdir -p $D
for f in kernels gram3 csr_build engine capi serving prep similar; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -munsafe-fp-atomics \
    -DMR_GRAM_PROBE=$N -c movie_recommender_amd/csrc/$f.hip -o $D/$f.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $D/*.o -o $D/cpp_ls_lib.so \
  -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
