"""MI355X-native ALS core for louisyang2015/movie_recommender.

Hot path: the per-user / per-movie least-squares half-steps of ALS training
(reference ``cpp/ls_lib/matrix.cpp:744-1031``) as hand-written HIP kernels for
gfx950, behind the reference's ctypes ABI (``cpp_ls_lib.so``).

Modules
  cpp_ls      drop-in for the reference ``cpp/python/cpp_ls.py``
  engine      device-resident ALS context (``include/mr_als.h``)
  distributed one process per GPU, users/items sharded, factor all-gather
  synth       seeded MovieLens-shaped ratings (benchmarks, statistical tests)
  build       compiles ``lib/cpp_ls_lib.so`` with hipcc for gfx950
"""
__version__ = "0.1.0"
