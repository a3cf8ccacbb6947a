"""CPU oracle for the ALS hot path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this package, and only as the checker.
The product (``movie_recommender_amd``) never imports it and has no CPU
fallback.

Contents
--------
``als_oracle``  NumPy/SciPy restatement of the reference algorithm
                (``cpp/ls_lib/matrix.cpp``) in two forms: the reference's own
                design-matrix form and the block-Gram form the HIP path uses.
``ref``         ctypes driver for ``oracle/_ref/cpp_ls_lib.so``, the
                reference library compiled from its own sources by
                ``oracle/Makefile`` (pins the restatement; CPU baseline).

Parity pinning: the restatement is checked against golden vectors produced by
the compiled reference (``tests/golden/``, generator
``tests/golden/make_golden.py``) in ``tests/test_oracle.py``.
"""
