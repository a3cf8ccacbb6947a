"""General sparse least squares benchmark: the reference's own published
per-CG-iteration number (doc para 885-946; harness
``cpp/ls/main.cpp:760-798`` ``benchmark_least_squares``).

    python bench_cg.py [--rows 27e6] [--cols 2.8e6] [--per-row 10] [--solves 2]
                       [--cpu-iterations 10] [--no-cpu]

Matrix: the harness's ``fill_matrix_with_sparse_random_data``
(``main.cpp:838-905``): every row holds ``per_row`` consecutive columns from a
uniform start, values uniform(-10, 10); b uniform(-10, 10); x starts at 0.
The GPU solves through a device-resident ``mr_cg`` context (include/mr_cg.h:
A uploaded and transposed once, then ``--solves`` right-hand sides; the
reference harness regenerates A per solve, which only changes the data).

Printed: ONE JSON line -- ms per CG iteration (device time of the whole
solves / their iterations, and per kernel class from HIP events), a
``roofline`` for the dominant kernel (algorithmic bytes below / its mean
launch time, HBM 8 TB/s), the reference's published figures, and a
``cpu_baseline``: the reference library compiled from source
(``oracle/_ref``) running the SAME matrix for ``--cpu-iterations`` CG
iterations on this host's CPU share.

Algorithmic bytes per CG iteration (nnz = rows x per_row):
  spmv_a   t = A p      nnz (8 value + 4 column) + rows (8 offset + 8 t write)
                        + cols (8 r + 8 p read once)
  spmv_at  q = A^T t    nnz (8 + 4 + 8 gathered t) + cols (8 offset + 8 q write
                        + 8 r read + 8 p read + 8 p write)
  update   x, r += ...  cols (8 x read + 8 x write + 8 r read + 8 r write + 8 p + 8 q)
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0
# per-launch HBM bytes from rocprofv3 PMC passes of this bench
# (tools/probes/r06pmc_cg.sh -> profiles/r06/pmc_cg.json)
PMC_FILE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "r06", "pmc_cg.json")
PMC_KERNEL = {"spmv_a": "void mr::csr_spmv_kernel<1, 0, true>",
              "spmv_at": "void mr::csr_spmv_kernel<0, 1, true>",
              "update": "mr::cgls_update_kernel"}


def pmc_traffic(cls, rows, cols, per_row):
    """HBM bytes per launch of kernel class `cls` from the committed PMC
    summary -- only for the shape it was collected on (the default one)."""
    if (rows, cols, per_row) != (27_000_000, 2_800_000, 10) or not os.path.exists(PMC_FILE):
        return None
    ent = json.load(open(PMC_FILE)).get("per_kernel", {}).get(PMC_KERNEL.get(cls, ""))
    return ent["bytes_corrected"] if ent else None
PUBLISHED = {"ms_per_cg_iteration": {
    "c5.18xlarge alg1 (SpMV^T) 4/9/18/36/72 threads": [763, 422, 275, 360, 367],
    "c5.18xlarge alg2 (explicit transpose) 4/9/18/36/72 threads": [1042, 481, 261, 278, 208],
    "desktop i5-3350 4 threads alg1 / alg2": [1422, 1111]},
    "source": "doc/movie_recommendation.docx para 885-946 (BASELINE.md)",
    "best": 208.0}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def bench_matrix(rows, cols, per_row, seed=20261017):
    rng = np.random.default_rng(seed)
    start = rng.integers(0, cols - per_row + 1, rows, dtype=np.int64)
    ci = np.empty(rows * per_row, np.int32)
    ci2 = ci.reshape(rows, per_row)
    for j in range(per_row):
        ci2[:, j] = start + j
    del start
    rp = np.arange(0, rows * per_row + 1, per_row, dtype=np.int64).astype(np.int32)
    v = rng.uniform(-10, 10, rows * per_row)
    b = rng.uniform(-10, 10, rows)
    return rp, ci, v, b


def alg_bytes(cls, rows, cols, nnz):
    if cls == "spmv_a":
        return nnz * 12 + rows * 16 + cols * 16
    if cls == "spmv_at":
        return nnz * 20 + cols * 40
    if cls == "update":
        return cols * 48
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=float, default=27e6)
    ap.add_argument("--cols", type=float, default=2.8e6)
    ap.add_argument("--per-row", type=int, default=10)
    ap.add_argument("--solves", type=int, default=2)
    ap.add_argument("--max-iteration", type=int, default=200)
    ap.add_argument("--cpu-iterations", type=int, default=10)
    ap.add_argument("--cpu-threads", type=int, default=None)
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()
    rows, cols, k = int(args.rows), int(args.cols), args.per_row
    t0 = time.perf_counter()
    rp, ci, v, b = bench_matrix(rows, cols, k)
    nnz = len(v)
    log(f"[bench_cg] A {rows} x {cols}, {nnz} non-zeros ({time.perf_counter() - t0:.1f} s)")

    from movie_recommender_amd import _lib
    L = _lib.lib()
    t0 = time.perf_counter()
    h = L.mr_cg_create(0, rows, cols, rp.ctypes.data_as(_lib.IP), ci.ctypes.data_as(_lib.IP),
                       v.ctypes.data_as(_lib.DP))
    if not h:
        raise RuntimeError(_lib.last_error())
    t_create = time.perf_counter() - t0
    log(f"[bench_cg] context (upload + device transpose + row blocks) {t_create:.2f} s")
    _lib.check(L.mr_cg_set_timing(h, 1), "mr_cg_set_timing")
    # warm-up solve (not timed): 2 iterations
    x = np.zeros(cols)
    rr = ctypes.c_double(0)
    _lib.check(L.mr_cg_solve(h, b.ctypes.data_as(_lib.DP), x.ctypes.data_as(_lib.DP), 0.01, 2,
                             ctypes.byref(rr)), "mr_cg_solve")
    _lib.check(L.mr_cg_reset_stats(h), "mr_cg_reset_stats")
    x = np.zeros(cols)
    its, walls = [], []
    rng = np.random.default_rng(5)
    for sv in range(args.solves):
        bb = b if sv == 0 else rng.uniform(-10, 10, rows)
        t0 = time.perf_counter()
        it = _lib.check(L.mr_cg_solve(h, bb.ctypes.data_as(_lib.DP), x.ctypes.data_as(_lib.DP),
                                      0.01, args.max_iteration, ctypes.byref(rr)), "mr_cg_solve")
        walls.append(time.perf_counter() - t0)
        its.append(it)
        log(f"[bench_cg] solve {sv}: {it} CG iterations, final rr {rr.value:.4e}, "
            f"wall {walls[-1]:.3f} s (incl. b / x transfers)")
    st = _lib.MrCgStats()
    _lib.check(L.mr_cg_get_stats(h, ctypes.byref(st)), "mr_cg_get_stats")
    s = st.as_dict()
    L.mr_cg_destroy(h)
    n_it = sum(its)
    ms_it = s["solve_ms"] / n_it
    table = {}
    for c in ("spmv_a", "spmv_at", "update", "setup"):
        n = s["kernel_launches"][c]
        if not n:
            continue
        avg = s["kernel_ms"][c] / n
        by = alg_bytes(c, rows, cols, nnz)
        table[c] = {"total_ms": round(s["kernel_ms"][c], 3), "launches": n,
                    "avg_us": round(avg * 1e3, 2),
                    "alg_bytes": by, "alg_GBps": round(by / (avg / 1e3) / 1e9, 1) if by else None}
    dom = max((c for c in table if c != "setup"), key=lambda c: table[c]["total_ms"])
    ach = table[dom]["alg_GBps"]
    per_it_bytes = sum(alg_bytes(c, rows, cols, nnz) for c in ("spmv_a", "spmv_at", "update"))
    out = {
        "metric": "ms per CG iteration, cg_least_squares (A = 27e6 x 2.8e6, 10 nnz/row)",
        "value": round(ms_it, 4), "unit": "ms/CG-iteration", "higher_is_better": False,
        "n_gpus": 1, "dtype": "f64",
        "data": "synthetic (the reference harness's fill_matrix_with_sparse_random_data)",
        "config": {"workload": "cg_least_squares_from_python", "rows": rows, "cols": cols,
                   "nnz": nnz, "per_row": k, "solves": args.solves,
                   "blocks_a": s["blocks_a"], "blocks_at": s["blocks_at"]},
        "iterations": its, "solve_wall_s": [round(w, 3) for w in walls],
        "context_create_s": round(t_create, 2),
        "kernels": table,
        "roofline": {"kernel": dom, "bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                     "alg_bytes_per_launch": table[dom]["alg_bytes"],
                     "avg_launch_us": table[dom]["avg_us"],
                     "traffic": pmc_traffic(dom, rows, cols, k)},
        "iteration_roofline": {"alg_bytes_per_cg_iteration": per_it_bytes,
                               "GBps": round(per_it_bytes / (ms_it / 1e3) / 1e9, 1),
                               "frac": round(per_it_bytes / (ms_it / 1e3) / 1e9 / HBM_PEAK_GBS, 4)},
        "published": PUBLISHED,
        "vs_published_best": round(PUBLISHED["best"] / ms_it, 1),
    }
    if not args.no_cpu:
        out["cpu_baseline"] = cpu_leg(rp, ci, v, b, cols, args)
    print(json.dumps(out), flush=True)


def cpu_leg(rp, ci, v, b, cols, args):
    """The compiled reference (oracle/_ref, test infra) on the same matrix:
    cg_least_squares_from_python for a bounded number of CG iterations on
    this host's CPU share; ms per CG iteration = wall / iterations (its b2 =
    A^T b and r0 setup included, as in the published harness)."""
    sys.path.insert(0, ROOT)
    from oracle import ref
    from bench import cpu_share
    if not ref.available():
        return None
    share, info = cpu_share()
    tc = args.cpu_threads or share
    ref.set_thread_count(tc)
    t0 = time.perf_counter()
    _, it, _ = ref.cg_least_squares(rp, ci, v, cols, b, np.zeros(cols), 0.01,
                                    args.cpu_iterations)
    wall = time.perf_counter() - t0
    ref.set_thread_count(1)
    return {"value": round(wall / max(it, 1) * 1e3, 2), "unit": "ms/CG-iteration", "cores": tc,
            **info, "kind": "reference",
            "sample": (f"the same matrix, {it} CG iterations (max_iteration "
                       f"{args.cpu_iterations}), wall {wall:.2f} s incl. the b2 / r0 setup; "
                       f"oracle/_ref/cpp_ls_lib.so -O2, {tc} threads")}


if __name__ == "__main__":
    main()
