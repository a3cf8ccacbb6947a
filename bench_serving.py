"""Benchmarks of the SURVEY.md 8(f) rows beside the ALS core, on MI355X.

    python bench_serving.py [--what topn,eval,foldin] [--reps 3] [--no-cpu]

One JSON line per workload (synthetic data of the ML-full shape, seeded):

* ``topn``   -- recommendation lists per second: for a batch of users, score
  every movie (the reference's fp64 predict, bit-exact order), drop the
  user's rated movies, keep the first 400 by (score, movie id)
  (``recommend.py:86-106``).  50,367 movies x k = 64 (the ML-full training
  shape of bench.py), 65,536 users, each excluding ~200 rated movies (lognormal list sizes).
* ``eval``   -- held-out test ratings per second of ``_als_eval``
  (``worker_process.py:262-306``): prediction + ranking agreement per test
  user; 103k users, 10 % of the ML-full ratings held out.
* ``foldin`` -- users per second folded in as ``models.ALS_Model`` does
  (lstsq on ``[V, 1]`` with the raw ratings), at the app's k = 11
  (``app_local/als11_*``), 65,536 users with 12-400 ratings.
* ``similar`` -- similar-movie lists per second (``build_similar_movies_db``:
  every movie against every movie through co-rating users, genre gate, top
  20), all 58k movies of the ML-full raw shape (23.3 M ratings).
* ``fsim``   -- movie-movie cosine lists per second on the ALS factor layout
  (north star; ``similar.similar_by_factors``): all 50,367 movies x k = 64,
  top 20 other movies each, on the serving score / select kernels.
* ``prep``   -- training ratings per second through the ALS data preparation
  (``movie_lens_data.py:547-680``): medians, the in-place shrink for the
  reference's factors (3, 5, 7, 9, 11), first-appearance id order and the
  training arrays, on the ML-full raw shape (27.75 M ratings before shrink).

``value`` is device throughput (sum of the HIP-event kernel times of the
call, inputs resident in HBM); ``wall_inclusive`` adds the host<->device
copies of the C-ABI call.  ``roofline`` prices the dominant kernel;
``cpu_baseline`` times the reference algorithm (``oracle/serving_oracle.py``,
the reference's own Python control flow with NumPy) on a bounded sample.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FP64_PEAK_TFS = 78.6     # MI355X FP64 vector peak (FMA = 2 flops)
HBM_PEAK_GBS = 8000.0


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def movie_side(k, n_movies, seed):
    rs = np.random.RandomState(seed)
    V = rs.normal(0, 0.35, (n_movies, k))
    mids = np.sort(rs.choice(np.arange(1, 200_000), n_movies, replace=False))
    als_ids = {int(m): j for j, m in enumerate(mids)}
    med = rs.choice(np.arange(1, 11) / 2.0, n_movies)
    has = rs.random_sample(n_movies) < 0.97
    medians = {int(m): float(v) for m, v, h in zip(mids, med, has) if h}
    pop = 1.0 / (1 + rs.permutation(n_movies)) ** 0.9
    pop /= pop.sum()
    return V.reshape(-1), als_ids, medians, mids, pop


def user_lists(rs, mids, pop, n_users, lo, hi, mean):
    """Per-user distinct movies, popularity-weighted, lognormal list sizes."""
    sizes = np.clip(rs.lognormal(np.log(mean), 1.0, n_users).astype(int), lo, hi)
    draw = (sizes * 1.3).astype(int) + 4
    cdf = np.cumsum(pop)
    picks = np.minimum(np.searchsorted(cdf, rs.random_sample(int(draw.sum())) * cdf[-1]),
                       len(mids) - 1)
    out, o = [], 0
    for n, d in zip(sizes, draw):
        u = np.unique(picks[o:o + d])
        o += d
        if len(u) < n:                       # top up with uniform picks
            extra = rs.choice(len(mids), n * 2, replace=False)
            u = np.unique(np.concatenate([u, extra]))
        out.append(mids[rs.permutation(u)[:n]])
    return out


def line(metric, value, unit, cfg, roof, cpu, extra):
    d = {"metric": metric, "value": value, "unit": unit, "n_gpus": 1,
         "higher_is_better": True, "dtype": "f64", "data": "synthetic (ML-full shape, seeded)",
         "config": cfg, "roofline": roof, "cpu_baseline": cpu}
    d.update(extra)
    print(json.dumps(d), flush=True)


def bench_topn(a):
    from movie_recommender_amd.serving import MovieTable
    from oracle import serving_oracle as O
    k, nm, B, N = 64, 50_367, a.users, 400
    V, als_ids, medians, mids, pop = movie_side(k, nm, 1)
    rs = np.random.RandomState(2)
    X = rs.normal(0, 0.35, (B, k + 1))
    X[:, k] = rs.normal(0, 0.3, B)
    rated = user_lists(rs, mids, pop, B, 20, 2000, 120)
    # the rated lists as one CSR pair of arrays (top_n_arrays' loop-free input)
    r_off = np.concatenate([[0], np.cumsum([len(l) for l in rated])]).astype(np.int64)
    r_ids = np.concatenate(rated).astype(np.int64)
    with MovieTable(k, V, als_ids, medians) as t:
        nc = t.num_candidates
        t.top_n_arrays(X[:256], rated[:256], N)                 # warm-up
        best = None
        for _ in range(a.reps):
            t0 = time.perf_counter()
            t.top_n_arrays(X, (r_off, r_ids), N)
            wall = time.perf_counter() - t0
            ms = t.kernel_ms()
            dev = ms["scores"] + ms["exclude"] + ms["select"]
            if best is None or dev < best[0]:
                best = (dev, wall, ms)
    dev, wall, ms = best
    flops = B * nc * (2.0 * k + 2)        # k mul + k add + bias + median per score
    score_tfs = flops / (ms["scores"] * 1e-3) / 1e12
    sel_bytes = B * nc * 8.0 * 2 + B * nc * 4.0 * 2          # 2 passes over keys + ids
    roof = {"kernel": "rec_score_kernel", "bound": "fp64-valu", "achieved": round(score_tfs, 2),
            "peak": FP64_PEAK_TFS, "unit": "TFLOP/s", "frac": round(score_tfs / FP64_PEAK_TFS, 4),
            "frac_of_no_fma_ceiling": round(score_tfs / (FP64_PEAK_TFS / 2), 4),
            "traffic": None,
            "note": "exact reference order forbids FMA: separate v_mul_f64 + v_add_f64, "
                    "so 0.5 of the FMA-counted peak is the ceiling",
            "avg_launch_ms": round(ms["scores"], 3),
            "select_ms": round(ms["select"], 3),
            "select_GBps_2pass": round(sel_bytes / (ms["select"] * 1e-3) / 1e9, 1)}
    cpu = None
    if not a.no_cpu:
        ns = 6
        t0 = time.perf_counter()
        for u in range(ns):
            O.recommend(X[u], set(int(m) for m in rated[u]), medians, V, als_ids, N)
        dt = time.perf_counter() - t0
        cpu = {"value": ns / dt, "unit": "lists/s", "cores": 1, "kind": "port",
               "sample": f"{ns} users of the same workload through the reference's "
                         "get_recommendations loop (oracle/serving_oracle.recommend)"}
    line("recommendation lists/s (top-400 of 50k movies, k=64, rated movies excluded)",
         B / (dev * 1e-3), "lists/s",
         {"workload": "top-N", "users": B, "movies": nc, "k": k, "num_results": N},
         roof, cpu, {"wall_inclusive": B / wall,
                     "wall_note": "MovieTable.top_n_arrays with the rated lists as a CSR pair: "
                                  "host exclusion mapping, copies and the kernels",
                     "kernel_ms": ms})


def bench_eval(a):
    from movie_recommender_amd.serving import MovieTable
    from oracle import serving_oracle as O
    k, nm, nu = 64, 50_367, 102_982
    V, als_ids, medians, mids, pop = movie_side(k, nm, 3)
    rs = np.random.RandomState(4)
    U = rs.normal(0, 0.35, nu * (k + 1))
    lists = user_lists(rs, mids, pop, nu, 2, 1500, 12)
    tests = [[(int(m), float(r)) for m, r in zip(l, rs.choice(np.arange(1, 11) / 2.0, len(l)))]
             for l in lists]
    rows = np.arange(nu, dtype=np.int32)
    n_r = sum(len(l) for l in tests)
    with MovieTable(k, V, als_ids, medians) as t:
        t.evaluate(U, rows[:100], tests[:100])
        best = None
        for _ in range(a.reps):
            t0 = time.perf_counter()
            res = t.evaluate(U, rows, tests)
            wall = time.perf_counter() - t0
            ms = t.kernel_ms()["evaluate"]
            if best is None or ms < best[0]:
                best = (ms, wall)
    ms, wall = best
    pairs = float(sum(len(l) ** 2 for l in tests))
    byts = n_r * (k * 8.0 + 8 + 4 + 8 + 8)        # gathered movie row + median + id + rating + pred
    roof = {"kernel": "rec_eval_kernel", "bound": "hbm", "achieved": round(byts / (ms * 1e-3) / 1e9, 1),
            "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(byts / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), "traffic": None,
            "pair_comparisons": pairs, "avg_launch_ms": round(ms, 3)}
    cpu = None
    if not a.no_cpu:
        ns = 3000
        ids = {u: u for u in range(ns)}
        t0 = time.perf_counter()
        O.als_eval([(u, tests[u]) for u in range(ns)], medians, U, ids, V, als_ids, k)
        dt = time.perf_counter() - t0
        cpu = {"value": sum(len(tests[u]) for u in range(ns)) / dt, "unit": "test ratings/s",
               "cores": 1, "kind": "port",
               "sample": f"first {ns} test users through the reference's _als_eval loop "
                         "(oracle/serving_oracle.als_eval)"}
    line("held-out test ratings/s evaluated (prediction + ranking agreement, k=64)",
         n_r / (ms * 1e-3), "test ratings/s",
         {"workload": "evaluation", "test_users": nu, "test_ratings": n_r, "k": k},
         roof, cpu, {"wall_inclusive": n_r / wall,
                     "users_with_agreement": int(np.isfinite(res["agreement"]).sum())})


def bench_foldin(a):
    from movie_recommender_amd.serving import MovieTable
    from oracle import serving_oracle as O
    k, nm, B = 11, 22_809, a.users
    V, als_ids, medians, mids, pop = movie_side(k, nm, 5)
    rs = np.random.RandomState(6)
    lists = user_lists(rs, mids, pop, B, k + 1, 400, 60)
    lists = [[(int(m), float(r)) for m, r in zip(l, rs.choice(np.arange(1, 11) / 2.0, len(l)))]
             for l in lists]
    rows = sum(len(l) for l in lists)
    with MovieTable(k, V, als_ids, medians) as t:
        t.fold_in(lists[:100])
        best = None
        for _ in range(a.reps):
            t0 = time.perf_counter()
            valid, X, method = t.fold_in(lists)
            wall = time.perf_counter() - t0
            ms = t.kernel_ms()
            dev = ms["fold_in"] + ms["fold_in_svd"]
            if best is None or dev < best[0]:
                best = (dev, wall, ms, int((method == 2).sum()))
    dev, wall, ms, n_svd = best
    K = k + 1
    flops = rows * 2.0 * (K * (K + 1) / 2 + K) + B * (K ** 3 / 3.0)
    tfs = flops / (ms["fold_in"] * 1e-3) / 1e12
    roof = {"kernel": "fold_in_kernel", "bound": "fp64-valu", "achieved": round(tfs, 3),
            "peak": FP64_PEAK_TFS, "unit": "TFLOP/s", "frac": round(tfs / FP64_PEAK_TFS, 4),
            "traffic": None, "avg_launch_ms": round(ms["fold_in"], 3), "svd_users": n_svd}
    cpu = None
    if not a.no_cpu:
        ns = 2000
        t0 = time.perf_counter()
        for u in range(ns):
            O.fold_in(k, lists[u], V, als_ids)
        dt = time.perf_counter() - t0
        cpu = {"value": ns / dt, "unit": "users/s", "cores": 1, "kind": "port",
               "sample": f"first {ns} users through models.ALS_Model's fold-in "
                         "(oracle/serving_oracle.fold_in: numpy.linalg.lstsq)"}
    line("users folded in per second (ALS_Model lstsq, k=11)", B / (dev * 1e-3), "users/s",
         {"workload": "fold-in", "users": B, "ratings": rows, "k": k}, roof, cpu,
         {"wall_inclusive": B / wall})


def bench_prep(a):
    from movie_recommender_amd import synth
    from movie_recommender_amd.prep import TrainingSet, _reference_set_order
    from oracle import prep_oracle as O
    nu, ni, nd = synth.SHAPES["ml-full"]
    u, i, r = synth.raw_pairs(nu, ni, nd)
    order = np.lexsort((np.random.RandomState(1).random_sample(len(u)), u))  # user lists
    u, i, r = u[order].astype(np.int32), i[order].astype(np.int32), r[order]
    factors = [3, 5, 7, 9, 11]
    n = len(r)
    best = None
    for _ in range(a.reps):
        t0 = time.perf_counter()
        with TrainingSet(u, i, r) as ts:
            ms = 0.0
            med = ts.medians()
            ms += ts.last_ms()
            for j, k in enumerate(factors):
                keep, rounds, nk, nus, nms = ts.shrink(k, restart=(j == 0))
                ms += ts.last_ms()
                per = ts.first_appearance(np.array([0, n], np.int64))
                ms += ts.last_ms()
                mo = _reference_set_order([per[0][1]])
                uo = _reference_set_order([per[0][0]])
                umap = np.full(ts.user_bound, -1, np.int32)
                mmap = np.full(ts.movie_bound, -1, np.int32)
                umap[uo] = np.arange(len(uo), dtype=np.int32)
                mmap[mo] = np.arange(len(mo), dtype=np.int32)
                ts.convert(umap, mmap, np.nan_to_num(med))
                ms += ts.last_ms()
                conv_ms = ts.last_ms()
        wall = time.perf_counter() - t0
        if best is None or ms < best[0]:
            best = (ms, wall, nk, nus, nms, conv_ms)
    ms, wall, nk, nus, nms, conv_ms = best
    # dominant call: the training-array build (flag -> scan -> scatter); bytes
    # = alive flag, 8-byte flag and position, ids and rating read per input
    # rating + 16 B written per kept rating
    byts = n * (1 + 8 + 8 + 4 + 4 + 8) + nk * 16.0
    roof = {"kernel": "mr_prep_convert (flag scan + prep_convert_kernel)", "bound": "hbm",
            "achieved": round(byts / (conv_ms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(byts / (conv_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "traffic": None, "avg_call_ms": round(conv_ms, 3), "total_device_ms": round(ms, 3)}
    cpu = None
    if not a.no_cpu:
        # the reference's Python loop on a user sample (one process)
        users = np.unique(u)
        pick = np.random.RandomState(3).choice(users, len(users) // 50, replace=False)
        sel = np.isin(u, pick)
        lists, cur, lst = [], None, None
        for uu, mm, rr in zip(u[sel].tolist(), i[sel].tolist(), r[sel].tolist()):
            if uu != cur:
                cur, lst = uu, []
                lists.append((uu, lst))
            lst.append((mm, rr))
        ns = sum(len(l) for _, l in lists)
        t0 = time.perf_counter()
        med_s = O.movie_medians(lists)
        O.als_data_set_shrink([lists], [None], med_s, factors)
        dt = time.perf_counter() - t0
        cpu = {"value": ns / dt, "unit": "ratings/s", "cores": 1, "kind": "port",
               "sample": f"{len(lists)} users (2 %), {ns} ratings through the reference's "
                         "preparation loop (oracle/prep_oracle, one process)"}
    line("training ratings/s prepared (medians + shrink for k=3,5,7,9,11 + id maps + arrays)",
         n / (ms * 1e-3), "ratings/s",
         {"workload": "prep", "ratings": n, "factors": factors, "kept_k11": nk,
          "users_k11": nus, "movies_k11": nms}, roof, cpu, {"wall_inclusive": n / wall})


def bench_similar(a):
    from movie_recommender_amd import synth
    from movie_recommender_amd.similar import SimilarMovieFinder
    from oracle import similar_oracle as O
    nu, ni, nd = synth.SHAPES["ml-full"]
    u, i, r = synth.raw_pairs(nu, ni, nd)
    order = np.argsort(i, kind="stable")
    u, i, r = u[order], i[order], r[order]
    M = int(i.max()) + 1
    off = np.zeros(M + 1, np.int64)
    np.cumsum(np.bincount(i, minlength=M), out=off[1:])
    rs = np.random.RandomState(7)
    gm = np.zeros(M, np.uint64)
    for g in range(3):
        gm |= (np.uint64(1) << rs.randint(0, 20, M).astype(np.uint64))
    has = (rs.random_sample(M) < 0.99).astype(np.uint8)
    r2 = np.round(2 * r).astype(np.uint8)
    ids = np.arange(1, M + 1, dtype=np.int64)
    with SimilarMovieFinder.from_arrays(ids, off, u, r2, int(u.max()) + 1, gm, has) as f:
        f.find_many(np.arange(64), 20)
        best = None
        for _ in range(max(1, a.reps - 1)):
            t0 = time.perf_counter()
            oj, os_, oc = f.find_many(None, 20)
            wall = time.perf_counter() - t0
            ms = f.last_ms()
            if best is None or ms < best[0]:
                best = (ms, wall)
    ms, wall = best
    # algorithmic work: every (query, co-rated movie) contribution = one
    # entry of a rater's list = sum over users of deg(u)^2
    deg = np.bincount(u).astype(np.float64)
    upd = float((deg ** 2).sum())
    roof = {"kernel": "sim_find_kernel", "bound": "lds-atomics",
            "achieved": round(upd / (ms * 1e-3) / 1e9, 2), "peak": None,
            "unit": "G pair-updates/s", "frac": None, "traffic": None,
            "pair_updates": upd, "avg_launch_ms": round(ms, 2),
            "note": "two 64-bit LDS atomics + one 5-byte list read per update"}
    cpu = None
    if not a.no_cpu:
        # the reference's find_similar_movie (oracle) over dicts of a 1/8 user sample
        keep = u % 8 == 0
        us, is_, rs_ = u[keep], i[keep], r[keep]
        mr = [(int(m + 1), {}) for m in range(M)]
        for uu, mm, x in zip(us.tolist(), is_.tolist(), rs_.tolist()):
            mr[mm][1][uu] = x
        genres = {int(m + 1): {int(b) for b in range(20) if (int(gm[m]) >> b) & 1}
                  for m in range(M) if has[m]}
        t0 = time.perf_counter()
        nq = 3
        for q in range(nq):
            O.find_similar_movie(genres, mr, q, 0.05, 100, 20)
        dt = time.perf_counter() - t0
        cpu = {"value": nq / dt, "unit": "lists/s", "cores": 1, "kind": "port",
               "sample": f"{nq} query movies through the reference's find_similar_movie "
                         f"(oracle) on a 1/8 user sample ({int(keep.sum())} ratings)"}
    line("similar-movie lists/s (all movies of ML-full shape, top 20, genre gate)",
         M / (ms * 1e-3), "lists/s",
         {"workload": "similar-movies", "movies": M, "users": int(u.max()) + 1,
          "ratings": int(len(r)), "num_results": 20}, roof, cpu,
         {"wall_inclusive": M / wall, "movies_with_results": int((oc > 0).sum())})


def bench_fsim(a):
    from movie_recommender_amd.serving import MovieTable
    k, nm, N = 64, 50_367, 20
    V, als_ids, _, mids, _ = movie_side(k, nm, 1)
    V = V.reshape(nm, k)
    Vn = V / np.linalg.norm(V, axis=1)[:, None]
    zero_med = {m: 0.0 for m in als_ids}
    X = np.zeros((nm, k + 1))
    X[:, :k] = Vn
    self_excl = [[int(m)] for m in mids]
    with MovieTable(k, Vn, als_ids, zero_med) as t:
        t.top_n_arrays(X[:256], self_excl[:256], N)                 # warm-up
        best = None
        for _ in range(a.reps):
            t0 = time.perf_counter()
            t.top_n_arrays(X, self_excl, N)
            wall = time.perf_counter() - t0
            ms = t.kernel_ms()
            dev = ms["scores"] + ms["exclude"] + ms["select"]
            if best is None or dev < best[0]:
                best = (dev, wall, ms)
    dev, wall, ms = best
    flops = nm * nm * (2.0 * k + 2)
    score_tfs = flops / (ms["scores"] * 1e-3) / 1e12
    roof = {"kernel": "rec_score_kernel", "bound": "fp64-valu", "achieved": round(score_tfs, 2),
            "peak": FP64_PEAK_TFS, "unit": "TFLOP/s", "frac": round(score_tfs / FP64_PEAK_TFS, 4),
            "frac_of_no_fma_ceiling": round(score_tfs / (FP64_PEAK_TFS / 2), 4),
            "traffic": None, "avg_launch_ms": round(ms["scores"], 3),
            "select_ms": round(ms["select"], 3)}
    cpu = None
    if not a.no_cpu:
        ns = 200
        t0 = time.perf_counter()
        for j in range(ns):          # cosine of one movie against all, top 20 by (score, id)
            sc = Vn @ Vn[j]
            sc[j] = -np.inf
            top = np.lexsort((-mids, -sc))[:N]
        dt = time.perf_counter() - t0
        cpu = {"value": ns / dt, "unit": "lists/s",
               "cores": int(os.environ.get("OMP_NUM_THREADS", "1")), "kind": "port",
               "sample": f"{ns} query movies: NumPy cosine against all {nm} (BLAS GEMV, "
                         "OMP_NUM_THREADS threads) and a (score, id) sort"}
    line("movie-movie cosine lists/s (factor layout, 50k movies, k=64, top 20)",
         nm / (dev * 1e-3), "lists/s",
         {"workload": "factor cosine top-N", "movies": nm, "k": k, "num_results": N},
         roof, cpu, {"wall_inclusive": nm / wall, "kernel_ms": ms})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--what", default="topn,eval,foldin,prep,similar,fsim")
    ap.add_argument("--users", type=int, default=65536)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--no-cpu", action="store_true")
    a = ap.parse_args()
    for w in a.what.split(","):
        t0 = time.time()
        {"topn": bench_topn, "eval": bench_eval, "foldin": bench_foldin, "prep": bench_prep,
         "similar": bench_similar, "fsim": bench_fsim}[w](a)
        log(f"[bench_serving] {w} done in {time.time() - t0:.1f}s")


if __name__ == "__main__":
    main()
