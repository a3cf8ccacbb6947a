"""CG-count parity at the bench workload: the engine's half-steps started
from the compiled reference's own states (GPU + the reference on the host).

    python tools/cg_count_parity.py [--scale 1.0] [--iterations 25] [--threads N]
                                    [--out F]

The reference's ALS (``oracle/ref_replay.als_replay``: ``als()``,
``matrix.cpp:814-892``, restated around the reference's own
``cg_least_squares``, bit-identical to ``als_from_python``) runs on the
bench data (ML-full shape at ``--scale``, k = 64, RandomState(0) start) with
its outer stop test off.  Before every one of its CG solves the engine gets
the same state (``set_factors``: U, V as the reference holds them, rounded to
the engine's fp32 tables) and runs the same half-step with the reference's
CG defaults (0.01, 200); its CG iteration count and final rr are recorded
beside the reference's.  Two runs of a chaotic trajectory part after a few
iterations (the reference's own thread counts do), so counts over a window
of two trajectories compare draws; from the same state they compare the
solvers.  With ``--alt-threads T`` every reference solve is also run at T
threads from the same state: the reference's own summation-order spread of
the counts, the yardstick for the engine's.  One JSON line per half-step
and a summary line.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(scale=1.0, iterations=25, threads=None, k=64, seed=0, out=None, log=print,
        alt_threads=None, engine=True):
    import bench
    from oracle import ref
    from oracle.ref_replay import als_replay
    if engine:
        from movie_recommender_amd.engine import AlsContext
    rs = bench.load_data("ml-full", k, scale=scale)
    U0, V0 = ref.init_factors(rs.num_users, rs.num_items, k, seed)
    if threads is None:
        threads, _ = bench.cpu_share()
    ref.set_thread_count(threads)
    recs = []
    t0 = time.time()
    import contextlib
    with (AlsContext(rs.user_ids, rs.item_ids, rs.ratings, k, rs.num_users, rs.num_items)
          if engine else contextlib.nullcontext()) as ctx:
        def on_half_step(side, it, U, V, alt):
            if engine:
                ctx.set_factors(U, V)
                its, rr = ctx.half_step(side)
            else:   # CPU exploration: the reference's own spread only
                its, rr = -1, float("nan")
            rec = {"iteration": it + 1, "side": side, "engine": [its, rr]}
            if alt_threads:
                rec["reference_alt"] = list(alt(alt_threads))
            recs.append(rec)

        def on_iteration(it, rec):
            for r in recs[-2:]:
                r["reference"] = [rec["cg_" + r["side"]],
                                  rec["rr"] if r["side"] == "items" else None]
                if out:
                    out.write(json.dumps(r) + "\n")
                    out.flush()
            log(f"[cg_count_parity] iteration {it + 1}: users engine {recs[-2]['engine'][0]} "
                f"reference {rec['cg_users']}, items engine {recs[-1]['engine'][0]} reference "
                f"{rec['cg_items']} ({time.time() - t0:.0f} s)")

        als_replay(rs.user_ids, rs.item_ids, rs.ratings, k, U0, V0, min_r_decrease=-np.inf,
                   max_iteration=iterations, on_iteration=on_iteration,
                   on_half_step=on_half_step)
    ref.set_thread_count(1)
    summ = {"scale": scale, "k": k, "n": int(rs.n), "iterations": iterations,
            "threads": threads, "alt_threads": alt_threads}
    for side in ("users", "items"):
        rr = [r for r in recs if r["side"] == side]
        eq = sum(r["engine"][0] == r["reference"][0] for r in rr)
        summ[side] = {"half_steps": len(rr), "equal_counts": eq,
                      "engine_total": sum(r["engine"][0] for r in rr),
                      "reference_total": sum(r["reference"][0] for r in rr),
                      "unequal": [[r["iteration"], r["engine"][0], r["reference"][0]]
                                  for r in rr if r["engine"][0] != r["reference"][0]]}
        if alt_threads:
            summ[side]["reference_alt_equal_counts"] = sum(
                r["reference_alt"][0] == r["reference"][0] for r in rr)
            summ[side]["reference_alt_unequal"] = [
                [r["iteration"], r["reference_alt"][0], r["reference"][0]]
                for r in rr if r["reference_alt"][0] != r["reference"][0]]
        if side == "items":
            rel = [abs(r["engine"][1] - r["reference"][1]) / abs(r["reference"][1]) for r in rr
                   if r["engine"][0] == r["reference"][0]]
            summ[side]["final_rr_max_rel_diff_equal_counts"] = max(rel) if rel else None
    return recs, summ


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--iterations", type=int, default=25)
    ap.add_argument("--threads", type=int, default=None)
    ap.add_argument("--alt-threads", type=int, default=None,
                    help="also run each reference solve at this thread count (its own spread)")
    ap.add_argument("--out", default=None)
    ap.add_argument("--no-engine", action="store_true", help="reference spread only (CPU)")
    a = ap.parse_args()
    f = open(a.out, "w") if a.out else None
    _, summ = run(a.scale, a.iterations, a.threads, out=f,
                  log=lambda m: print(m, file=sys.stderr, flush=True), alt_threads=a.alt_threads,
                  engine=not a.no_engine)
    line = json.dumps({"summary": summ})
    print(line, flush=True)
    if f:
        f.write(line + "\n")
        f.close()


if __name__ == "__main__":
    main()
