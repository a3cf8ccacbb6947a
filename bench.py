"""Headline benchmark: ratings processed per second per ALS iteration
(BASELINE.json metric), MovieLens-full shape, k = 64, on MI355X.

    python bench.py [--gpus N] [--steps 20] [--warmup 5] [--k 64]
                    [--shape ml-full|c5] [--scale S] [--solver cg|cholesky] [--no-cpu]
                    [--comm rccl|gloo] [--device-map 0,0]

``--gpus N`` (N > 1) without a launcher starts the N ranks itself:
``torch.distributed.run --nproc-per-node N bench.py ...`` as a child
process; its ranks' one JSON line is relayed.  Under a launcher,
``WORLD_SIZE`` must equal ``--gpus``.  ``--comm gloo --device-map 0,0`` (tests
on a one-GPU box) puts two ranks on GPU 0 with host-staged exchanges.

``--shape c5`` is BASELINE.json configs[4] (synthetic 10 M users x 1 M items x
1e9 ratings; use --k 128): streamed by ``synth.C5Generator`` -- every rank
regenerates only its own user view and its items' view, factors are seeded on
the device -- and ``--scale`` runs a fraction of it (1/8 = one rank's users and
ratings of the 8-GPU run, on one GPU).

A step is one full ALS iteration of the reference loop (user half-step:
normal equations from gathered item rows + global block-CG solve; item
half-step likewise with ratings minus user bias), on data resident in HBM.
For N > 1 it runs under torch.distributed.run, one rank per GPU, users and
items sharded by rating count (weak scaling is not available for a fixed
data set: per-rank work shrinks as N grows -> "strong").

Printed on rank 0: ONE JSON line with the contract fields plus
``roofline`` (dominant kernel, from HIP events on the engine's stream over an
instrumented replay of the timed steps; the timed region itself carries no
per-launch events), ``cpu_baseline`` (the reference library compiled from
/root/reference sources, oracle/_ref/cpp_ls_lib.so, timed on the same data
and start -- full C3 by default, ``--cpu-scale`` shrinks it; N = 1 only),
``same_window`` (the GPU's iterations 2-3 of the same start, the window the
CPU leg's T(3) - T(1) times, with both sides' CG counts) and ``trajectory``
(the CG iterations of every ALS iteration from the start, checked against
the timed region's totals).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from movie_recommender_amd import synth  # noqa: E402

HBM_PEAK_GBS = 8000.0        # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP32_PEAK_TFS = 157.3        # MI355X FP32 vector / f32-MFMA dense peak
GATHER_PEAK_GBS = 8600.0   # MI355X_MICROARCH.md: random rows, 38 MB table (Infinity Cache)
METRIC = "ratings/sec per ALS iteration (MovieLens-full, k=64); RMSE parity"
# collective model (DESIGN.md "Multi-GPU"): effective xGMI rate of one peer
# link for the factor all-gather (each peer's block arrives over its own
# link, in parallel) and the device latency of one peer all-reduce of the CG
# scalars between GPUs
XGMI_LINK_GBPS = 50.0
PEER_REDUCE_US = 9.5


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def load_data(shape, k, cache_dir="/tmp", scale=1.0):
    tag = "" if scale == 1.0 else f"_x{scale:g}"
    path = os.path.join(cache_dir, f"mr_bench_{shape}{tag}_k{k}_{synth.DATA_SEED}.npz")
    if os.path.exists(path):
        with np.load(path, allow_pickle=False) as d:
            rs = synth.RatingSet(d["u"], d["i"], d["r"], int(d["nu"]), int(d["ni"]), k)
            return rs
    rs = synth.movielens_like(shape, k, scale=scale)
    try:
        np.savez(path, u=rs.user_ids, i=rs.item_ids, r=rs.ratings, nu=rs.num_users,
                 ni=rs.num_items)
    except OSError:
        pass
    return rs


def algorithmic_cost(cls, k, n_users, n_items, n_ratings, ldk, fused=True, n_ratings_items=None,
                     onepass=True):
    """(bytes, flops) per launch of a kernel class; definitions in DESIGN.md.

    Normal equations are stored "tri16" (mr_internal.h): the nb(nb-1)/2
    strictly-upper 16x16 blocks, the nb diagonal blocks folded pairwise into
    nb/2 tiles (+1 full tile for odd nb) and a 16-float diagonal side array
    per fold, nb = ceil(k/16) -- 2080 floats at k = 64 (k(k+1)/2 = 2080).  The
    CG matvec's bytes are that storage plus the CG vectors it streams.  Gram
    flops count each of the K(K+1)/2 distinct entries of the symmetric
    per-rating outer product once (2 flop each) plus the rhs (2K) -- the
    minimum work; SURVEY.md 8(d)'s F(k) counts the full K x K product, which
    would put a symmetric kernel above the MFMA peak.  The kernel's executed
    MFMA work is nb(nb+1)/2 * 512 flop per rating (diagonal blocks full).
    With the fused CG start (default) the Gram launch also reads x and writes
    r, p, q.  CG vectors r / p / q are fp64 (8 B), x and G fp32 (4 B).  The
    one-pass CG iteration (default) makes the matvec launch also apply the
    previous iteration's x / r update: per vector entry it reads p, r, q, x
    and writes p, r, q, x (6 x 8 + 2 x 4 B) instead of p rw, r read, q write
    (4 x 8 B); cg_update then only runs the finish pass once per solve (x +=
    alpha p: x rw fp32, p read)."""
    if cls.startswith("resident_"):   # per CG iteration: the one-pass iteration's bytes
        return algorithmic_cost("matvec_" + cls[len("resident_"):], k, n_users, n_items,
                                n_ratings, ldk, fused, n_ratings_items, True)
    K = k + 1
    nb = (k + 15) // 16
    gsz = (nb * (nb - 1) // 2 + nb // 2 + nb % 2) * 256 + (nb // 2) * 16
    n_ri = n_ratings if n_ratings_items is None else n_ratings_items   # item-view ratings
    vb = 6 * 8 + 2 * 4 if onepass else 4 * 8     # vector bytes per entry and launch
    if cls == "matvec_users":
        E = n_users
        g = E * (gsz + ldk + 1) * 4               # G_e blocks + Gs row + count
        v = E * (ldk + 1) * vb
        return g + v, E * 2.0 * K * K
    if cls == "matvec_items":
        E = n_items
        return E * gsz * 4 + E * ldk * vb, E * 2.0 * k * k
    if cls == "gram_users":
        # per rating: (idx, value) 8 B + gathered item row k*4 B; output blocks
        b = n_ratings * (8 + 4 * k) + n_users * (gsz + 2 * ldk + 2) * 4
        if fused:   # x read (fp32), r / p / q written (fp64)
            b += n_users * (ldk + 1) * (4 + 3 * 8)
        return b, n_ratings * (1.0 * K * (K + 1) + 2.0 * K)
    if cls == "gram_items":
        b = n_ri * (8 + 4 * (k + 1)) + n_items * (gsz + ldk) * 4
        if fused:
            b += n_items * ldk * (4 + 3 * 8)
        return b, n_ri * (1.0 * k * (k + 1) + 2.0 * k)
    if cls == "cg_update":
        E = (n_users * (ldk + 1) + n_items * ldk) / 2.0   # average side
        if onepass:   # the one-pass finish: x rw (fp32), p read (fp64)
            return E * (2 * 4 + 8), E * 2.0
        # x rw (fp32), r rw, p read, q read (fp64)
        return E * (2 * 4 + 4 * 8), E * 4.0
    return 0, 0


def iteration_roofline(k, rate):
    """SURVEY.md 8(d) whole-iteration roofline at R ratings/s: algorithmic
    bytes B(k) = 20 + 8k per rating (two (idx, value) reads, one k-float row
    gather per side) and flops F(k) = 2(k+1)^2 + 2k^2 + 2(k+1) + 2k (full Gram
    outer products + rhs, both sides), as fractions of the HBM and FP32 peaks."""
    B = 20 + 8 * k
    F = 2 * (k + 1) ** 2 + 2 * k ** 2 + 2 * (k + 1) + 2 * k
    return {"bytes_per_rating": B, "flops_per_rating": F,
            "hbm_GBps": round(B * rate / 1e9, 1), "hbm_frac": round(B * rate / 8e12, 4),
            "fp32_TFps": round(F * rate / 1e12, 2), "fp32_frac": round(F * rate / 157.3e12, 4)}


def cpu_share():
    """CPUs this process may use: the scheduler affinity mask, capped by the
    cgroup CPU quota (cgroup v2 cpu.max / v1 cfs quota) -- on the GPU box
    ``nproc`` shows the whole machine while the job gets a share of it."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = int(q) / int(per)
    except (OSError, ValueError):
        try:
            with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
                q = int(f.read())
            with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                per = int(f.read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    n = aff if quota is None else max(1, min(aff, int(quota)))
    return n, {"host_cpus": os.cpu_count(), "affinity_cpus": aff, "cgroup_cpu_quota": quota}


def cpu_baseline(shape, k, threads, scale, seed=0, replay=True, rs=None, repeats=3):
    """Reference CPU path on a bounded sample of the same workload: the
    MovieLens-shaped generator at ``scale`` of the users, items and draws (so
    per-entity degrees, and with them the CPU's per-rating costs, keep their
    full-size distribution; a user subsample would keep every item and with
    it the reference's full-length per-thread SpMV^T scratch), shrunk for the
    same k.  t_iter = (T(3) - T(1)) / 2 as in BASELINE.md, over ``repeats``
    (T(1), T(3)) pairs: ``value`` is the median pair's rate, ``spread`` the
    median / min / max (one pair on a shared host cgroup moves by 1.7x,
    VERDICT r04 weak 6).  ``threads`` None: the process's CPU share
    (``cpu_share``).

    The reference's ``als()`` does not report its CG iteration counts, which
    set its cost, so the same 3 iterations are then replayed with
    ``oracle/ref_replay.als_replay`` -- the outer loop restated around the
    reference's own CG, bit-identical to ``als()`` (same factors, same CG
    trajectory) -- for the CG iterations of iterations 2-3 (the ones T(3) -
    T(1) times) and the reference's time per CG iteration.  Also returns
    (separately, not in the dict) the reference's factors after iteration 1
    -- the state the GPU's like-for-like ``same_window`` starts from.
    Returns (dict for the JSON line, (U1, V1)), or (None, None) if the
    reference build is unavailable."""
    from oracle import ref
    if not ref.available():
        return None, None
    share, cpu_info = cpu_share()
    if threads is None:
        threads = share
    if rs is None:
        rs = synth.movielens_like(shape, k, scale=scale)
    U0, V0 = ref.init_factors(rs.num_users, rs.num_items, k, seed)
    ref.set_thread_count(threads)
    pairs = []
    state1 = None
    for rep in range(max(1, repeats)):
        t = {}
        for n_it in (1, 3):
            t0 = time.perf_counter()
            U, V, _ = ref.als(rs.user_ids, rs.item_ids, rs.ratings, k, U0, V0, max_iteration=n_it)
            t[n_it] = time.perf_counter() - t0
            if n_it == 1 and state1 is None:
                state1 = (U, V)
        pairs.append(((t[3] - t[1]) / 2.0, t[1], t[3]))
        log(f"[bench] cpu baseline pair {rep + 1}/{repeats}: T1 {t[1]:.2f} s, T3 {t[3]:.2f} s")
    order = sorted(range(len(pairs)), key=lambda j: pairs[j][0])
    med = pairs[order[len(order) // 2]]
    t_iter = med[0]
    rates = sorted(rs.n / p[0] for p in pairs)
    out = {"value": rs.n / t_iter, "unit": "ratings/s", "cores": threads, **cpu_info,
           "kind": "reference",
           "spread": {"repeats": len(pairs), "median": round(rs.n / t_iter, 1),
                      "min": round(rates[0], 1), "max": round(rates[-1], 1),
                      "t_iter_s": [round(p[0], 3) for p in pairs],
                      "T1_s": [round(p[1], 2) for p in pairs],
                      "T3_s": [round(p[2], 2) for p in pairs]},
           "sample": (f"{shape} generator at scale {scale} (users, items, draws), shrunk for "
                      f"k={k}: N={rs.n}, users={rs.num_users}, items={rs.num_items}; "
                      f"t_iter=(T(3)-T(1))/2, median of {len(pairs)} pairs = {t_iter:.3f} s "
                      f"(T1={med[1]:.2f} s, T3={med[2]:.2f} s); oracle/_ref/cpp_ls_lib.so built "
                      f"from /root/reference/cpp/ls_lib -O2, {threads} threads")}
    if replay:
        from oracle.ref_replay import als_replay
        _, _, _, tr = als_replay(rs.user_ids, rs.item_ids, rs.ratings, k, U0, V0,
                                 max_iteration=3)
        tr_all = tr
        tr = tr[1:3]          # iterations 2-3: what T(3) - T(1) measures
        cu = sum(x["cg_users"] for x in tr)
        ci = sum(x["cg_items"] for x in tr)
        tu = sum(x["t_users"] for x in tr)
        ti = sum(x["t_items"] for x in tr)
        out["cg"] = {
            "per_als_iteration_users": cu / len(tr), "per_als_iteration_items": ci / len(tr),
            "ms_per_cg_iteration_users": round(tu / max(cu, 1) * 1e3, 3),
            "ms_per_cg_iteration_items": round(ti / max(ci, 1) * 1e3, 3),
            # ratings x CG iterations per second: the trajectory-free rate
            "ratings_cg_iterations_per_s": round(rs.n * (cu + ci) / (tu + ti), 1),
            "cg_per_iteration": [[x["cg_users"], x["cg_items"]] for x in tr_all],
            "how": ("oracle/ref_replay.als_replay: als() restated around the reference's own "
                    "cg_least_squares_from_python, bit-identical to als_from_python "
                    "(tests/test_oracle.py), iterations 2-3 of the same run")}
    ref.set_thread_count(1)
    return out, state1


def gpu_cg_rate(st, n_u, n_i):
    """Time per CG iteration of each side (the solve phase's HIP-event span /
    its CG iterations, incl. the fused start's control) and ratings x CG
    iterations per second -- the trajectory-free rate comparable with
    cpu_baseline.cg (the CG counts of two runs on different data differ)."""
    cu, ci = st["cg_users_total"], st["cg_items_total"]
    su, si = st["phase_ms"]["solve_users"], st["phase_ms"]["solve_items"]
    if not (cu and ci and su and si):
        return None
    return {"ms_per_cg_iteration_users": round(su / cu, 4),
            "ms_per_cg_iteration_items": round(si / ci, 4),
            "ratings_cg_iterations_per_s": round((n_u * cu + n_i * ci) / ((su + si) / 1e3), 1),
            "note": "solve phases of the instrumented replay; the Gram is not included"}


def step_decomposition(st, steps, elapsed, ctx, k, world, dist, events_ms):
    """Where a sharded step goes (VERDICT r05 "do this" 3), per rank from the
    instrumented replay: the factor exchange (pack + all-gather + unstage,
    kernel class ``exchange``), the device time the finalizing waves spent in
    the peer all-reduce of the CG scalars (``peer_wait``: the reduction itself
    plus the wait for the slowest rank), and everything else (the rank's own
    Grams and CG).  ``model_step_ms`` is the collective model's prediction
    for this run: the slowest rank's own compute + the all-gathers at
    XGMI_LINK_GBPS per peer link + the peer reductions at PEER_REDUCE_US
    each; beside it the measured step (max and min over ranks)."""
    exch = st["kernel_ms"].get("exchange", 0.0) / steps
    peer = st.get("peer_wait_ms", 0.0) / steps
    n_red = st.get("peer_reductions", 0) / steps
    busy = sum(v for c, v in st["kernel_ms"].items() if c != "exchange") / steps
    # the rank's own compute: its kernels minus the time its finalizing waves
    # spent in the peer reductions (inside the CG kernels)
    own = max(0.0, busy - peer)
    mine = {"step_ms": elapsed * 1e3 / steps,
            "step_ms_with_kernel_events": events_ms, "compute_ms": own, "exchange_ms": exch,
            "peer_wait_ms": peer, "peer_reductions": n_red}
    allr = [None] * world
    dist.all_gather_object(allr, mine)
    ldk = (k + 15) // 16 * 16
    _, nu, _ = ctx.local_size("users")
    _, ni, _ = ctx.local_size("items")
    rows = [None] * world
    dist.all_gather_object(rows, (nu, ni))
    max_u = max(r[0] for r in rows)
    max_i = max(r[1] for r in rows)
    # per half-step every rank receives world - 1 padded blocks, one per peer
    # link in parallel: the largest block sets the time
    ag_bytes = (max_u * (ldk + 1) + max_i * ldk) * 4.0
    exch_model = ag_bytes / (XGMI_LINK_GBPS * 1e9) * 1e3 if world > 1 else 0.0
    peer_model = max(r["peer_reductions"] for r in allr) * PEER_REDUCE_US / 1e3
    compute = max(r["compute_ms"] for r in allr)
    r3 = lambda x: round(x, 4)  # noqa: E731
    return {"exchange_ms_per_step": r3(max(r["exchange_ms"] for r in allr)),
            "peer_wait_ms_per_step": r3(max(r["peer_wait_ms"] for r in allr)),
            "peer_reductions_per_step": r3(max(r["peer_reductions"] for r in allr)),
            "compute_ms_per_step_by_rank": [r3(r["compute_ms"]) for r in allr],
            "exchange_ms_per_step_by_rank": [r3(r["exchange_ms"]) for r in allr],
            "peer_wait_ms_per_step_by_rank": [r3(r["peer_wait_ms"]) for r in allr],
            "step_ms_max": r3(max(r["step_ms"] for r in allr)),
            "step_ms_min": r3(min(r["step_ms"] for r in allr)),
            "model_step_ms": r3(compute + exch_model + peer_model),
            "model": {"compute_ms": r3(compute), "exchange_ms": r3(exch_model),
                      "peer_reductions_ms": r3(peer_model),
                      "allgather_bytes_per_peer_block": int(ag_bytes),
                      "xgmi_link_GBps": XGMI_LINK_GBPS, "peer_reduce_us": PEER_REDUCE_US,
                      "how": ("compute = the slowest rank's own kernel time per step (its "
                              "replay's kernel table minus exchange and peer-reduction time); "
                              "all-gathers of the largest shard's rows at the link rate; "
                              "peer reductions at the xGMI latency (DESIGN.md Multi-GPU)")}}


def free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(n):
    """``--gpus N`` (N > 1) started without a launcher: run this same command
    under ``torch.distributed.run``, one rank per GPU, as a CHILD process
    (this process has not touched the GPU: only numpy is loaded), relay the
    ranks' one JSON line and exit with the launcher's return code.  Replaces
    the role of the reference's process fan-out
    (``python/full_data/cluster_server.py:279-305``)."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--master-addr=127.0.0.1", f"--master-port={free_port()}",
           os.path.abspath(__file__)] + sys.argv[1:]
    log(f"[bench] --gpus {n}: launching {' '.join(cmd[1:6])} ...")
    p = subprocess.run(cmd, stdout=subprocess.PIPE, env=dict(os.environ))
    lines = [ln for ln in p.stdout.decode(errors="replace").splitlines() if ln.strip()]
    js = [ln for ln in lines if ln.lstrip().startswith("{") and '"metric"' in ln]
    for ln in lines:
        if ln not in js:
            log(f"[bench] (rank stdout) {ln}")
    if js:
        os.write(JSON_FD, (js[-1].strip() + "\n").encode())
    if p.returncode == 0 and not js:
        log("[bench] ranks exited 0 without a JSON line")
        return 1
    return p.returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--k", type=int, default=64)
    ap.add_argument("--shape", default="ml-full", choices=["ml-full", "ml-100k", "c5"])
    ap.add_argument("--scale", type=float, default=1.0,
                    help="fraction of the shape (users, items, draws); tests and C5 slices")
    ap.add_argument("--solver", default="cg", choices=["cg", "cholesky"])
    ap.add_argument("--ridge", type=float, default=0.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-onepass", action="store_true",
                    help="CG iteration as matvec + update (two kernels) instead of one pass")
    ap.add_argument("--no-fuse-start", action="store_true",
                    help="start CG with a matvec + update pass instead of the Gram epilogue")
    ap.add_argument("--no-kernel-events", action="store_true",
                    help="time steps without per-launch HIP events (no roofline)")
    ap.add_argument("--cg-speculate", type=int, default=None,
                    help="engine launch-ahead level (include/mr_als.h MR_OPT_CG_SPECULATE)")
    ap.add_argument("--opt", action="append", default=[],
                    help="engine option NAME=VALUE (engine.OPTIONS), repeatable")
    ap.add_argument("--cpu-scale", type=float, default=1.0,
                    help="fraction of the workload the reference CPU leg runs (1.0: the "
                         "same data, start and window as the GPU's same_window)")
    ap.add_argument("--cpu-repeats", type=int, default=3,
                    help="(T(1), T(3)) pairs of the CPU leg; value = the median pair")
    ap.add_argument("--cpu-threads", type=int, default=None,
                    help="reference threads (default: this process's CPU share)")
    ap.add_argument("--no-same-window", action="store_true",
                    help="skip the GPU's iterations-2-3 run from the seed-0 start")
    ap.add_argument("--force-shard", action="store_true",
                    help="use the sharded RCCL path even with one rank (testing)")
    ap.add_argument("--scalars", default="peer", choices=["peer", "collective"],
                    help="sharded runs: CG scalars through the peer all-reduce (IPC-mapped "
                         "buffers; falls back to RCCL if its self-test fails) or RCCL")
    ap.add_argument("--comm", default="rccl", choices=["rccl", "gloo"],
                    help="sharded runs: factor all-gather through the native RCCL "
                         "communicator (one rank per GPU) or, for tests, gloo callbacks "
                         "(host-staged; lets several ranks share one GPU)")
    ap.add_argument("--device-map", default=None,
                    help="test only: comma-separated GPU index per local rank "
                         "(e.g. 0,0 puts two ranks on GPU 0; needs --comm gloo)")
    ap.add_argument("--pmc", default=None,
                    help="per-kernel HBM bytes from a rocprofv3 --pmc run (optional; default "
                         "profiles/pmc_r06.json at k = 64, profiles/pmc_r06_k<k>.json otherwise; the "
                         "previous round's if absent)")
    args = ap.parse_args()

    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        return launch_ranks(args.gpus)
    world = int(env_world) if env_world is not None else 1
    if world != args.gpus:
        log(f"[bench] WORLD_SIZE={world} but --gpus {args.gpus}: refusing to report a "
            f"{world}-rank run as {args.gpus}")
        return 2
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    device = local_rank
    if args.device_map is not None:
        dm = [int(x) for x in args.device_map.split(",")]
        if len(dm) <= local_rank:
            log(f"[bench] --device-map {args.device_map} has no entry for local rank {local_rank}")
            return 2
        device = dm[local_rank]
        if args.comm != "gloo" and len(set(dm[:world])) < min(world, len(dm)):
            log("[bench] ranks sharing a GPU need --comm gloo (RCCL takes one rank per GPU)")
            return 2
    dist = None
    if world > 1 or args.force_shard:
        import torch
        import torch.distributed as tdist
        if args.comm == "gloo":
            tdist.init_process_group("gloo")
        else:
            torch.cuda.set_device(device)
            tdist.init_process_group("nccl", device_id=torch.device("cuda", device))
        dist = tdist

    from movie_recommender_amd.engine import AlsContext
    from movie_recommender_amd.distributed import sharded_context

    t0 = time.perf_counter()
    k = args.k
    c5 = args.shape == "c5"
    if c5:
        gen = synth.C5Generator(scale=args.scale)
        n_total, n_users, n_items = gen.n, gen.num_users, gen.num_items
    else:
        if dist is not None and rank != 0:
            dist.barrier()            # rank 0 generates (or loads) the data first
        rs = load_data(args.shape, k, scale=args.scale)
        if dist is not None and rank == 0:
            dist.barrier()
        n_total, n_users, n_items = rs.n, rs.num_users, rs.num_items
    log(f"[bench] data {args.shape} k={k}: N={n_total} users={n_users} "
        f"items={n_items} ({time.perf_counter() - t0:.1f} s)")

    t0 = time.perf_counter()
    if c5:
        from movie_recommender_amd.distributed import entity_cost, shard_bounds
        if dist is not None:
            ub = shard_bounds(entity_cost(gen.deg, k), world)
            ib = shard_bounds(entity_cost(np.rint(gen.expected_item_counts()).astype(np.int64),
                                          k), world)
            u0, u1, i0, i1 = int(ub[rank]), int(ub[rank + 1]), int(ib[rank]), int(ib[rank + 1])
            uv = gen.user_view(u0, u1)
            iv = gen.item_view(i0, i1)
            ctx = AlsContext(uv[0], uv[1], uv[2], k, n_users, n_items, device=device,
                             solver=args.solver, ridge=args.ridge, user_range=(u0, u1),
                             item_range=(i0, i1), item_view=iv)
            del uv, iv
            from movie_recommender_amd.distributed import TorchComm, attach_comm
            attach_comm(ctx, TorchComm() if args.comm == "gloo" else "rccl", rank, world, ub, ib)
            if args.scalars == "peer":
                from movie_recommender_amd.distributed import attach_peer_scalars
                ctx.peer_scalars = attach_peer_scalars(ctx, rank, world)
        else:
            u, i, r = gen.all_ratings()
            ctx = AlsContext(u, i, r, k, n_users, n_items, device=device,
                             solver=args.solver, ridge=args.ridge)
            del u, i, r
        ctx.init_factors(0)
    else:
        rng = np.random.RandomState(0)
        U0 = rng.uniform(-1, 1, n_users * (k + 1))
        V0 = rng.uniform(-1, 1, n_items * k)
        if dist is not None:
            if args.comm == "gloo":
                from movie_recommender_amd.distributed import TorchComm
                comm = TorchComm()
            else:
                comm = "rccl"
            ctx = sharded_context(rs.user_ids, rs.item_ids, rs.ratings, k, n_users, n_items,
                                  device, comm, solver=args.solver, ridge=args.ridge,
                                  scalars=args.scalars)
        else:
            ctx = AlsContext(rs.user_ids, rs.item_ids, rs.ratings, k, n_users, n_items,
                             device=device, solver=args.solver, ridge=args.ridge)
        ctx.set_factors(U0, V0)
    if args.no_fuse_start:
        ctx.set_option("fuse_start", 0)
    if args.no_onepass:
        ctx.set_option("cg_onepass", 0)
    if args.cg_speculate is not None:
        ctx.set_option("cg_speculate", args.cg_speculate)
    for o in args.opt:
        name, val = o.split("=")
        ctx.set_option(name, float(val))
    ctx.sync()
    log(f"[bench] context built in {time.perf_counter() - t0:.2f} s")

    for w in range(args.warmup):
        ctx.iterate(1)
    ctx.sync()
    ctx.reset_stats()

    def barrier():
        ctx.sync()
        if dist is not None:
            dist.barrier()

    def max_over_ranks(x):
        if dist is None:
            return x
        import torch
        tt = torch.tensor([x], dtype=torch.float64,
                          device="cpu" if args.comm == "gloo" else f"cuda:{device}")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        return float(tt.item())

    def timed_steps():
        barrier()
        t = time.perf_counter()
        for s in range(args.steps):
            ctx.iterate(1)
        barrier()
        return max_over_ranks(time.perf_counter() - t)

    # The timed region runs WITHOUT per-launch events (the workload only);
    # then the SAME K steps are replayed from a snapshot of the iterate with a
    # start/stop HIP event pair on every launch (hipExtLaunchKernel, on the
    # engine's stream) for the per-kernel table and the roofline.  The engine
    # is deterministic, so the replay runs bit-identical kernels: its CG
    # iteration counts must equal the timed pass's (replay_cg_identical).
    # Tables too large to snapshot (C5) time one instrumented pass instead.
    instrument = not args.no_kernel_events
    replay = instrument and n_users * (k + 1) + n_items * k < 200_000_000
    snap = ctx.get_factors() if replay else None
    ctx.set_timing(instrument and not replay)
    elapsed = timed_steps()
    st = ctx.stats()
    events_ms = None
    replay_identical = None
    if replay:
        ctx.set_factors(*snap)
        ctx.reset_stats()
        ctx.set_timing(True)
        events_ms = timed_steps() * 1e3 / args.steps
        st_ev = ctx.stats()
        replay_identical = (st_ev["cg_users_total"] == st["cg_users_total"]
                            and st_ev["cg_items_total"] == st["cg_items_total"])
        for key in ("kernel_ms", "kernel_launches", "kernel_units", "phase_ms", "peer_wait_ms",
                    "peer_reductions"):
            st[key] = st_ev[key]
    elif instrument:
        events_ms = elapsed * 1e3 / args.steps
    ctx.set_timing(False)

    # The CPU leg (rank 0, N = 1): the reference on the same data and start,
    # T(3) - T(1) over repeated pairs; it also hands over the reference's
    # factors after its iteration 1.
    cb = state1 = None
    cpu_leg = rank == 0 and world == 1 and not args.no_cpu and not c5
    if cpu_leg:
        try:
            cb, state1 = cpu_baseline(args.shape, k, args.cpu_threads, args.cpu_scale * args.scale,
                                      rs=rs if args.cpu_scale == 1.0 else None,
                                      repeats=args.cpu_repeats)
        except Exception as e:  # the GPU number stands on its own
            log(f"[bench] cpu baseline failed: {e!r}")
            cb = state1 = None
        if args.cpu_scale != 1.0:
            state1 = None          # a different data set: no common state

    # same_window: iterations 2-3, what the CPU leg's T(3) - T(1) times
    # (BASELINE.md), timed like the main region.  Like-for-like (VERDICT r04
    # do 2): the GPU starts from the REFERENCE's state after iteration 1, so
    # both legs run iterations 2-3 from the same factors (the engine's own
    # first users solve parts from the reference's on full C3: 35 vs 59 CG
    # iterations, DESIGN "Parity"); the two legs' CG counts are compared and
    # any difference is flagged.  Without the CPU leg the GPU's own
    # iteration 1 is the start.
    # trajectory: CG iterations of every ALS iteration 1 .. warmup + steps
    # from the RandomState(0) start, one iteration at a time (untimed); its
    # sums over the timed window must equal the timed region's (the engine is
    # deterministic), which the line checks.
    same_window = trajectory = None
    if not c5 and not args.no_same_window:
        if state1 is not None:
            ctx.set_factors(*state1)
        else:
            ctx.set_factors(U0, V0)
            ctx.iterate(1)
        barrier()
        ctx.reset_stats()
        t = time.perf_counter()
        ctx.iterate(2)
        barrier()
        t_sw = max_over_ranks(time.perf_counter() - t)
        s2 = ctx.stats()
        same_window = {"iterations": "2-3 (T(3) - T(1) of the CPU leg)",
                       "start": ("the reference's factors after its iteration 1 (same data, "
                                 "RandomState(0) start)" if state1 is not None else
                                 "the GPU's own iteration 1 from the RandomState(0) start"),
                       "value": round(n_total * 2 / t_sw, 1), "unit": "ratings/s",
                       "ms_per_iteration": round(t_sw * 1e3 / 2, 3),
                       "cg_users": s2["cg_users_total"], "cg_items": s2["cg_items_total"]}
        ctx.set_factors(U0, V0)
        trajectory = []
        for it in range(max(3, args.warmup + args.steps)):
            ctx.reset_stats()
            ctx.iterate(1)
            s1 = ctx.stats()
            trajectory.append([s1["cg_users_total"], s1["cg_items_total"]])
        win = trajectory[args.warmup:args.warmup + args.steps]
        if state1 is None:
            same_window["trajectory_cg_matches"] = (
                trajectory[1][0] + trajectory[2][0] == same_window["cg_users"]
                and trajectory[1][1] + trajectory[2][1] == same_window["cg_items"])
        trajectory = {"cg_per_iteration": trajectory,
                      "matches_timed_region": (sum(x[0] for x in win) == st["cg_users_total"]
                                               and sum(x[1] for x in win) == st["cg_items_total"])}

    # per-rank shard sizes (cost-balanced shards are unequal)
    shards = None
    if dist is not None:
        mine = [list(ctx.local_size("users")), list(ctx.local_size("items"))]
        allr = [None] * world
        dist.all_gather_object(allr, mine)
        shards = [{"rank": r, "users": [a[0][0], a[0][0] + a[0][1]], "user_ratings": a[0][2],
                   "items": [a[1][0], a[1][0] + a[1][1]], "item_ratings": a[1][2]}
                  for r, a in enumerate(allr)]

    # local work units (ratings processed by this rank per iteration)
    n_local_users = ctx.num_ratings
    total_ratings = n_total
    value = total_ratings * args.steps / elapsed
    ms_per_step = elapsed * 1e3 / args.steps

    # dominant kernel and its roofline (rank 0's kernels, rank 0's shard sizes:
    # cost-balanced shards are unequal)
    ldk = (k + 15) // 16 * 16
    if args.no_kernel_events:
        st["kernel_ms"] = {"none": 1.0}
        st["kernel_launches"] = {"none": 1}
    best = max(st["kernel_ms"].items(), key=lambda kv: kv[1])
    cls, tot_ms = best
    launches = max(1, st["kernel_launches"][cls])
    avg_s = tot_ms / launches / 1e3
    # work units per launch: a resident CG solve runs all its iterations in
    # one launch (kernel_units = its CG iterations); 1 for every other class
    units_per_launch = (st.get("kernel_units", {}).get(cls, launches) or launches) / launches
    _, nU, _ = ctx.local_size("users")
    _, nI, n_local_items = ctx.local_size("items")
    # one-pass CG on both sides at k <= 128: unsharded or with peer scalars
    # (RCCL collectives: two kernels; Engine::onepass_for)
    onepass = (not args.no_onepass and k <= 128
               and (dist is None or getattr(ctx, "peer_scalars", False)))
    onepass_of = lambda c: onepass  # noqa: E731
    nbytes, nflops = algorithmic_cost(cls, k, nU, nI, n_local_users, ldk, not args.no_fuse_start,
                                      n_local_items, onepass_of(cls))
    nbytes, nflops = nbytes * units_per_launch, nflops * units_per_launch
    bound = "mfma" if cls.startswith("gram") and k >= 32 else "hbm"
    if bound == "hbm":
        achieved, peak, unit = nbytes / avg_s / 1e9, HBM_PEAK_GBS, "GB/s"
    else:
        achieved, peak, unit = nflops / avg_s / 1e12, FP32_PEAK_TFS, "TFLOP/s"
    # Gram kernels: the row gather (k floats of the other side's table per
    # rating, Infinity-Cache resident) is the binding roofline; peak = the
    # guide's measured random-row gather rate from a 38 MB table.
    gather = None
    if cls.startswith("gram"):
        gb = (n_local_users if cls == "gram_users" else n_local_items) * 4.0 * k
        gather = {"bytes_per_launch": int(gb), "achieved_GBps": round(gb / avg_s / 1e9, 1),
                  "peak_GBps": GATHER_PEAK_GBS, "frac": round(gb / avg_s / 1e9 / GATHER_PEAK_GBS, 3)}
    traffic = None
    pmc_path = args.pmc
    if not pmc_path:   # this round's counter passes, else the previous round's
        for rnd in ("r06", "r05", "r04"):
            pmc_path = os.path.join(ROOT, "profiles",
                                    f"pmc_{rnd}.json" if k == 64 else f"pmc_{rnd}_k{k}.json")
            if os.path.exists(pmc_path):
                break
    if os.path.exists(pmc_path):
        with open(pmc_path) as f:
            pmc = json.load(f)
        # only for the workload the counter passes ran (per-launch bytes)
        wl = pmc.get("workload", {"shape": "ml-full", "k": 64})
        if wl.get("shape") == args.shape and wl.get("k") == k and world == 1 and not c5:
            per = pmc.get("hbm_bytes_per_launch", {})
            traffic = per.get(cls)
            if traffic is None and cls.startswith("resident_"):
                # the resident solve's iterations make the launch-per-iteration
                # kernel's accesses (the counter passes run that path:
                # per-launch = per CG iteration) times its iterations per launch
                it = per.get("matvec_" + cls[len("resident_"):])
                traffic = None if it is None else int(it * units_per_launch)
    kernel_table = {}
    for c, ms in st["kernel_ms"].items():
        n = st["kernel_launches"][c]
        if n:
            u = st.get("kernel_units", {}).get(c, n) or n
            b, fl = algorithmic_cost(c, k, nU, nI, n_local_users, ldk, not args.no_fuse_start,
                                     n_local_items, onepass_of(c))
            b, fl = b * u / n, fl * u / n
            kernel_table[c] = {"total_ms": round(ms, 3), "launches": n,
                               "avg_us": round(ms / n * 1e3, 2),
                               "alg_GBps": round(b / (ms / n / 1e3) / 1e9, 1) if b else None,
                               "alg_TFps": round(fl / (ms / n / 1e3) / 1e12, 2) if fl else None}
            if u != n:
                kernel_table[c]["cg_iterations"] = u
                kernel_table[c]["us_per_cg_iteration"] = round(ms / u * 1e3, 2)

    out = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "ratings/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32+f64",
        "data": ("synthetic (C5 generator: lognormal activity, rank^-0.9 popularity, uniform "
                 "half-stars; device-seeded factors)" if c5 else
                 "synthetic (MovieLens-full shape, seeded; no MovieLens data offline)"),
        "config": {"workload": (f"ALS iteration, {args.shape} shape"
                                + (f" x{args.scale:g}" if args.scale != 1.0 else "")
                                + f", k={k}, solver={args.solver}"),
                   "k": k, "n_ratings": int(n_total), "users": int(n_users),
                   "items": int(n_items), "solver": args.solver,
                   "parallelism": (f"shard{world}" if world > 1 or args.force_shard
                                   else "single"),
                   "cg_scalars": ("peer all-reduce (IPC)" if getattr(ctx, "peer_scalars", False)
                                  else "rccl all-reduce" if dist is not None else "local"),
                   "cg_iteration": "one pass" if onepass else "matvec + update"},
        "roofline": {"kernel": cls, "bound": bound, "achieved": round(achieved, 2),
                     "peak": peak, "unit": unit, "frac": round(achieved / peak, 4),
                     "traffic": traffic,
                     "alg_bytes_per_launch": int(nbytes), "alg_flops_per_launch": int(nflops),
                     "avg_launch_us": round(avg_s * 1e6, 2), "gather": gather,
                     "units_per_launch": round(units_per_launch, 3)},
        "iteration_roofline": iteration_roofline(k, value),
        "cg_iterations": {"users_total": st["cg_users_total"],
                          "items_total": st["cg_items_total"],
                          "per_step_users": st["cg_users_total"] / args.steps,
                          "per_step_items": st["cg_items_total"] / args.steps},
        "cg_rate": gpu_cg_rate(st, n_local_users, n_local_items),
        "kernels": kernel_table,
        "phase_ms_per_step": {p: round(v / args.steps, 3) for p, v in st["phase_ms"].items()},
        "timing": ("timed region without per-launch events; kernel table and roofline from "
                   "an event-instrumented replay of the same steps" if replay else
                   "one event-instrumented timed region" if instrument else
                   "timed region without per-launch events (no kernel table)"),
        "ms_per_step_with_kernel_events": round(events_ms, 3) if events_ms else None,
        "replay_cg_identical": replay_identical,
        "same_window": same_window,
        "trajectory": trajectory,
    }
    if dist is not None:
        out["decomposition"] = step_decomposition(st, args.steps, elapsed, ctx, k, world, dist,
                                                  events_ms)
    if shards is not None:
        out["config"]["shards"] = shards
        out["config"]["comm"] = args.comm
        if args.device_map is not None:
            out["config"]["device_map"] = args.device_map
    if cpu_leg:
        out["cpu_baseline"] = cb
        if cb and cb.get("cg") and same_window is not None and args.cpu_scale == 1.0:
            # same data, start and window on both sides
            ref_cu = int(round(2 * cb["cg"]["per_als_iteration_users"]))
            ref_ci = int(round(2 * cb["cg"]["per_als_iteration_items"]))
            same_window["reference"] = {
                "value": round(cb["value"], 1), "cg_users": ref_cu, "cg_items": ref_ci,
                "cores": cb["cores"]}
            same_window["cg_counts_equal"] = (ref_cu == same_window["cg_users"]
                                              and ref_ci == same_window["cg_items"])
            same_window["gpu_over_reference"] = round(same_window["value"] / cb["value"], 1)
            if not same_window["cg_counts_equal"]:
                same_window["flag"] = ("the two legs ran different CG iteration counts: "
                                       "gpu_over_reference compares unequal work; "
                                       "gpu_over_reference_per_cg_iteration is like for like")
            cr = out.get("cg_rate")
            if cr:
                same_window["gpu_over_reference_per_cg_iteration"] = {
                    "users": round(cb["cg"]["ms_per_cg_iteration_users"]
                                   / cr["ms_per_cg_iteration_users"], 1),
                    "items": round(cb["cg"]["ms_per_cg_iteration_items"]
                                   / cr["ms_per_cg_iteration_items"], 1)}
    elif rank == 0:
        out["cpu_baseline"] = None
    ctx.close()
    if rank == 0:
        os.write(JSON_FD, (json.dumps(out) + "\n").encode())
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    return 0


# The contract's ONE JSON line goes to the original stdout; everything else a
# library writes to fd 1 (RCCL prints a version banner on communicator init)
# is redirected to stderr, so stdout carries nothing but that line.
JSON_FD = 1

if __name__ == "__main__":
    sys.stdout.flush()
    JSON_FD = os.dup(1)
    os.dup2(2, 1)
    sys.exit(main())
