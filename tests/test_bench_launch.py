"""bench.py's multi-rank launch (VERDICT r03 "do this" 1): ``--gpus N``
without a launcher starts N ranks under torch.distributed.run as a child
process and relays their one JSON line; a rank count that differs from
``--gpus`` is refused.  On the one-GPU box the ranks share GPU 0 through the
test-only ``--device-map 0,0 --comm gloo``; the one-pass CG's exact sums make
the sharded run take the single-GPU trajectory, so the CG counts must be
equal (DESIGN.md "Order-independent CG sums")."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

BENCH = os.path.join(ROOT, "bench.py")
SMALL = ["--shape", "ml-full", "--scale", "0.125", "--k", "64", "--steps", "3", "--warmup", "2",
         "--no-cpu"]


def run_bench(args, timeout=600, env=None):
    r = subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True,
                       timeout=timeout, cwd=ROOT, env=dict(os.environ, **(env or {})))
    return r


def test_world_size_mismatch_is_refused():
    """A launcher world that differs from --gpus is an error, never a
    silently mislabelled line (CPU: refused before anything loads)."""
    r = run_bench(["--gpus", "1"], timeout=120, env={"WORLD_SIZE": "2"})
    assert r.returncode == 2 and r.stdout == "", (r.returncode, r.stdout)
    assert "refusing" in r.stderr
    r = run_bench(["--gpus", "4"], timeout=120, env={"WORLD_SIZE": "2", "RANK": "0",
                                                       "LOCAL_RANK": "0"})
    assert r.returncode == 2 and r.stdout == ""


@pytest.mark.gpu
def test_bench_gpus2_matches_gpus1(gpu):
    one = run_bench(["--gpus", "1"] + SMALL)
    assert one.returncode == 0, one.stderr[-3000:]
    two = run_bench(["--gpus", "2", "--comm", "gloo", "--device-map", "0,0"] + SMALL)
    assert two.returncode == 0, two.stderr[-3000:]
    lines1 = [ln for ln in one.stdout.splitlines() if ln.strip()]
    lines2 = [ln for ln in two.stdout.splitlines() if ln.strip()]
    assert len(lines1) == 1 and len(lines2) == 1, (one.stdout, two.stdout)
    a, b = json.loads(lines1[0]), json.loads(lines2[0])
    assert a["n_gpus"] == 1 and b["n_gpus"] == 2
    assert b["config"]["parallelism"] == "shard2"
    assert b["config"]["cg_scalars"].startswith("peer")
    sh = b["config"]["shards"]
    assert len(sh) == 2
    assert sh[0]["users"][0] == 0 and sh[0]["users"][1] == sh[1]["users"][0]
    assert sh[1]["users"][1] == a["config"]["users"] and sh[1]["items"][1] == a["config"]["items"]
    assert sh[0]["user_ratings"] + sh[1]["user_ratings"] == a["config"]["n_ratings"]
    assert sh[0]["item_ratings"] + sh[1]["item_ratings"] == a["config"]["n_ratings"]
    assert min(s["user_ratings"] for s in sh) > 0.3 * a["config"]["n_ratings"]
    # N-invariance at bench level: the same CG iterations in the window and
    # in every iteration of the trajectory
    assert a["cg_iterations"] == b["cg_iterations"], (a["cg_iterations"], b["cg_iterations"])
    assert a["trajectory"]["cg_per_iteration"] == b["trajectory"]["cg_per_iteration"]
    assert a["trajectory"]["matches_timed_region"] and b["trajectory"]["matches_timed_region"]
    assert a["same_window"]["cg_users"] == b["same_window"]["cg_users"]
    assert a["same_window"]["trajectory_cg_matches"]
    # the sharded line decomposes its step (VERDICT r05 "do this" 3)
    dc = b["decomposition"]
    assert dc["exchange_ms_per_step"] > 0 and dc["peer_wait_ms_per_step"] > 0
    assert dc["peer_reductions_per_step"] >= 2     # >= one per half-step's solve
    assert len(dc["compute_ms_per_step_by_rank"]) == 2
    assert min(dc["compute_ms_per_step_by_rank"]) > 0
    assert dc["step_ms_max"] >= dc["step_ms_min"] > 0
    assert abs(dc["step_ms_max"] - b["ms_per_step"]) <= 1e-3 * b["ms_per_step"] + 1e-3
    m = dc["model"]
    assert dc["model_step_ms"] == pytest.approx(m["compute_ms"] + m["exchange_ms"]
                                                + m["peer_reductions_ms"], abs=1e-3)
    assert "decomposition" not in a


@pytest.mark.gpu
def test_bench_forced_shard_world1_resident_peer(gpu):
    """One rank through the whole sharded path on its own GPU: RCCL
    communicator, the peer all-reduce (mapped onto its own buffer) and the
    resident CG solve together -- the combination an N-GPU run uses, which the
    shared-GPU layouts above cannot run (they switch the resident solve off).
    Same trajectory as the unsharded run, a decomposed line, and the peer
    reductions counted."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0", "MASTER_ADDR": "127.0.0.1",
           "MASTER_PORT": str(port)}
    one = run_bench(["--gpus", "1"] + SMALL)
    assert one.returncode == 0, one.stderr[-3000:]
    sh = run_bench(["--gpus", "1", "--force-shard"] + SMALL, env=env)
    assert sh.returncode == 0, sh.stderr[-3000:]
    a = json.loads([ln for ln in one.stdout.splitlines() if ln.strip()][0])
    b = json.loads([ln for ln in sh.stdout.splitlines() if ln.strip()][0])
    assert b["config"]["parallelism"] == "shard1"
    assert b["config"]["cg_scalars"].startswith("peer"), b["config"]["cg_scalars"]
    assert "resident_users" in b["kernels"] and "resident_items" in b["kernels"]
    assert a["cg_iterations"] == b["cg_iterations"]
    assert a["trajectory"]["cg_per_iteration"] == b["trajectory"]["cg_per_iteration"]
    dc = b["decomposition"]
    assert dc["peer_reductions_per_step"] >= 2 and dc["peer_wait_ms_per_step"] > 0
