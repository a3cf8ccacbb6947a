"""Sharded ALS: one process per GPU, users and movies partitioned by per-step cost.

Replaces the *role* of the reference's process fan-out
(``python/full_data/cluster_server.py`` / ``worker_server.py`` and the
multiprocessing pipes of ``movie_lens_data_proc.py``), which the reference
uses for evaluation, never for the ALS solve.  Here the solve itself shards:

* rank r owns users ``[ub[r], ub[r+1])`` and items ``[ib[r], ib[r+1])``;
  boundaries balance the per-step cost ``n_e + C(k)`` of each entity
  (``entity_cost``: the Gram's work is per rating, the CG's per entity);
* each rank builds its users' normal equations from a full replica of V and
  its items' from a full replica of U, so no rating crosses ranks;
* the reference's global CG scalars (``matrix.cpp:485, 497, 507``) are
  all-reduced (2 doubles per CG iteration) and the freshly solved factor
  shard is all-gathered after every half-step (RCCL: one ncclAllGather of
  equal padded shards).

The collectives are supplied through ``mr_comm`` callbacks backed by
``torch.distributed`` (``nccl`` = RCCL over xGMI on MI355X, or ``gloo``).
"""
import ctypes

import numpy as np

from . import _lib


# entities per term of the one-pass CG's order-independent sums (kernels.hip
# kXChunk): interior shard boundaries at multiples of it give every rank the
# single-GPU run's terms, so a sharded run reproduces its scalars bit for bit
SUM_CHUNK = 4


def shard_bounds(counts, world, align=SUM_CHUNK):
    """Contiguous id ranges with ~equal rating counts: ``world+1`` boundaries,
    the interior ones rounded to the nearest multiple of ``align``."""
    counts = np.asarray(counts, np.int64)
    n = len(counts)
    csum = np.concatenate([[0], np.cumsum(counts)])
    total = csum[-1]
    b = [0]
    for r in range(1, world):
        c = int(np.searchsorted(csum, total * r / world, side="left"))
        b.append(int(round(c / align)) * align)
    b.append(n)
    b = np.maximum.accumulate(np.minimum(np.array(b, np.int64), n))
    return b


def entity_cost(counts, k, cg_iterations=6):
    """Per-step cost of each entity in rating units: its ratings (the Gram
    gathers a 4k-byte row per rating) plus ``cg_iterations`` block-GEMV
    passes over its normal equations and fp64 CG vectors (4 gsize(k) + 40
    (ldk + 1) bytes each, the CG's cost is per entity, not per rating)."""
    counts = np.asarray(counts, np.int64)
    if k is None:
        return counts
    nb = (k + 15) // 16
    gsize = (nb * (nb - 1) // 2 + nb // 2 + nb % 2) * 256 + (nb // 2) * 16
    ldk = nb * 16
    c = int(round(cg_iterations * (4 * gsize + 40 * (ldk + 1)) / (4 * k + 8)))
    return counts + c


def shard_views(user_ids, item_ids, ratings, num_users, num_items, rank, world, k=None,
                bounds=None):
    """(user_range, item_range, user_view, item_view, ub, ib) for ``rank``;
    with ``k`` the boundaries balance ``entity_cost``, else rating counts;
    ``bounds=(ub, ib)`` imposes them (tests of uneven shards)."""
    if bounds is not None:
        ub, ib = (np.asarray(b, np.int64) for b in bounds)
        assert len(ub) == len(ib) == world + 1
        assert ub[0] == 0 and ub[-1] == num_users and ib[0] == 0 and ib[-1] == num_items
    else:
        uc = np.bincount(user_ids, minlength=num_users)
        ic = np.bincount(item_ids, minlength=num_items)
        ub = shard_bounds(entity_cost(uc, k), world)
        ib = shard_bounds(entity_cost(ic, k), world)
    u0, u1 = int(ub[rank]), int(ub[rank + 1])
    i0, i1 = int(ib[rank]), int(ib[rank + 1])
    su = (user_ids >= u0) & (user_ids < u1)
    si = (item_ids >= i0) & (item_ids < i1)
    uview = (user_ids[su], item_ids[su], ratings[su])
    iview = (user_ids[si], item_ids[si], ratings[si])
    return (u0, u1), (i0, i1), uview, iview, ub, ib


class TorchComm:
    """``mr_comm`` callbacks over an initialised ``torch.distributed`` group.

    Data is staged through host memory by the engine; with the ``nccl``
    backend the exchange itself runs as RCCL collectives on the rank's GPU.
    """

    def __init__(self, device=None):
        import torch
        import torch.distributed as dist
        self.torch = torch
        self.dist = dist
        self.rank = dist.get_rank()
        self.world = dist.get_world_size()
        self.backend = dist.get_backend()
        self.device = device if self.backend == "nccl" else "cpu"
        self._ar = _lib.ALLREDUCE_CB(self._allreduce)
        self._ag = _lib.ALLGATHER_CB(self._allgather)
        self.struct = _lib.MrComm(None, self.rank, self.world, self._ar, self._ag)
        self.errors = []

    def _allreduce(self, user, buf, count):
        try:
            a = np.ctypeslib.as_array(buf, shape=(count,))
            t = self.torch.from_numpy(a.copy()).to(self.device)
            self.dist.all_reduce(t)
            a[:] = t.cpu().numpy()
            return 0
        except Exception as e:  # pragma: no cover - surfaced by the engine
            self.errors.append(repr(e))
            return -1

    def _allgather(self, user, table, row_floats, row_begin, world):
        try:
            rb = np.ctypeslib.as_array(row_begin, shape=(world + 1,)).copy()
            rows = int(rb[-1])
            tab = np.ctypeslib.as_array(table, shape=(rows * row_floats,))
            counts = np.diff(rb)
            maxr = int(counts.max()) if len(counts) else 0
            mine = tab[rb[self.rank] * row_floats: rb[self.rank + 1] * row_floats]
            send = np.zeros(maxr * row_floats, np.float32)
            send[:len(mine)] = mine
            st = self.torch.from_numpy(send).to(self.device)
            outs = [self.torch.empty_like(st) for _ in range(world)]
            self.dist.all_gather(outs, st)
            for r in range(world):
                n = int(counts[r]) * row_floats
                tab[rb[r] * row_floats: rb[r] * row_floats + n] = outs[r].cpu().numpy()[:n]
            return 0
        except Exception as e:  # pragma: no cover
            self.errors.append(repr(e))
            return -1


def agree_rhs_path(ctx):
    """Every rank takes the same user-side Gram rhs path: the matrix-core
    rhs needs every weight exact in bf16, which each context checks on its
    own ratings (``mr_als_weights_bf16``); the ranks AND their flags so that
    no rank takes a path that rounds differently from the others'.
    Collective."""
    import torch
    import torch.distributed as dist
    L = _lib.lib()
    mine = _lib.check(L.mr_als_weights_bf16(ctx._h, -1), "mr_als_weights_bf16")
    flag = torch.tensor([mine], dtype=torch.int32)
    if dist.get_backend() == "nccl":
        flag = flag.cuda()
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    if int(flag.item()) == 0 and mine:
        _lib.check(L.mr_als_weights_bf16(ctx._h, 0), "mr_als_weights_bf16")
    return int(flag.item()) == 1


def attach_comm(ctx, comm, rank, world, user_begin, item_begin):
    """Attach this rank's factor all-gather transport: ``comm="rccl"`` (the
    native RCCL communicator) or a ``TorchComm`` (host-staged callbacks over
    any torch.distributed backend), then agree on the rhs path.
    Collective."""
    if comm == "rccl":
        attach_rccl(ctx, rank, world, user_begin, item_begin)
    else:
        ctx.set_comm(comm.struct, user_begin, item_begin)
        ctx._comm_owner = comm
    agree_rhs_path(ctx)


def attach_rccl(ctx, rank, world, user_begin, item_begin):
    """Give ``ctx`` a native RCCL communicator: rank 0 draws the unique id,
    ``torch.distributed`` (any backend) broadcasts its 128 bytes, then every
    rank builds the communicator inside the library (collective call)."""
    import torch.distributed as dist
    L = _lib.lib()
    buf = ctypes.create_string_buffer(128)
    if rank == 0:
        _lib.check(L.mr_rccl_unique_id(buf), "mr_rccl_unique_id")
    obj = [bytes(buf.raw) if rank == 0 else None]
    if world > 1:
        dist.broadcast_object_list(obj, src=0)
    uid = ctypes.create_string_buffer(obj[0], 128)
    ub = np.ascontiguousarray(user_begin, dtype=np.int64)
    ib = np.ascontiguousarray(item_begin, dtype=np.int64)
    _lib.check(L.mr_als_set_rccl(ctx._h, uid, int(rank), int(world),
                                 ub.ctypes.data_as(_lib.LLP), ib.ctypes.data_as(_lib.LLP)),
               "mr_als_set_rccl")
    ctx._rccl = (ub, ib)


def attach_peer_scalars(ctx, rank, world, _fail_set_peer=False):
    """Switch ``ctx``'s CG scalars to the peer all-reduce (include/mr_als.h
    ``mr_als_set_peer``): every rank exports its exchange buffer's IPC handle,
    ``torch.distributed`` gathers the handles in rank order, every rank maps
    its peers', and one self-test reduction checks the sums.  Collective: all
    ranks call it.  Returns True on success; on any rank's failure every rank
    keeps its collective scalars (each step's outcome is agreed by an
    all-reduce, and a rank whose own step succeeded switches back with
    ``mr_als_set_peer(world=0)``; a failure of that reset raises).
    ``_fail_set_peer`` (tests only) makes this rank's ``mr_als_set_peer``
    fail (an out-of-range world)."""
    import torch
    import torch.distributed as dist
    L = _lib.lib()
    buf = ctypes.create_string_buffer(64)
    ok = L.mr_als_peer_handle(ctx._h, buf) == 0
    handles = [None] * world
    dist.all_gather_object(handles, bytes(buf.raw) if ok else None)
    if any(h is None for h in handles):
        return False
    joined = ctypes.create_string_buffer(b"".join(handles), 64 * world)

    def agree(ok):
        flag = torch.tensor([1 if ok else 0], dtype=torch.int32)
        if dist.get_backend() == "nccl":
            flag = flag.cuda()
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        return int(flag.item()) == 1

    def reset():
        _lib.check(L.mr_als_set_peer(ctx._h, None, int(rank), 0), "mr_als_set_peer(world=0)")
        return False

    w_arg = 1 << 20 if _fail_set_peer else int(world)
    if not agree(L.mr_als_set_peer(ctx._h, joined, int(rank), w_arg) == 0):
        return reset()
    # one reduction through the mapped buffers on every rank before trusting them
    if not agree(L.mr_als_peer_selftest(ctx._h) == 0):
        return reset()
    ctx._peer = joined
    if ranks_share_a_gpu(ctx):
        # two resident CG grids on one GPU would each hold every CU slot
        # while waiting for the other's reduction (include/mr_als.h
        # MR_OPT_CG_RESIDENT): one launch per CG iteration instead
        ctx.set_option("cg_resident", 0)
    return True


def ranks_share_a_gpu(ctx):
    """Collective: True when two ranks of the group run on one physical GPU
    (same host and PCI bus id) -- the test layouts with --device-map 0,0."""
    import socket
    import torch.distributed as dist
    buf = ctypes.create_string_buffer(64)
    _lib.check(_lib.lib().mr_device_pci_bus_id(ctx.device, buf, 64), "mr_device_pci_bus_id")
    me = (socket.gethostname(), buf.value.decode())
    allr = [None] * dist.get_world_size()
    dist.all_gather_object(allr, me)
    return len(set(allr)) < len(allr)


def sharded_context(user_ids, item_ids, ratings, k, num_users, num_items, device,
                    comm="rccl", bounds=None, scalars="collective", **kw):
    """Build this rank's ``AlsContext`` over an initialised torch.distributed
    group and attach its collectives: ``comm="rccl"`` (native, device-side),
    or a ``TorchComm`` (host-staged callbacks carrying the same padded
    exchange buffers; works with gloo).  ``bounds=(ub, ib)`` imposes the
    shard boundaries (default: cost-balanced).  ``scalars="peer"``: the CG
    scalars go through the peer all-reduce (``attach_peer_scalars``)."""
    import torch.distributed as dist
    from .engine import AlsContext
    rank, world = dist.get_rank(), dist.get_world_size()
    (u0, u1), (i0, i1), uv, iv, ub, ib = shard_views(
        user_ids, item_ids, ratings, num_users, num_items, rank, world, k=k, bounds=bounds)
    fail_peer = kw.pop("_fail_set_peer", False)
    ctx = AlsContext(uv[0], uv[1], uv[2], k, num_users, num_items, device=device,
                     user_range=(u0, u1), item_range=(i0, i1), item_view=iv, **kw)
    attach_comm(ctx, comm, rank, world, ub, ib)
    ctx.peer_scalars = scalars == "peer" and attach_peer_scalars(ctx, rank, world,
                                                                 _fail_set_peer=fail_peer)
    return ctx
