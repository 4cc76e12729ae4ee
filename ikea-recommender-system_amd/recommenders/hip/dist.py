"""Collectives for the multi-GPU step (one process per GPU, torch.distributed).

With the "nccl" backend (= RCCL on ROCm, xGMI inside a node) device tensors
go straight to torch.distributed's RCCL collectives, which run on the process
group's own stream.  RG_COMM=native routes them to the library's own RCCL
communicator instead (csrc/comm.hip): every collective enqueued on the
CURRENT stream — no cross-stream hops, less host bookkeeping (11 vs 15 µs a
call at one rank, profiles/r06/commlat_one_rank.txt).  It is not the default:
without the process group's stream the step's streams land on the GPU's four
hardware queues differently, and at one rank the default stream then shared
a queue with the head's pass-2 stream — the trunk backward waited for pass 2,
C2 item-sharded 285K (torch) vs 265K (native) session-steps/s; with 16
hardware queues the order flipped (286K native vs 231K torch) and C4 lost
7 % (profiles/r06/hwqueue_ab.txt), so neither is a fix by itself.
With "gloo" the same calls are staged through host memory — used to run
several ranks on one GPU in tests and on CPU.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

# dtype codes of csrc/comm.hip
_DT = {torch.uint8: 0, torch.int32: 1, torch.float32: 2, torch.float16: 3, torch.int64: 4}
_NATIVE = {}   # (process group, world, rank) -> (group, communicator handle)


def _native_comm(dist, group, host_group, rank, world):
    """The library's RCCL communicator for this process group (one per group
    and process: trainers built on the same group share it)."""
    from . import call
    pg = group if group is not None else dist.distributed_c10d._get_default_group()
    key = (id(pg), world, rank)
    hit = _NATIVE.get(key)
    if hit is not None:
        return hit[1]
    uid = torch.zeros(call("rg_comm_id_bytes"), dtype=torch.uint8)
    if rank == 0:
        call("rg_comm_unique_id", uid.data_ptr())
    src = dist.get_global_rank(host_group, 0) if host_group is not None else 0
    dist.broadcast(uid, src=src, group=host_group)
    h = ctypes.c_void_p()
    call("rg_comm_init", uid.data_ptr(), world, rank, torch.cuda.current_device(), ctypes.addressof(h))
    if not _NATIVE:
        import atexit
        atexit.register(destroy_native_comms)
    _NATIVE[key] = (pg, h.value)   # (the group is kept alive: its id stays unique)
    return h.value


def destroy_native_comms():
    """Free every communicator of the library's own RCCL path (rg_comm_destroy),
    after the device has drained; registered with atexit by the first one and
    safe to call earlier, e.g. before the process group is destroyed."""
    from . import call
    if not _NATIVE:
        return
    torch.cuda.synchronize()
    for key in list(_NATIVE):
        _, h = _NATIVE.pop(key)
        call("rg_comm_destroy", h)


class _Done:
    """Work handle of a stream-ordered native collective: already ordered on
    the stream it was issued on."""

    def wait(self):
        return None


class Comm:
    def __init__(self, group=None):
        import torch.distributed as dist
        if not dist.is_initialized():
            raise RuntimeError("item sharding needs torch.distributed to be initialised")
        self.dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.native = dist.get_backend(group) == "nccl"
        # host-side group for the small per-step routing counts (computed on
        # the host from the host batch): a gloo group next to RCCL, so the
        # count exchange never waits on the device stream
        self.host_group = dist.new_group(backend="gloo") if self.native else group
        self.rc = None
        if self.native and os.environ.get("RG_COMM", "torch") == "native":
            self.rc = _native_comm(dist, group, self.host_group, self.rank, self.world)

    def _st(self):
        from . import stream_ptr
        return stream_ptr()

    @staticmethod
    def _dt(t):
        return _DT.get(t.dtype, 0)

    @staticmethod
    def _units(t):
        """elements of the collective's dtype per row of t (bytes for other dtypes)"""
        n = int(np.prod(t.shape[1:])) if t.dim() > 1 else 1
        return n if t.dtype in _DT else n * t.element_size()

    def host_all_gather(self, t):
        """(world, *t.shape) CPU tensor of every rank's CPU tensor ``t`` (no device sync)."""
        t = t.contiguous()
        parts = [torch.empty_like(t) for _ in range(self.world)]
        self.dist.all_gather(parts, t, group=self.host_group)
        return torch.stack(parts)

    def all_gather(self, out, inp):
        """out (world·n) ← concat over ranks of inp (n), rank-major."""
        if self.rc is not None:
            inp = inp.contiguous()
            assert out.is_contiguous() and out.numel() == self.world * inp.numel() and out.dtype == inp.dtype
            n = inp.numel() if inp.dtype in _DT else inp.numel() * inp.element_size()
            from . import call
            call("rg_comm_allgather", self.rc, inp.data_ptr(), out.data_ptr(), n, self._dt(inp), self._st())
            return out
        if self.native:
            self.dist.all_gather_into_tensor(out, inp.contiguous(), group=self.group)
            return out
        parts = [torch.empty(inp.shape, dtype=inp.dtype) for _ in range(self.world)]
        self.dist.all_gather(parts, inp.detach().cpu().contiguous(), group=self.group)
        out.copy_(torch.cat(parts).view(out.shape))
        return out

    def reduce_scatter(self, out, inp):
        """out (n) ← slice `rank` of the elementwise sum over ranks of inp (world·n)."""
        if self.rc is not None:
            inp = inp.contiguous()
            assert out.is_contiguous() and inp.numel() == self.world * out.numel() and inp.dtype in _DT
            from . import call
            call("rg_comm_reduce_scatter", self.rc, inp.data_ptr(), out.data_ptr(), out.numel(), self._dt(inp),
                 self._st())
            return out
        if self.native:
            self.dist.reduce_scatter_tensor(out, inp.contiguous(), group=self.group)
            return out
        t = inp.detach().cpu().contiguous()
        self.dist.all_reduce(t, group=self.group)
        n = out.numel()
        out.copy_(t.view(-1)[self.rank * n:(self.rank + 1) * n].view(out.shape))
        return out

    def all_to_all(self, out, inp, out_splits, in_splits):
        """Variable all-to-all along dim 0: rows [Σ in_splits[:q], +in_splits[q])
        of ``inp`` go to rank q; ``out`` receives out_splits[q] rows from q."""
        if self.rc is not None:
            inp = inp.contiguous()
            assert out.is_contiguous() and out.dtype == inp.dtype
            from . import call
            u = self._units(inp)
            sc = (ctypes.c_int64 * self.world)(*[int(x) * u for x in in_splits])
            rc = (ctypes.c_int64 * self.world)(*[int(x) * u for x in out_splits])
            call("rg_comm_alltoallv", self.rc, inp.data_ptr() if inp.numel() else None, sc,
                 out.data_ptr() if out.numel() else None, rc, self._dt(inp), self._st())
            return out
        if self.native:
            self.dist.all_to_all_single(out, inp.contiguous(), list(out_splits), list(in_splits), group=self.group)
            return out
        o = torch.empty((out.shape[0],) + tuple(out.shape[1:]), dtype=out.dtype)
        self.dist.all_to_all_single(o, inp.detach().cpu().contiguous(), list(out_splits), list(in_splits),
                                    group=self.group)
        out.copy_(o)
        return out

    def all_reduce(self, t, async_op=False):
        if self.rc is not None:
            assert t.is_contiguous() and t.dtype in _DT and t.dtype != torch.uint8
            from . import call
            call("rg_comm_allreduce", self.rc, t.data_ptr(), t.data_ptr(), t.numel(), self._dt(t), self._st())
            return _Done() if async_op else None
        if self.native:
            return self.dist.all_reduce(t, group=self.group, async_op=async_op)
        c = t.detach().cpu().contiguous()
        self.dist.all_reduce(c, group=self.group)
        t.copy_(c.view(t.shape))
        return None


def item_shard(A, world, rank):
    """Contiguous, balanced item range [lo, hi) owned by `rank`."""
    return (rank * A) // world, ((rank + 1) * A) // world


def distinct_ids(s, lens, L, packed, n_rows):
    """The distinct item ids among this batch's packed tokens, sorted, −1
    first when a token's id is outside [0, n_rows) — the ids the row-sharded
    table's exchange requests, in the order csrc/segsum.hip rg_shard_dedup
    ranks them (tokens t < clamp(len, 1, L) of every row, all L when
    unpacked).  int32."""
    s = np.asarray(s)
    B = s.shape[0]
    ln = np.clip(np.asarray(lens, dtype=np.int64), 1, L) if packed else np.full(B, L, dtype=np.int64)
    ids = s[np.arange(L)[None, :] < ln[:, None]]
    ok = (ids >= 0) & (ids < n_rows)
    # distinct ids through a reusable bitmap over the table (cheaper than a sort
    # at ~90K tokens): mark, list, unmark
    mark = _BITMAPS.get(n_rows)
    if mark is None:
        mark = _BITMAPS[n_rows] = np.zeros(n_rows, dtype=np.bool_)
    good = ids[ok]
    mark[good] = True
    u = np.flatnonzero(mark).astype(np.int32)
    mark[good] = False
    if not ok.all():
        u = np.concatenate([np.full(1, -1, dtype=np.int32), u])
    return u


def owner_counts(s, lens, L, packed, n_rows, world, uids=None):
    """Per owner rank, the number of DISTINCT item ids among this batch's
    packed tokens whose table row it holds — the splits of the deduplicated
    exchange (host restatement of csrc/emb_shard.hip k_token_ids +
    csrc/segsum.hip rg_shard_dedup; owner ⌈(id+1)·W/N1⌉ − 1 = the item_shard
    range holding id; every id outside [0, N1) is one entry (−1) of rank 0).
    ``uids``: distinct_ids of the batch, when already computed."""
    u = distinct_ids(s, lens, L, packed, n_rows) if uids is None else uids
    bad = int(u.size > 0 and u[0] < 0)
    bounds = [(r * n_rows) // world for r in range(world + 1)]
    out = np.diff(np.searchsorted(u[bad:], bounds)).astype(np.int64)
    out[0] += bad
    return out


_BITMAPS = {}


def target_owner_counts(a, n_items, world):
    """Per owner rank, the number of this batch's targets whose output row it
    holds (host restatement of csrc/sampled_shard.hip k_target_ids +
    k_shard_route: owner ⌈(a+1)·W/A⌉ − 1, targets outside [0, A) to rank 0)."""
    return np.bincount(_target_owners(a, n_items, world), minlength=world).astype(np.int64)


def _target_owners(a, n_items, world):
    a = np.asarray(a, dtype=np.int64).reshape(-1)
    ok = (a >= 0) & (a < n_items)
    return np.where(ok, ((a + 1) * world + n_items - 1) // n_items - 1, 0)


def target_route(a, n_items, world):
    """The sharded sampled head's target exchange from the host batch, as
    k_target_ids + k_shard_route compute it on the device: one int32 array
    [t32 | slot | send] of 3·B — t32[b] = a[b] (−1 outside [0, A)), the stable
    partition of the rows by owner (slot[b] = send position of row b) and
    send[slot[b]] = t32[b]."""
    a = np.asarray(a, dtype=np.int64).reshape(-1)
    B = a.size
    t32 = np.where((a >= 0) & (a < n_items), a, -1).astype(np.int32)
    order = np.argsort(_target_owners(a, n_items, world), kind="stable")
    out = np.empty(3 * B, dtype=np.int32)
    out[:B] = t32
    out[B + order] = np.arange(B, dtype=np.int32)
    out[2 * B:] = t32[order]
    return out


def host_routes(comm, trunk, passes, targets=None):
    """Send / receive splits of every trunk pass's id / row exchange, from
    the host batch: distinct-id owner counts per pass, one host all-gather
    over the gloo group (W × passes × W ints).  passes: [(s, lens)] host tensors; targets:
    optional (a, n_items) — the item-sharded sampled head's target-row
    exchange, routed the same way (appended last).  Returns
    [(send_splits, recv_splits, plan)] — plan: the pass's distinct_ids (the
    device then skips the dedup's mark / scan, rg_shard_dedup_ids) or, for
    the targets, their target_route — or None when a batch is already on the
    device (then the exchange routes on the device and reads the counts back)."""
    for s, ln in passes:
        if torch.as_tensor(s).device.type != "cpu" or torch.as_tensor(ln).device.type != "cpu":
            return None
    if targets is not None and torch.as_tensor(targets[0]).device.type != "cpu":
        return None
    plans, rows = [], []
    for s, ln in passes:
        s_np = torch.as_tensor(s).numpy()
        u = distinct_ids(s_np, torch.as_tensor(ln).numpy(), s_np.shape[1], trunk.packed, trunk.N1)
        plans.append(u)
        rows.append(owner_counts(None, None, None, None, trunk.N1, comm.world, uids=u))
    if targets is not None:
        a_np = torch.as_tensor(targets[0]).numpy()
        rows.append(target_owner_counts(a_np, int(targets[1]), comm.world))
        plans.append(target_route(a_np, int(targets[1]), comm.world))
    mine = np.stack(rows)
    allc = comm.host_all_gather(torch.from_numpy(mine)).numpy()   # (W, P, W): [q, p, r]
    r = comm.rank
    return [(allc[r, p, :].tolist(), allc[:, p, r].tolist(), plans[p]) for p in range(len(rows))]


class HostStage:
    """A pinned host buffer for one small per-step host → device copy (the
    exchange plans of host_routes): the previous copy out of it is waited for
    before it is overwritten."""

    def __init__(self):
        self.buf = None
        self.ev = None

    def to_device(self, arr, dst):
        """dst[:arr.size] ← arr (int32 numpy) on the current stream; returns that view."""
        n = int(arr.size)
        if self.buf is None or self.buf.numel() < n:
            self.buf = torch.empty(max(n, 1024), dtype=torch.int32).pin_memory()
            self.ev = None
        if self.ev is not None:
            self.ev.synchronize()
        self.buf.numpy()[:n] = arr
        out = dst[:n]
        out.copy_(self.buf[:n], non_blocking=True)
        self.ev = torch.cuda.Event()
        self.ev.record()
        return out
