"""Host orchestration of one training step on the MI355X (Python on
PyTorch-ROCm; every FLOP runs in the HIP kernels of csrc/ via the C ABI).

PyTorch is used for device memory (parameters, Adam moments, workspaces are
torch tensors), streams and one-time CPU initialisation; nothing here
computes the step with torch ops.

Objects
-------
Param        p / m / v fp32 device tensors of one reference parameter.
AdamClock    per-optimizer step counter -> the six fp32 scalars the kernels
             need, rounded like torch's CPU Adam sees them.
Trunk        embedding + GRU (layer 0; optional reverse direction) — the
             SURVEY §8 rows A3/A4/A5 — forward, BPTT, gradient reductions and
             the Adam sweeps of its parameters.
SoftmaxHead  full-softmax Linear + CE (A6/A7) with fused dW+Adam (A8).
LinearHead   a Linear(H→A) used only through row gathers / argmax (Q heads).
"""
from __future__ import annotations

import math
import os
import weakref

import numpy as np
import torch

from . import call, host_floats, host_ptr_array, load_library, ptr, stream_ptr
from .timing import region


def _f32(x: float) -> float:
    return float(np.float32(x))


# --------------------------------------------------------------- params ----
class Param:
    __slots__ = ("name", "p", "m", "v")

    def __init__(self, name, cpu_tensor, device):
        self.name = name
        self.p = cpu_tensor.to(device=device, dtype=torch.float32).contiguous()
        self.m = torch.zeros_like(self.p)
        self.v = torch.zeros_like(self.p)

    def numel(self):
        return self.p.numel()


class AdamClock:
    """torch.optim.Adam hyper-parameters + step counter (GRU4Rec/model.py:124-127)."""

    def __init__(self, lr, betas=(0.9, 0.999), eps=1e-8):
        self.lr, self.b1, self.b2, self.eps = float(lr), betas[0], betas[1], eps
        self.t = 0

    def next_args(self):
        self.t += 1
        t = float(self.t)
        bc1 = 1 - self.b1 ** t
        bc2 = 1 - self.b2 ** t
        step_size = self.lr / bc1
        bc2_sqrt = bc2 ** 0.5
        return host_floats([_f32(1 - self.b1), _f32(self.b2), _f32(1 - self.b2), _f32(bc2_sqrt),
                            _f32(self.eps), _f32(-step_size)])

    def state(self):
        return {"step": self.t, "lr": self.lr, "betas": (self.b1, self.b2), "eps": self.eps}


# --------------------------------------------------------- reference init ---
# RNG consumption order = the reference's module construction order after
# torch.manual_seed(torch_rand_seed) (GRU4Rec/model.py:103-104).

def init_embedding(n_rows, dim, pad, train_pad):
    w = torch.empty(n_rows, dim)
    torch.nn.init.normal_(w)                     # nn.Embedding.reset_parameters
    if not train_pad:
        with torch.no_grad():
            w[pad].fill_(0)
    w.normal_(mean=0, std=0.01)                  # GRU4Rec/model.py:42
    if not train_pad:
        with torch.no_grad():
            w[pad] = torch.zeros(dim)            # :45-47
    return w


def init_gru(input_size, hidden, layers, bidir):
    """nn.GRU.reset_parameters: U(-1/sqrt(H), 1/sqrt(H)) over parameters in
    registration order (l0: w_ih, w_hh, b_ih, b_hh, [l0_reverse ...], l1 ...)."""
    stdv = 1.0 / math.sqrt(hidden)
    out = []
    ndir = 2 if bidir else 1
    for layer in range(layers):
        in_sz = input_size if layer == 0 else hidden * ndir
        for d in range(ndir):
            sfx = f"_l{layer}" + ("_reverse" if d == 1 else "")
            shapes = [("weight_ih" + sfx, (3 * hidden, in_sz)), ("weight_hh" + sfx, (3 * hidden, hidden)),
                      ("bias_ih" + sfx, (3 * hidden,)), ("bias_hh" + sfx, (3 * hidden,))]
            for name, shp in shapes:
                out.append((name, torch.empty(shp)))
    for _, t in out:
        torch.nn.init.uniform_(t, -stdv, stdv)
    return out


def init_linear(in_f, out_f):
    """nn.Linear.reset_parameters: kaiming_uniform_(a=sqrt(5)) + U(-1/sqrt(in), 1/sqrt(in))."""
    w = torch.empty(out_f, in_f)
    torch.nn.init.kaiming_uniform_(w, a=math.sqrt(5))
    b = torch.empty(out_f)
    bound = 1 / math.sqrt(in_f) if in_f > 0 else 0
    torch.nn.init.uniform_(b, -bound, bound)
    return w, b


_WIDTHS = (16, 32, 64, 128, 256)


def _round_up(x, m):
    return (x + m - 1) // m * m


# ------------------------------------------------------- catch-up Adam ----
# Tables read a few rows per step — the item embedding (the batch's tokens) and
# the sampled head's W / b (targets and negatives) — take their zero-gradient
# Adam steps only when a row is next read (csrc/optim.hip rg_lazy_*): bitwise
# the reference's dense torch.optim.Adam (GRU4Rec/model.py:124-127,153; every
# row moves every step), without the sweep over every row (C3: 1.6 of 3.7 ms).
# False: the eager sweeps (rg_adam_rows), e.g. for A/B checks.
LAZY_ADAM = True
# floats per step of the catch-up history (csrc/optim.hip LAZY_HS)
LAZY_HS = 8
# a sampled head's backward queues the catch-up of the next draw's negatives on
# a side stream (LazyRows.catch_up_async), under the trunk backward
PREFETCH_NEGATIVES = True
# ... and the step's targets are caught up on that side stream beside the trunk
# forward (SampledSoftmaxHead.prepare_rows(early=True)); RG_TARGETS_ASYNC=0: on
# the launch stream before it (A/B; default off until measured)
TARGETS_ASYNC = os.environ.get("RG_TARGETS_ASYNC", "0") != "0"


class LazyRows:
    """Catch-up bookkeeping of one table (and an optional one-column
    companion, a head's bias): last[r] = table steps applied to row r, hist
    = every step's Adam scalars, LAZY_HS floats (written by the step's own kernel), need /
    stamp = the rows a read is about to touch.  ``tab``: (P, M, V, cols, P16,
    Pb, Mb, Vb) device pointers / widths of the table."""

    def __init__(self, rows, device):
        self.rows = int(rows)
        self.device = device
        self.last = torch.zeros(self.rows, dtype=torch.int32, device=device)
        self.need = torch.zeros(self.rows, dtype=torch.int32, device=device)
        self.stamp = 0
        self.n = 0        # table steps so far
        self.full = 0     # n at the last catch-up of every row
        self.hist = torch.zeros(256, LAZY_HS, device=device)
        self.side = None      # stream of catch_up_async
        self.pending = None   # its event, until a use of the table joins it

    def catch_up(self, tab, ids=None, n_ids=0, seed=0, counter=0, S=0, more=(), ids32=None):
        """Bring the rows a read is about to touch — ``n_ids`` int64 ids at
        ``ids`` (device), the S negatives of draw ``counter`` and the (ptr, n)
        id sets of ``more`` — up to date.  On the stream every read of the
        table is ordered behind (two streams must not catch up one table
        concurrently: the double-Q step catches up all its passes' rows first)."""
        self.join()
        n32 = ids32[1] if ids32 is not None else 0
        if self.n == self.full or n_ids + S + n32 + sum(n for _, n in more) == 0:
            return
        st = stream_ptr()
        self.stamp += 1
        for p, n, sd, cn, ns in [(ids, n_ids, seed, counter, S)] + [(p, n, 0, 0, 0) for p, n in more]:
            if n + ns:
                call("rg_lazy_mark_rows", p, n, self.rows, sd, cn, ns, self.need.data_ptr(), self.stamp, st)
        if n32:   # (ptr, n, lo): int32 global ids of a row shard starting at lo
            call("rg_lazy_mark_rows32", ids32[0], n32, ids32[2], self.rows, self.need.data_ptr(), self.stamp, st)
        call("rg_lazy_catch_up", *tab, self.rows, self.last.data_ptr(), self.need.data_ptr(), self.stamp, self.n,
             self.hist.data_ptr(), st)

    def catch_up_async(self, tab, seed, counter, S, ids=None, n_ids=0):
        """catch_up of the S negatives of draw ``counter`` (and of ``n_ids``
        int64 ids at ``ids``) on a side stream, ordered after everything
        queued so far on the current stream (the step's own Adam): it runs
        under the rest of the step (the trunk backward, the next step's trunk
        forward).  The next use of the table on any stream — catch_up, adam,
        materialize, join — waits for it first."""
        self.join()
        if self.n == self.full or S + n_ids == 0:
            return
        cur = torch.cuda.current_stream(self.device)
        if self.side is None:
            self.side = torch.cuda.Stream(device=self.device)
        self.side.wait_stream(cur)
        with torch.cuda.stream(self.side):
            self.catch_up(tab, ids, n_ids, seed, counter, S)
        self.pending = torch.cuda.Event()
        self.pending.record(self.side)

    def join(self):
        """Order the current stream after a pending catch_up_async."""
        if self.pending is not None:
            torch.cuda.current_stream(self.device).wait_event(self.pending)
            self.pending = None

    def materialize(self, tab):
        """Every row up to date (before a read of the whole table: evaluation,
        state_dict, the optimizer state, a load)."""
        self.join()
        if self.n > self.full:
            call("rg_lazy_catch_up", *tab, self.rows, self.last.data_ptr(), None, 0, self.n, self.hist.data_ptr(),
                 stream_ptr())
            self.full = self.n

    def adam(self, tab, G, Gb, tags, tag, adam6):
        """Table step n + 1 on the rows tagged ``tag`` (their gradient rows G / Gb)."""
        self.join()
        n = self.n + 1
        if n > self.hist.shape[0]:
            grown = torch.zeros(2 * self.hist.shape[0], LAZY_HS, device=self.device)
            grown[:self.hist.shape[0]].copy_(self.hist)
            self.hist = grown
        P, M, V, cols, P16, Pb, Mb, Vb = tab
        call("rg_lazy_adam_rows", P, M, V, G, cols, P16, Pb, Mb, Vb, Gb, self.rows, self.last.data_ptr(), tags, tag, n,
             self.hist.data_ptr(), adam6, stream_ptr())
        self.n = n


# ---------------------------------------------------------------- trunk ----
class SegScatter:
    """Deterministic row scatter-add (csrc/segsum.hip rg_scatter_rows: sort by
    id, ordered per-row sums, no float atomics) with a workspace that grows to
    the largest row count seen."""

    def __init__(self, device):
        self.device = device
        self.work = None
        self.sizes = {}

    def __call__(self, ids, src, E, n_ptr, n_max, skip, G, n_rows, tags, tag, st, reuse_sort=False, ld=None):
        """ld: floats between consecutive source rows (default E)."""
        need = self.sizes.get((n_max, E, n_rows))
        if need is None:
            need = self.sizes[(n_max, E, n_rows)] = int(call("rg_scatter_rows_work_bytes", n_max, E, n_rows))
        if self.work is None or self.work.numel() < need:
            self.work = torch.empty(need, dtype=torch.uint8, device=self.device)
        call("rg_scatter_rows", ids, src, E, E if ld is None else ld, n_ptr, n_max, skip, G, n_rows, tags, tag,
             1 if reuse_sort else 0, self.work.data_ptr(), self.work.numel(), st)


class _TrunkWS:
    """Workspace of one trunk pass for a (B, L) batch shape."""

    def __init__(self, B, L, E, H, ndir, save, device):
        TM = B * L  # token upper bound (T is only known on the device)
        z = lambda *s, dt=torch.float32: torch.empty(*s, dtype=dt, device=device)
        self.B, self.L, self.TM = B, L, TM
        self.lens = z(B, dt=torch.int64)
        self.perm = z(B, dt=torch.int32)
        self.lsort = z(B, dt=torch.int32)
        self.offs = z(B + 1, dt=torch.int32)
        self.tok_id = [z(TM, dt=torch.int32) for _ in range(ndir)]
        self.X = [z(TM, E) for _ in range(ndir)]
        self.Gi = [z(TM, 3 * H) for _ in range(ndir)]
        self.h = torch.zeros(B, ndir * H, device=device)
        self.plane = TM * H
        # H = 256: W_hh's MFMA fragments for the persistent wide GRU (csrc/gru.hip)
        self.wfrag = z(call("rg_gru_wide_work_bytes", H) // 4) if H > 128 else None
        self.saved = [z(5, TM, H) for _ in range(ndir)] if save else None
        if save:
            self.dGi = [z(TM, 3 * H) for _ in range(ndir)]
            self.dGh = [z(TM, 3 * H) for _ in range(ndir)]
            self.dX = [z(TM, E) for _ in range(ndir)]
            self.splits = int(min(128, max(1, TM // 1024)))
            S = self.splits
            self.sl_ih = [z(S, 3 * H, E) for _ in range(ndir)]
            self.sl_hh = [z(S, 3 * H, H) for _ in range(ndir)]
            self.cs_ih = [z(S, 3 * H) for _ in range(ndir)]
            self.cs_hh = [z(S, 3 * H) for _ in range(ndir)]

    @property
    def ntok_ptr(self):
        return self.offs.data_ptr() + 4 * self.B  # &offs[B] = T


class Trunk:
    """Item embedding + GRU trunk.  Only layer 0 feeds the heads (h[0] quirk,
    GRU4Rec/model.py:77); deeper layers are initialised for RNG / state_dict
    parity but are mathematically inert (zero gradient => Adam leaves them
    unchanged), so they are not computed."""

    def __init__(self, gru_attr, item_num, E, H, layers, train_pad_embed, packed, pad_idx, bidir, device,
                 fp16_embeddings=False, comm=None):
        self.gru_attr = gru_attr
        self.N1 = item_num + 1
        self.E, self.H, self.layers, self.bidir = E, H, layers, bidir
        self.ndir = 2 if bidir else 1
        self.packed = packed
        self.pad = pad_idx
        self.train_pad = train_pad_embed
        self.device = device
        if E not in _WIDTHS or H not in _WIDTHS:
            raise RuntimeError(f"unsupported trunk shape E={E} H={H} (E, H in {_WIDTHS})")
        # H <= 128: persistent recurrence with W_hh in VGPRs; H = 256: persistent
        # wide recurrence streaming W_hh (768 KB) from L2 (csrc/gru.hip
        # rg_gru_fwd_wide / rg_gru_bwd_wide)
        self.wide = H > 128
        # comm (multi-GPU): the table is row-sharded, this rank holds rows
        # [lo, hi) (full init drawn first: RNG parity with one GPU); the rows a
        # pass needs are exchanged by all-to-all (csrc/emb_shard.hip)
        self.comm = comm
        full = init_embedding(self.N1, E, pad_idx, train_pad_embed)
        if comm is not None:
            from .dist import item_shard
            self.lo, self.hi = item_shard(self.N1, comm.world, comm.rank)
            full = full[self.lo:self.hi].contiguous()
        else:
            self.lo, self.hi = 0, self.N1
        self.n_local = self.hi - self.lo
        self.emb = Param("embedding.weight", full, device)
        gru = init_gru(E, H, layers, bidir)
        self.gru_params = [Param(f"{gru_attr}.{n}", t, device) for n, t in gru]
        per = 4
        self.dirs = [self.gru_params[d * per:(d + 1) * per] for d in range(self.ndir)]  # layer 0
        self.G_emb = torch.zeros_like(self.emb.p)
        self.tags = torch.zeros(self.n_local, dtype=torch.int32, device=device)
        self.err = torch.zeros(1, dtype=torch.int32, device=device)  # out-of-range item ids seen
        self.scatter = SegScatter(device)
        self._ws = {}
        # bf16 plane products of the trunk GEMMs (csrc/gemm.hip rg_gemm_x6 / rg_wgrad_x6; the
        # nets set it with the heads' matmul_precision); 0: the fp32 MFMA kernels.  Needs
        # E % 32 == 0 and H % 32 == 0 (the GEMMs' K and N), else the fp32 kernels run
        self.gemm_terms = 0
        # emit_planes (set for the sampled head's split logits): the training
        # forward's GRU launch also writes the final h as bf16 K-planes
        # (rg_gru_fwd_dirs_planes), left in h_planes for the head
        self.emit_planes = False
        self.h_planes = None
        self.neg_job = None   # set by the sampled step for the next forward (SampledSoftmaxHead.neg_job)
        # fp16 embedding storage (config C5): the gather reads this copy, Adam
        # keeps the fp32 master and refreshes it in the same sweep
        self.emb16 = torch.empty(self.n_local, E, dtype=torch.float16, device=device) if fp16_embeddings else None
        self.refresh_half()
        # catch-up Adam of the table (row-sharded: of this rank's rows, caught up on
        # the owner for the ids the ranks request, _exchange_rows)
        self.lazy = LazyRows(self.n_local, device) if LAZY_ADAM else None

    def _lazy_tab(self):
        return (self.emb.p.data_ptr(), self.emb.m.data_ptr(), self.emb.v.data_ptr(), self.E,
                None if self.emb16 is None else self.emb16.data_ptr(), None, None, None)

    def materialize(self):
        """Every row of the table up to date (catch-up Adam)."""
        if self.lazy is not None:
            self.lazy.materialize(self._lazy_tab())

    def catch_up_rows(self, *states):
        """Catch up every row the trunk passes over ``states`` (device int64
        (B, L) tensors) will read, on the current stream — for passes that then
        run on other streams (forward(..., catch_up=False))."""
        if self.lazy is not None and states and self.comm is None:   # (row-sharded: in _exchange_rows)
            sts = [x.contiguous() for x in states]
            self._keep = sts   # (alive until the kernels reading them have run: the next call replaces it)
            self.lazy.catch_up(self._lazy_tab(), sts[0].data_ptr(), sts[0].numel(),
                               more=[(x.data_ptr(), x.numel()) for x in sts[1:]])

    def refresh_half(self):
        """Re-derive the fp16 table from the fp32 master (init, load_state_dict)."""
        if self.emb16 is not None:
            call("rg_f32_to_f16", self.emb.p.data_ptr(), self.emb.numel(), self.emb16.data_ptr(), stream_ptr())

    # parameters in reference registration order (every row up to date: the
    # callers read or write whole tables)
    def named_params(self):
        self.materialize()
        return [self.emb] + self.gru_params

    def ws(self, slot, B, L, save):
        key = (slot, B, L, save)
        w = self._ws.get(key)
        if w is None:
            # keep one shape per slot (drop stale shapes, e.g. a short last batch)
            for k in [k for k in self._ws if k[0] == slot]:
                del self._ws[k]
            w = _TrunkWS(B, L, self.E, self.H, self.ndir, save, self.device)
            self._ws[key] = w
        return w

    def forward(self, s, lens, slot="main", save=False, route=None, catch_up=True, lens_dev=None):
        """s: int64 (B, L) device; lens: int64 (B,) device or CPU. Returns h (B, ndir*H).
        route (item-sharded table): this pass's (send_splits, recv_splits) from
        the host batch (dist.host_routes); None routes on the device and reads
        the counts back (one sync).  lens_dev: lens already on the device (the
        step's InputStage copy), copied from instead of the host lens."""
        B, L = s.shape
        w = self.ws(slot, B, L, save)
        st = stream_ptr()
        w.lens.copy_(lens_dev if lens_dev is not None else lens, non_blocking=True)
        # host bound of the packed token count (the scatter sorts this many keys)
        lt = torch.as_tensor(lens)
        w.T_host = int(lt.clamp(1, L).sum()) if self.packed and lt.device.type == "cpu" else B * L
        with region("pack"):
            call("rg_pack", w.lens.data_ptr(), B, L, 0 if self.packed else 1, w.perm.data_ptr(),
                 w.lsort.data_ptr(), w.offs.data_ptr(), st)
        H, E = self.H, self.E
        if self.comm is not None:   # the whole row-sharded gather: route, id / row all-to-alls, placement
            with region("gather"):
                self._exchange_rows(w, s, B, L, st, route)
                for d in range(self.ndir):
                    call("rg_place_rows", w.rows_in.data_ptr(), 1 if self.emb16 is not None else 0,
                         w.slot.data_ptr(), w.lsort.data_ptr(), w.offs.data_ptr(), B, E, d, w.X[d].data_ptr(), st)
        if self.lazy is not None and catch_up and self.comm is None:   # the rows this pass reads (every position of s)
            s = s.contiguous()
            self.lazy.catch_up(self._lazy_tab(), s.data_ptr(), B * L)
        # a sampled head's negatives row gather rides in the first gather launch
        # (rg_gather_neg; SampledSoftmaxHead.neg_job)
        job, self.neg_job = self.neg_job, None
        if job is not None and (self.comm is not None or L > 64 or E not in (32, 64, 128, 256)):
            job = None
        for d in range(self.ndir):
            w_ih, w_hh, b_ih, b_hh = self.dirs[d]
            if self.comm is None:
                table = (self.emb16 if self.emb16 is not None else self.emb.p).data_ptr()
                with region("gather", exact=True):
                    if job is not None and d == 0:
                        call("rg_gather_neg", s.data_ptr(), B, L, w.perm.data_ptr(), w.lsort.data_ptr(),
                             w.offs.data_ptr(), table, 1 if self.emb16 is not None else 0, self.N1, E, d,
                             w.tok_id[d].data_ptr(), w.X[d].data_ptr(), self.err.data_ptr(), *job.args(), st)
                        job.done()
                    else:
                        call("rg_gather_h" if self.emb16 is not None else "rg_gather", s.data_ptr(), B, L,
                             w.perm.data_ptr(), w.lsort.data_ptr(), w.offs.data_ptr(), table, self.N1, E, d,
                             w.tok_id[d].data_ptr(), w.X[d].data_ptr(), self.err.data_ptr(), st)
            with region("gemm_ih"):
                if self._x6():
                    call("rg_gemm_x6", w.X[d].data_ptr(), E, w_ih.p.data_ptr(), E, 1, w.Gi[d].data_ptr(), 3 * H,
                         b_ih.p.data_ptr(), w.TM, w.ntok_ptr, 3 * H, E, self.gemm_terms, st)
                else:
                    call("rg_gemm_f32", w.X[d].data_ptr(), E, 1, w_ih.p.data_ptr(), 1, E, w.Gi[d].data_ptr(), 3 * H,
                         b_ih.p.data_ptr(), w.TM, w.ntok_ptr, 3 * H, E, None, 1, st)
            if self.wide:
                with region("gru_fwd"):
                    call("rg_gru_fwd_wide", w.Gi[d].data_ptr(), w_hh.p.data_ptr(), b_hh.p.data_ptr(),
                         w.perm.data_ptr(), w.lsort.data_ptr(), w.offs.data_ptr(), B, H, w.h.data_ptr(),
                         self.ndir * H, d * H, w.saved[d].data_ptr() if save else None, w.plane,
                         w.wfrag.data_ptr(), st)
        self.h_planes = None
        if not self.wide:   # every direction in one launch (grid.y = direction)
            with region("gru_fwd"):
                nd = range(self.ndir)
                args = (host_ptr_array([w.Gi[d] for d in nd]), host_ptr_array([self.dirs[d][1].p for d in nd]),
                        host_ptr_array([self.dirs[d][3].p for d in nd]),
                        host_ptr_array([w.saved[d] if save else None for d in nd]), self.ndir, w.perm.data_ptr(),
                        w.lsort.data_ptr(), w.offs.data_ptr(), B, H, w.h.data_ptr(), self.ndir * H, 0, w.plane)
                if self.emit_planes and save and self.ndir * H in (32, 64, 128, 256):
                    if getattr(w, "hk", None) is None:
                        w.hk = torch.empty(call("rg_head_plane_bytes", B, self.ndir * H), dtype=torch.uint8,
                                           device=self.device)
                    call("rg_gru_fwd_dirs_planes", *args, w.hk.data_ptr(), st)
                    self.h_planes = w.hk
                else:
                    call("rg_gru_fwd_dirs", *args, st)
        return w.h

    def backward(self, dh, slot="main"):
        """BPTT + gradient reductions.  dh: (B, ndir*H).  Leaves embedding grads
        in G_emb (tagged) and GRU grads in slabs; call step() afterwards."""
        w = next(v for k, v in self._ws.items() if k[0] == slot and k[3])
        st = stream_ptr()
        H, E, B, TM, S = self.H, self.E, w.B, w.TM, w.splits
        with region("gru_bwd"):
            if self.wide:
                for d in range(self.ndir):
                    call("rg_gru_bwd_wide", w.saved[d].data_ptr(), w.plane, self.dirs[d][1].p.data_ptr(),
                         w.perm.data_ptr(), w.lsort.data_ptr(), w.offs.data_ptr(), B, H, dh.data_ptr(),
                         self.ndir * H, d * H, w.dGi[d].data_ptr(), w.dGh[d].data_ptr(), w.wfrag.data_ptr(), st)
            else:   # every direction in one launch
                nd = range(self.ndir)
                call("rg_gru_bwd_dirs", host_ptr_array([w.saved[d] for d in nd]),
                     host_ptr_array([self.dirs[d][1].p for d in nd]), host_ptr_array([w.dGi[d] for d in nd]),
                     host_ptr_array([w.dGh[d] for d in nd]), self.ndir, w.plane, w.perm.data_ptr(),
                     w.lsort.data_ptr(), w.offs.data_ptr(), B, H, dh.data_ptr(), self.ndir * H, 0, st)
        self._pending = (w, S)

    # The backward's two gradient paths run on two streams: the GRU weights'
    # (wgrad, slab reduction, Adam / the all-reduce) on the trunk's side
    # stream, the embedding's (dX, scatter or row exchange, the dense Adam
    # sweep) on the current one — each a chain of small kernels that, beside
    # the head's pass 2, wait for CUs one launch at a time.  dX = dGi·W_ih is
    # issued first: it reads W_ih before the side stream's Adam moves it.  The
    # current stream joins the side stream before returning.
    def _wside(self):
        if getattr(self, "_wstream", None) is None:
            self._wstream = torch.cuda.Stream(device=self.device)
        return self._wstream

    def step(self, adam6, tag):
        """Weight gradients + Adam for the trunk (after every use of the weights)."""
        w, S = self._pending
        main = torch.cuda.current_stream(self.device)
        self._grads_dx(w)
        ws = self._wside()
        ws.wait_stream(main)
        with torch.cuda.stream(ws):
            self._grads_w(w, S)
            st = stream_ptr()
            for d in range(self.ndir):
                w_ih, w_hh, b_ih, b_hh = self.dirs[d]
                for prm, sl in ((w_ih, w.sl_ih[d]), (w_hh, w.sl_hh[d]), (b_ih, w.cs_ih[d]), (b_hh, w.cs_hh[d])):
                    call("rg_adam_slabs", prm.p.data_ptr(), prm.m.data_ptr(), prm.v.data_ptr(), sl.data_ptr(), S,
                         prm.numel(), adam6, None, st)
        self._grads_scatter(w, tag)
        self._adam_emb(adam6, tag)
        main.wait_stream(ws)
        self._pending = None

    def _grads_dx(self, w):
        """dX = dGi · W_ih (T × E) of every direction."""
        st = stream_ptr()
        H, E, TM = self.H, self.E, w.TM
        for d in range(self.ndir):
            with region("gemm_dx"):
                if self._x6():
                    call("rg_gemm_x6", w.dGi[d].data_ptr(), 3 * H, self.dirs[d][0].p.data_ptr(), E, 0,
                         w.dX[d].data_ptr(), E, None, TM, w.ntok_ptr, E, 3 * H, self.gemm_terms, st)
                else:
                    call("rg_gemm_f32", w.dGi[d].data_ptr(), 3 * H, 1, self.dirs[d][0].p.data_ptr(), E, 1,
                         w.dX[d].data_ptr(), E, None, TM, w.ntok_ptr, E, 3 * H, None, 1, st)

    def _grads_w(self, w, S):
        """dW_ih = dGiᵀ·X, db_ih = Σ dGi ; dW_hh = dGhᵀ·H_prev, db_hh = Σ dGh (token slabs)."""
        st = stream_ptr()
        H, E, TM = self.H, self.E, w.TM
        x6 = self._x6()
        for d in range(self.ndir):
            with region("wgrad"):
                if x6:
                    call("rg_wgrad_x6", w.dGi[d].data_ptr(), 3 * H, w.X[d].data_ptr(), E, TM, w.ntok_ptr, S,
                         w.sl_ih[d].data_ptr(), w.cs_ih[d].data_ptr(), self.gemm_terms, st)
                    call("rg_wgrad_x6", w.dGh[d].data_ptr(), 3 * H, w.saved[d].data_ptr(), H, TM, w.ntok_ptr, S,
                         w.sl_hh[d].data_ptr(), w.cs_hh[d].data_ptr(), self.gemm_terms, st)
                else:
                    call("rg_wgrad", w.dGi[d].data_ptr(), 3 * H, w.X[d].data_ptr(), E, TM, w.ntok_ptr, S,
                         w.sl_ih[d].data_ptr(), w.cs_ih[d].data_ptr(), st)
                    call("rg_wgrad", w.dGh[d].data_ptr(), 3 * H, w.saved[d].data_ptr(), H, TM, w.ntok_ptr, S,
                         w.sl_hh[d].data_ptr(), w.cs_hh[d].data_ptr(), st)

    def _x6(self):
        return self.gemm_terms and self.E % 32 == 0 and self.H % 32 == 0

    def _grads_scatter(self, w, tag):
        """The embedding rows' gradients: scatter into G_emb, or (item-sharded
        table) sent to their owners."""
        st = stream_ptr()
        if self.comm is not None:
            with region("scatter"):
                self._exchange_grads(w, tag, st)
            return
        skip = -1 if self.train_pad else self.pad
        with region("scatter"):
            if self.ndir == 2:
                # Bidir: the reverse direction's token gradients (stored time-reversed) are
                # added into the forward direction's first (rg_combine_dirs), so one sort and
                # one segmented sum scatter both (as the row-sharded exchange does)
                call("rg_combine_dirs", w.dX[0].data_ptr(), w.dX[1].data_ptr(), w.lsort.data_ptr(),
                     w.offs.data_ptr(), w.B, self.E, st)
            self.scatter(w.tok_id[0].data_ptr(), w.dX[0].data_ptr(), self.E, w.ntok_ptr, w.T_host, skip,
                         self.G_emb.data_ptr(), self.n_local, self.tags.data_ptr(), tag, st)

    # ---- data-parallel variant: gradients summed over ranks before Adam ----
    def grads_for_allreduce(self, tag):
        """Compute this rank's trunk gradients into flat buffers (GRU: gflat on
        the side stream, embedding: rows sent to their owners) ready for a SUM
        all-reduce of gflat."""
        w, S = self._pending
        self._tag = tag
        if getattr(self, "gflat", None) is None:
            n = sum(p.numel() for p in self.gru_params[:4 * self.ndir])
            self.gflat = torch.zeros(n, device=self.device)
        main = torch.cuda.current_stream(self.device)
        self._grads_dx(w)
        ws = self._wside()
        ws.wait_stream(main)
        with torch.cuda.stream(ws):
            self._grads_w(w, S)
            st = stream_ptr()
            off = 0
            for d in range(self.ndir):
                for prm, sl in zip(self.dirs[d], (w.sl_ih[d], w.sl_hh[d], w.cs_ih[d], w.cs_hh[d])):
                    n = prm.numel()
                    call("rg_adam_slabs", prm.p.data_ptr(), prm.m.data_ptr(), prm.v.data_ptr(), sl.data_ptr(), S,
                         n, None, self.gflat.data_ptr() + 4 * off, st)
                    off += n
        self._grads_scatter(w, tag)

    def allreduce_start(self, comm):
        """SUM all-reduce of the GRU gradients (~0.4 MB; the embedding rows went
        to their owners by all-to-all in _exchange_grads), ordered after the
        side stream's slab reduction."""
        with torch.cuda.stream(self._wside()):
            return [comm.all_reduce(self.gflat, async_op=True)]

    def adam_after_allreduce(self, adam6, works=()):
        """The GRU weights' Adam after the all-reduce (side stream), the
        embedding's on the current stream; the current stream joins."""
        main = torch.cuda.current_stream(self.device)
        ws = self._wside()
        with torch.cuda.stream(ws):
            for wk in works:
                if wk is not None:
                    wk.wait()
            st = stream_ptr()
            off = 0
            for d in range(self.ndir):
                for prm in self.dirs[d]:
                    n = prm.numel()
                    call("rg_adam_dense", prm.p.data_ptr(), prm.m.data_ptr(), prm.v.data_ptr(),
                         self.gflat.data_ptr() + 4 * off, n, adam6, 0, st)
                    off += n
        self._adam_emb(adam6, self._tag)
        main.wait_stream(ws)
        self._pending = None

    def _adam_emb(self, adam6, tag):
        """Dense-semantics Adam over this rank's rows (all of them on one GPU):
        row-sparse gradient rows tagged with this step's epoch."""
        st = stream_ptr()
        with region("adam_emb"):
            if self.lazy is not None:   # only the rows with a gradient (catch-up Adam)
                self.lazy.adam(self._lazy_tab(), self.G_emb.data_ptr(), None, self.tags.data_ptr(), tag, adam6)
            elif self.emb16 is not None:
                call("rg_adam_rows_h", self.emb.p.data_ptr(), self.emb.m.data_ptr(), self.emb.v.data_ptr(),
                     self.G_emb.data_ptr(), self.tags.data_ptr(), tag, self.n_local, self.E, adam6,
                     self.emb16.data_ptr(), st)
            else:
                call("rg_adam_rows", self.emb.p.data_ptr(), self.emb.m.data_ptr(), self.emb.v.data_ptr(),
                     self.G_emb.data_ptr(), self.tags.data_ptr(), tag, self.n_local, self.E, adam6, st)

    # ---- row-sharded table: id / row / gradient exchange (csrc/emb_shard.hip) ----
    def _xbuf(self, w, name, rows, cols=None, dtype=torch.int32):
        """Exchange buffer of at least ``rows`` rows, kept on the pass's
        workspace and grown (×1.25) only when a step needs more."""
        t = getattr(w, name, None)
        if t is None or t.shape[0] < rows or t.dtype != dtype:
            n = max(16, int(rows * 1.25) if t is not None else rows)
            t = torch.empty((n,) if cols is None else (n, cols), dtype=dtype, device=self.device)
            setattr(w, name, t)
        return t

    def _exchange_rows(self, w, s, B, L, st, route=None):
        """Rows of the distinct ids of this rank's batch from their owners
        (rg_shard_dedup: one row per distinct id, not per token): all-to-all
        of the ids, owners gather, all-to-all of the rows back.  With
        ``route`` (the distinct-id splits computed on the host from the host
        batch, dist.owner_counts) no device value is read back; otherwise the
        device counts are (one sync)."""
        comm, W = self.comm, self.comm.world
        n_max = max(1, w.T_host)
        if getattr(w, "uslot", None) is None:
            w.uslot = torch.empty(w.TM, dtype=torch.int32, device=self.device)
            w.uids = torch.empty(w.TM, dtype=torch.int32, device=self.device)
            w.counts = torch.zeros(W, dtype=torch.int32, device=self.device)
            w.counts_all = torch.zeros(W * W, dtype=torch.int32, device=self.device)
            w.nuniq = torch.zeros(1, dtype=torch.int32, device=self.device)
            w.nrecv = torch.zeros(1, dtype=torch.int32, device=self.device)
        need = int(call("rg_shard_dedup_work_bytes", n_max, self.E, self.N1))
        dd = self._xbuf(w, "dd_work", need, dtype=torch.uint8)
        w.dd_nmax = n_max
        plan = route[2] if route is not None and len(route) > 2 else None
        if plan is not None:   # the distinct ids from the host batch: token ids + slots in two launches
            if getattr(w, "dd_map", None) is None:
                from .dist import HostStage
                w.dd_map = torch.empty(self.N1 + 1, dtype=torch.int32, device=self.device)
                w.dd_stage = HostStage()
            U = int(plan.size)
            w.dd_stage.to_device(plan, w.uids)
            call("rg_shard_dedup_ids", s.data_ptr(), B, L, w.perm.data_ptr(), w.lsort.data_ptr(), w.offs.data_ptr(),
                 w.ntok_ptr, n_max, self.N1, w.uids.data_ptr(), U, w.dd_map.data_ptr(), w.tok_id[0].data_ptr(),
                 w.uslot.data_ptr(), self.err.data_ptr(), self.E, dd.data_ptr(), dd.numel(), st)
        else:
            call("rg_token_ids", s.data_ptr(), B, L, w.perm.data_ptr(), w.lsort.data_ptr(), w.offs.data_ptr(),
                 self.N1, w.tok_id[0].data_ptr(), self.err.data_ptr(), st)
            call("rg_shard_dedup", w.tok_id[0].data_ptr(), w.ntok_ptr, n_max, self.N1, W, self.E,
                 w.uslot.data_ptr(), w.uids.data_ptr(), w.counts.data_ptr(), w.nuniq.data_ptr(), dd.data_ptr(),
                 dd.numel(), st)
        if route is not None:
            w.send_splits, w.recv_splits = list(route[0]), list(route[1])
            if plan is not None and sum(w.send_splits) != U:
                raise RuntimeError(f"host exchange plan: {U} distinct ids, splits {w.send_splits}")
        else:
            comm.all_gather(w.counts_all, w.counts)
            M = w.counts_all.view(W, W).cpu()            # M[q][r]: distinct ids of rank q owned by rank r (one sync)
            w.send_splits = M[comm.rank].tolist()
            w.recv_splits = M[:, comm.rank].tolist()
        U, R = sum(w.send_splits), sum(w.recv_splits)
        w.U, w.R = U, R
        half = self.emb16 is not None
        rdt = torch.float16 if half else torch.float32
        recv_ids = self._xbuf(w, "recv_ids", max(R, 1))
        w.local_ids = self._xbuf(w, "local_ids_buf", max(R, 1))
        comm.all_to_all(recv_ids[:R], w.uids[:U], w.recv_splits, w.send_splits)
        if self.lazy is not None:   # the requested rows of this shard, caught up before they are read
            self.lazy.catch_up(self._lazy_tab(), ids32=(recv_ids.data_ptr(), R, self.lo))
        rows_out = self._xbuf(w, "rows_out", max(R, 1), self.E, rdt)
        call("rg_rows_gather", recv_ids.data_ptr(), R, self.lo, self.n_local,
             (self.emb16 if half else self.emb.p).data_ptr(), self.E, 1 if half else 0, rows_out.data_ptr(),
             w.local_ids.data_ptr(), st)
        w.rows_in = self._xbuf(w, "rows_in_buf", max(U, 1), self.E, rdt)
        comm.all_to_all(w.rows_in[:U], rows_out[:R], w.send_splits, w.recv_splits)
        w.slot = w.uslot   # rg_place_rows: X[t] = rows_in[uslot[t]]

    def _exchange_grads(self, w, tag, st):
        """Per distinct id, the sum of its tokens' row-gradients (in token
        order) goes to the owner, which adds the ranks' sums into its
        gradient rows (tagged for the row-sparse Adam)."""
        comm = self.comm
        if self.ndir == 2:
            call("rg_combine_dirs", w.dX[0].data_ptr(), w.dX[1].data_ptr(), w.lsort.data_ptr(), w.offs.data_ptr(),
                 w.B, self.E, st)
        gsend = self._xbuf(w, "gsend", max(w.U, 1), self.E, torch.float32)
        call("rg_shard_dedup_grads", w.dX[0].data_ptr(), self.E, w.dd_nmax, self.N1, gsend.data_ptr(),
             w.dd_work.data_ptr(), w.dd_work.numel(), st)
        grecv = self._xbuf(w, "grecv", max(w.R, 1), self.E, torch.float32)
        w.nrecv.fill_(w.R)   # (the scatter's device row count; off the forward's gather)
        comm.all_to_all(grecv[:w.R], gsend[:w.U], w.recv_splits, w.send_splits)
        pad = self.pad - self.lo
        skip = -1 if self.train_pad or not (0 <= pad < self.n_local) else pad
        self.scatter(w.local_ids.data_ptr(), grecv.data_ptr(), self.E, w.nrecv.data_ptr(), max(w.R, 1), skip,
                     self.G_emb.data_ptr(), self.n_local, self.tags.data_ptr(), tag, st)


# ----------------------------------------------------------------- heads ----
class _HeadWS:
    def __init__(self, B, A, HF, store_z, device):
        self.B = B
        self.ldz = _round_up(B, 4)
        pb = load_library().rg_partial_block()   # items per softmax partial (32)
        self.nJ = (A + pb - 1) // pb
        z = lambda *s, dt=torch.float32: torch.empty(*s, dtype=dt, device=device)
        self.ZT = z(A, self.ldz) if store_z else None
        self.pmax = z(self.nJ, B)
        self.psum = z(self.nJ, B)
        self.parg = z(self.nJ, B, dt=torch.int32)
        S = min(128, self.nJ)
        self.work = z(3 * S * B)
        self.lse = z(B)
        self.amax = z(B, dt=torch.int32)
        self.mx = z(B)                  # row maxima (argmax path)
        self.loss_row = z(B)
        self.loss = torch.zeros(1, device=device)
        # dh kernel: ~512 workgroups of 128 rows x one item split (2 per CU)
        self.dh_splits = int(max(1, min(16, 512 // ((B + 127) // 128), A // 1024)))
        self.dh_slabs = z(self.dh_splits, B, HF) if store_z else None


class _FlashWS:
    """Workspace of the fused split-bf16 training head (csrc/head_flash.hip):
    bf16 operand planes of h and W (K- and R-layouts), the bias padded with
    -inf to whole 32-item chunks, per-(split, row) softmax partials and the
    unnormalised dh partials O (nsplit × HF × B).  zs: the logits pass 1
    stores for pass 2 (SoftmaxHead.zs_buffer; None until decided, False when
    they stay recomputed).  With top_k >= 1 pass 1 also leaves every split's
    (best logit, item) and, for top_k > 1, every 32-item chunk's row maximum
    (the fused top-k)."""

    def __init__(self, B, A, HF, device, top_k=0):
        u8 = lambda n: torch.empty(int(n), dtype=torch.uint8, device=device)  # noqa: E731
        z = lambda *s, dt=torch.float32: torch.empty(*s, dtype=dt, device=device)  # noqa: E731
        self.B, self.top_k = B, top_k
        self.terms = 0
        self.h = None
        self.wgen = -1   # generation of the head's W / b its W planes hold (SoftmaxHead._wgen)
        nrb = -(-B // call("rg_flash_rows_per_block", HF))  # row blocks of pass 1
        # about one pass-1 workgroup per CU; a multiple of 8 for the XCD order
        self.nsplit = _round_up(min(max(1, 256 // nrb), -(-A // 32)), 8)
        hb, wb = call("rg_head_plane_bytes", B, HF), call("rg_head_plane_bytes", A, HF)
        self.Hk, self.Hr, self.Wk, self.Wr = u8(hb), u8(hb), u8(wb), u8(wb)
        self.bias_pad = z(_round_up(A, 32))
        self.pm, self.pl = z(self.nsplit, B), z(self.nsplit, B)
        self.pO = z(self.nsplit, HF, B)
        self.rows = z(B, 2)
        # pass 2's split-tail partials (rg_flash_dw_work_bytes; 0 when the grid has no tail to split)
        self.dw_work_bytes = int(call("rg_flash_dw_work_bytes", B, A, HF))
        self.dw_work = u8(max(self.dw_work_bytes, 16))
        self.lse, self.zt, self.loss_row = z(B), z(B), z(B)
        self.loss = torch.zeros(1, device=device)
        self.zs = None
        self.zs_live = False   # zs holds the logits of the last pass 1 on this workspace
        self.cmax = self.cand = self.ncand = None
        if top_k >= 1:
            self.top_idx, self.top_val = z(B, top_k, dt=torch.int32), z(B, top_k)
        # chunk maxima for the exact top-K, from one buffer per device shared
        # by every head (a pass 1 with top-k outputs is consumed by its
        # top_entries on the same stream before any other head's pass 1); K = 1
        # uses them while they fit the free device memory (CMAX_FREE_MARGIN),
        # else the row-chunked screening argmax on this workspace's planes
        # (SoftmaxHead.top_entries)
        # The view is taken per pass 1 (fetch_cmax) and dropped by its top_entries, so a workspace
        # never pins an outgrown buffer.
        self.top1 = None
        self.A, self.device = A, device
        self.tk_work = None

    def fetch_cmax(self):
        """Before a pass 1 with top-k outputs: this pass's view of the shared
        chunk-maxima buffer (None: K = 1 without room, top_entries screens)."""
        A, B, K = self.A, self.B, self.top_k
        cm = _shared_cmax(self.device, -(-A // 32) * B, required=K > 1) if K >= 1 else None
        self.cmax = None if cm is None else cm.view(-(-A // 32), B)
        if self.cmax is not None and self.tk_work is None:
            self.cand = torch.empty(B, call("rg_flash_topk_cap"), dtype=torch.int32, device=self.device)
            self.ncand = torch.empty(B, dtype=torch.int32, device=self.device)
            self.tk_work = torch.empty(call("rg_flash_topk_work_bytes", B, A, K), dtype=torch.uint8,
                                       device=self.device)


# the chunk maxima of the fused heads' top-k (_FlashWS.cmax): one growing
# buffer per device; a K = 1 consumer takes it only while this much device
# memory stays free beside it (else the screening argmax runs in row chunks)
CMAX_FREE_MARGIN = 6 << 30
_CMAX = {}


def _shared_cmax(device, n, required):
    """A float tensor of at least n elements shared by every head on
    ``device`` (grown when needed), or None when K = 1 (not required) and it
    would not fit beside CMAX_FREE_MARGIN of free memory."""
    dev = torch.device(device)
    t = _CMAX.get(dev)
    if t is not None and t.numel() >= n:
        return t[:n]
    # (the buffer being outgrown is not counted as reclaimable: a view of it may still be alive)
    if not required and torch.cuda.mem_get_info(dev)[0] - 4 * n < CMAX_FREE_MARGIN:
        return None
    _CMAX.pop(dev, None)
    del t
    try:
        t = _CMAX[dev] = torch.empty(n, dtype=torch.float32, device=dev)
    except torch.cuda.OutOfMemoryError:
        if required:
            raise
        return None
    return t


# evaluation scoring (SoftmaxHead.score_topk): rows per chunk such that the
# chunk maxima (ceil(A/32) x rows floats) stay within this many bytes
EVAL_CMAX_BYTES = 1 << 30


class _ScoreWS:
    """Workspace of SoftmaxHead.score_topk for B rows and top-K: one row
    chunk's operands (R rows, R % 32 == 0) and the whole batch's outputs."""

    @staticmethod
    def get(head, slot, B, K):
        d = head.__dict__.setdefault("_sws_eval", {})
        w = d.get(slot)
        if w is None or w.B != B or w.K != K:
            d.pop(slot, None)
            w = d[slot] = _ScoreWS(B, K, head.A, head.HF, head.device)
        return w

    def __init__(self, B, K, A, HF, device):
        z = lambda *s, dt=torch.float32: torch.empty(*s, dtype=dt, device=device)  # noqa: E731
        nct = -(-A // 32)
        self.B, self.K = B, K
        rmax = max(32, EVAL_CMAX_BYTES // (4 * nct) // 32 * 32)
        self.R = R = min(_round_up(B, 32), rmax)
        nrb = -(-R // call("rg_flash_rows_per_block", HF))
        self.nsplit = _round_up(min(max(1, 256 // nrb), nct), 8)
        self.h = torch.zeros(R, HF, device=device)
        self.t = torch.zeros(R, dtype=torch.int64, device=device)
        self.Hk = torch.empty(call("rg_head_plane_bytes", R, HF), dtype=torch.uint8, device=device)
        self.pm, self.pl, self.pbest = z(self.nsplit, R), z(self.nsplit, R), z(self.nsplit, R)
        self.parg = z(self.nsplit, R, dt=torch.int32)
        self.cmax = z(nct, R)
        self.lse, self.zt = z(R), z(R)
        self.wnorm = z(1)
        self.cand = z(R, call("rg_flash_topk_cap"), dt=torch.int32)
        self.ncand = z(R, dt=torch.int32)
        self.tk_work = torch.empty(call("rg_flash_topk_work_bytes", R, A, K), dtype=torch.uint8, device=device)
        Bp = _round_up(B, R)
        self.idx, self.vals = z(Bp, K, dt=torch.int32), z(Bp, K)
        self.loss_row = z(Bp)


class _AmaxWS:
    """Workspace of the split-bf16 argmax (K-planes of h and W, per-split bests;
    with ``screen`` the chunk maxima, candidates and max row norm of the
    screening argmax)."""

    def __init__(self, B, A, HF, device, screen=False, planes=True):
        u8 = lambda n: torch.empty(int(n), dtype=torch.uint8, device=device)  # noqa: E731
        z = lambda *s, dt=torch.float32: torch.empty(*s, dtype=dt, device=device)  # noqa: E731
        self.B, self.screen = B, screen
        rpb = call("rg_flash_rows_per_block", HF)
        nct = -(-A // 32)
        # screening runs over row chunks of Bc rows (all B when the chunk maxima fit
        # SCREEN_CMAX_BYTES; else 2048-row chunks, 16 row blocks × 16 splits at HF 128)
        self.Bc = B
        if screen and nct * B * 4 > SCREEN_CMAX_BYTES:
            self.Bc = min(B, SCREEN_ROW_CHUNK)
        nrb = -(-self.Bc // rpb)
        self.nsplit = _round_up(min(max(1, 256 // nrb), nct), 8)
        self.Hk = self.Wk = self.bias_pad = None   # (planes=False: the caller's, e.g. a pass-1 workspace's)
        if planes:
            self.Hk = u8(call("rg_head_plane_bytes", B, HF))
            self.Wk = u8(call("rg_head_plane_bytes", A, HF))
            self.bias_pad = z(_round_up(A, 32))
        self.pbest, self.parg = z(self.nsplit, self.Bc), z(self.nsplit, self.Bc, dt=torch.int32)
        self.amax, self.mx = z(B, dt=torch.int32), z(B)
        if screen:
            self.cmax = z(nct, self.Bc)
            self.cand = z(B, call("rg_flash_topk_cap"), dt=torch.int32)
            self.ncand = z(B, dt=torch.int32)
            self.wnorm, self.lim = z(1), z(B)


# Head-GEMM arithmetic (build extension; the reference computes in fp32):
#   "f32"   native fp32 MFMA (v_mfma_f32_32x32x2_f32: bitwise an fmaf chain)
#   "f32x9" fp32 operands split exactly into three bf16 planes, all nine
#           plane products on bf16 MFMAs (exact products, fp32 accumulation)
#   "f32x6" the same without the three sub-ulp terms (csrc/common.h)
#   "f32x6d3" logits at f32x6; the fused head's O = P·W contraction (→ dh)
#           at the three leading plane products (its dh error stays at the
#           reference CPU fp32 path's); dW and every other GEMM
#           as f32x6
# SPLIT_TERMS: the fused full-softmax head's `terms` code (csrc/common.h
# RG_TERMS_*); LOGIT_TERMS: every logits-only split GEMM (sampled head, Q
# argmax)
SPLIT_TERMS = {"f32x9": 9, "f32x6": 6, "f32x6d3": 636}
# split-bf16 argmax (SQN / SMORL double-Q target): screening on 3 plane products, then every item
# of every 32-item chunk whose screened maximum lies within SCREEN_TOL·||h_b||·max_a||W_a|| of the
# row's best is re-scored in fp32 (first maximum).  The bound covers the dropped plane products
# (3·2^-18), fp32 accumulation of both sums (384 + 128 terms at 2^-24) on both sides, with margin
# (DESIGN §4a).  Needs ceil(A/32)·B floats of chunk maxima; above SCREEN_CMAX_BYTES the rows
# are screened in 2048-row chunks (C5 at one GPU).
SCREEN_TOL = 1e-4
# screening plane products of the double-Q argmax: 1 (the leading bf16 planes
# only: a third of the MFMA work of 3) with the wider bound SCREEN_TOL_1 =
# 2 × 3.91e-3 + margin (csrc/head_flash.hip rg_flash_amax_screen) — C4 184.6K
# -> 198.6K session-steps/s with no row past the candidate cap
# (profiles/r06/ab_c4_screen_terms.txt); 3 keeps SCREEN_TOL
SCREEN_TERMS = 1
SCREEN_TOL_1 = 8e-3
SCREEN_CMAX_BYTES = 2 << 30
SCREEN_ROW_CHUNK = 2048
# the sampled step's pre-gathered negatives (rg_gather_neg) as fp32 fragments
# the logits kernel splits itself (draw 3), not bf16 planes (draw 2), at HF <= 128
NEG_FP32_FRAGS = True
LOGIT_TERMS = {"f32x9": 9, "f32x6": 6, "f32x6d3": 6}
# HIP stream priority of the fused head's pass 2 (its side stream, §4b of
# DESIGN): pass 2 is the step's critical path, the trunk work beside it is not
PASS2_STREAM_PRIORITY = 0
# stored logits of the fused head (pass 1 writes z = S + b, pass 2 reads it
# instead of recomputing the S contraction: 21 -> 15 bf16 plane-product terms
# per step at f32x6d3): used while every head's buffers on the device together
# (ceil(A/32)·32 × B floats each, 16.4 GB at C2) stay within this budget and a
# third of the memory they and the free HBM make up (SoftmaxHead.zs_buffer)
ZSTORE_MAX_BYTES = 48 << 30
PRECISIONS = ("f32",) + tuple(SPLIT_TERMS)


def check_precision(precision):
    if precision not in PRECISIONS:
        raise ValueError(f"matmul_precision must be one of {PRECISIONS}, got {precision!r}")
    return precision


class SoftmaxHead:
    """Linear(HF→A) + CrossEntropyLoss(mean) with fused backward/Adam.
    With ``shard=(lo, hi)`` only items [lo, hi) are held (multi-GPU item
    sharding); the full init is drawn first so every rank consumes the RNG
    exactly like the single-GPU (and reference) construction."""

    _wgen = 0   # (class default: heads built with __new__, qlearn.py)
    _live = weakref.WeakSet()   # every head, for the per-device stored-logit budget

    @property
    def top_scanned(self):
        """Device int32 count of rows whose top-k / exact-argmax candidates
        overflowed the cap and were scanned whole (exact either way)."""
        t = self.__dict__.get("_top_scanned")
        if t is None:
            t = self.__dict__["_top_scanned"] = torch.zeros(1, dtype=torch.int32, device=self.device)
        return t

    def __init__(self, name, A, HF, device, shard=None):
        w, b = init_linear(HF, A)
        self.lo, self.hi = (0, A) if shard is None else shard
        self.A_full = A
        if shard is not None:
            w, b = w[self.lo:self.hi].contiguous(), b[self.lo:self.hi].contiguous()
        self.name, self.A, self.HF, self.device = name, self.hi - self.lo, HF, device
        self.precision = "f32"  # see set_matmul_precision
        # generation of W / b: bumped by every access through the W / b
        # properties (any of them may write) and by the fused pass 2; a fused
        # workspace's operand planes are current while its wgen matches
        self._wgen = 0
        self._Wp = Param(f"{name}.weight", w, device)
        self._bp = Param(f"{name}.bias", b, device)
        self._joined = True
        self._ws = {}
        self._fws = {}
        # entries of the row top-k a caller reads after forward_loss (SMORL's
        # rewards, ``top_entries``); the fused head computes them in pass 1
        self.top_k = 0
        # stored-logit top-k (rg_topk, K > 32 only) candidate overflow flag
        self.top_err = torch.zeros(1, dtype=torch.int32, device=device)
        SoftmaxHead._live.add(self)

    # W / b (and their Adam moments) are only reachable through these
    # properties, which first order the current stream after an overlapped
    # pass 2 still running on the side stream (backward_step(overlap=True)):
    # nothing can read or write the parameters before their update lands.
    @property
    def W(self):
        self.join()
        self._wgen += 1
        return self._Wp

    @W.setter
    def W(self, v):
        self.join()
        self._wgen += 1
        self._Wp = v

    @property
    def b(self):
        self.join()
        self._wgen += 1
        return self._bp

    @b.setter
    def b(self, v):
        self.join()
        self._wgen += 1
        self._bp = v

    def params_ro(self):
        """(W, b) for a read-only use on the current stream: joins like the
        properties but keeps the fused workspaces' operand planes current."""
        self.join()
        return self._Wp, self._bp

    def named_params(self):
        return [self.W, self.b]

    def set_matmul_precision(self, precision):
        self.precision = check_precision(precision)

    # ---- fused training head (csrc/head_flash.hip) ----
    def flash_terms(self, B):
        """bf16 terms of the fused training head for a batch of B rows; 0
        selects the native fp32 path that stores Zᵀ."""
        if self.precision == "f32" or self.HF not in (32, 64, 128, 256) or B % 32:
            return 0
        return SPLIT_TERMS[self.precision]

    def fws(self, slot, B):
        self.join()   # the workspace's h planes / row records are pass 2's inputs
        w = self._fws.get(slot)
        if w is None or w.B != B or w.top_k != self.top_k:
            self._fws.pop(slot, None)
            w = _FlashWS(B, self.A, self.HF, self.device, self.top_k)
            self._fws[slot] = w
        return w

    @staticmethod
    def zs_bytes_on(device):
        """Bytes of stored-logit buffers every live head holds on ``device``."""
        dev = torch.device(device)
        return sum(w.zs.numel() * 4 for h in list(SoftmaxHead._live) if torch.device(h.device) == dev
                   for w in h.__dict__.get("_fws", {}).values() if isinstance(w.zs, torch.Tensor))

    def zs_buffer(self, w):
        """The stored-logit buffer of workspace w, or None (recomputed in pass
        2).  Needs B a multiple of pass 1's row blocks (256 rows; 128 at HF 256).
        ``zstore``: None = auto, True / False force it (tests).  Auto: one
        budget for all heads of the device — the buffers already held plus
        this one within ZSTORE_MAX_BYTES and within a third of (held + free
        device memory) — so a double-Q trainer's two heads cannot pin most of
        the HBM; an allocation that fails leaves the logits recomputed."""
        mode = getattr(self, "zstore", None)
        if mode is False or w.B % call("rg_flash_rows_per_block", self.HF):
            return None
        if w.zs is None:
            nb = int(call("rg_flash_zs_bytes", w.B, self.A))
            held = self.zs_bytes_on(self.device)
            if mode is None and (held + nb > ZSTORE_MAX_BYTES
                                 or held + nb > (held + torch.cuda.mem_get_info(self.device)[0]) // 3):
                w.zs = False
            else:
                try:
                    w.zs = torch.empty(nb // 4, dtype=torch.float32, device=self.device)
                except torch.cuda.OutOfMemoryError:
                    if mode:
                        raise
                    w.zs = False
        return w.zs if w.zs is not False else None

    def release_stored_logits(self):
        """Free every workspace's stored-logit buffer (pass 2 recomputes the
        logits from then on; the next pass 1 re-decides)."""
        self.join()   # an overlapped pass 2 may still read them
        for w in self._fws.values():
            w.zs, w.zs_live = None, False

    def stored_logits(self):
        """True when a fused workspace of this head keeps its logits for pass 2."""
        return any(isinstance(w.zs, torch.Tensor) for w in self._fws.values())

    def flash_forward(self, h, tgt, slot, terms):
        """Pass 1 + this head's lse and target logit (zt = 0 when the target
        lies outside the held items [lo, hi))."""
        B, A, HF = h.shape[0], self.A, self.HF
        w = self.fws(slot, B)
        w.terms = terms
        w.h = h
        st = stream_ptr()
        Wp, bp = self.params_ro()
        W, b = Wp.p.data_ptr(), bp.p.data_ptr()
        ptr = lambda t: None if t is None else t.data_ptr()  # noqa: E731
        with region("head_fwd"):
            call("rg_head_planes", h.data_ptr(), B, HF, w.Hk.data_ptr(), w.Hr.data_ptr(), None, None, st)
            if w.wgen != self._wgen:   # else the previous pass 2 left this W's planes here
                call("rg_head_planes", W, A, HF, w.Wk.data_ptr(), w.Wr.data_ptr(), b, w.bias_pad.data_ptr(), st)
                w.wgen = self._wgen
            zs = self.zs_buffer(w)
            w.fetch_cmax()
            # top-k outputs: the chunk maxima only (top_entries re-scores the candidate chunks; without
            # them K = 1 re-screens) — no per-split first maximum
            call("rg_flash_fwd_top", w.Hk.data_ptr(), w.Wk.data_ptr(), w.Wr.data_ptr(), w.bias_pad.data_ptr(), B, A,
                 HF, terms, w.nsplit, w.pm.data_ptr(), w.pl.data_ptr(), w.pO.data_ptr(), None, None,
                 ptr(w.cmax), ptr(zs), st)
            w.zs_live = zs is not None
        call("rg_flash_lse", w.pm.data_ptr(), w.pl.data_ptr(), w.nsplit, h.data_ptr(), W, b, tgt.data_ptr(), self.lo,
             A, self.A_full, B, HF, w.lse.data_ptr(), w.zt.data_ptr(), st)
        return w

    # split-bf16 error allowance of the chunk maxima that select the top-k
    # candidates (|f32x6 - fp32| is ~1e-7 relative to sum |h||w|)
    TOP_TOL_ABS, TOP_TOL_REL = 1e-4, 1e-4

    def top_entries(self, w):
        """(idx (B, K) int32 local item ids, values (B, K)) of every row's top-K
        logits in the canonical (value desc, index asc) order, after
        forward_loss with ``top_k = K`` (reference: torch.topk of the fp32
        logits, diversity.py:15-73, novelty.py:12-47).  Fused head: the items of
        the candidate chunks (chunk maximum within the split-bf16 error of the
        K-th largest) are re-scored in fp32 (rg_flash_topk; a row past the
        candidate cap is scanned whole).  K = 1 when the chunk maxima would
        exceed SCREEN_CMAX_BYTES (C5 on one GPU): the screening argmax in row
        chunks on the planes pass 1 just read, then the same fp32 re-scoring
        (_screened_argmax).  Native head: rg_topk over the stored Zᵀ."""
        K, B = self.top_k, w.B
        st = stream_ptr()
        if isinstance(w, _FlashWS):
            if K == 1 and w.cmax is None:
                if w.top1 is None:
                    w.top1 = _AmaxWS(B, self.A, self.HF, self.device, screen=True, planes=False)
                self._screened_argmax(w.top1, w.Hk, w.Wk, w.bias_pad, w.h, self._Wp, self._bp, w.top_idx,
                                      w.top_val)
            else:
                call("rg_flash_topk", w.cmax.data_ptr(), B, B, self.A, K, _f32(self.TOP_TOL_ABS),
                     _f32(self.TOP_TOL_REL), w.h.data_ptr(), self._Wp.p.data_ptr(), self._bp.p.data_ptr(), self.HF,
                     w.cand.data_ptr(), w.ncand.data_ptr(), w.top_idx.data_ptr(), w.top_val.data_ptr(),
                     self.top_scanned.data_ptr(), w.tk_work.data_ptr(), st)
            w.cmax = None   # (consumed: the shared buffer may be regrown before the next pass 1)
            return w.top_idx, w.top_val
        idx = torch.empty(B, K, dtype=torch.int32, device=self.device)
        vals = torch.empty(B, K, device=self.device)
        call("rg_topk", w.ZT.data_ptr(), w.ldz, w.pmax.data_ptr(), B, self.A, K, idx.data_ptr(), vals.data_ptr(),
             self.top_err.data_ptr(), st)
        return idx, vals

    def _screened_argmax(self, aw, Hk, Wk, bias_pad, h, Wp, bp, out_idx, out_val, wnorm_ready=False):
        """First maximum of the fp32 logits h·Wᵀ + b per row into out_idx /
        out_val: screening on SCREEN_TERMS plane products (rows in aw.Bc chunks, so the
        chunk maxima fit SCREEN_CMAX_BYTES), then every item of every chunk
        within the screening's error bound re-scored in fp32
        (rg_flash_argmax_exact; a row past the candidate cap is scanned whole).
        wnorm_ready: aw.wnorm already holds max_a ||W_a||₂ (rg_qcomb)."""
        B, A, HF = h.shape[0], self.A, self.HF
        st = stream_ptr()
        W, b = Wp.p.data_ptr(), bp.p.data_ptr()
        if not wnorm_ready:
            call("rg_row_norm_max", W, A, HF, aw.wnorm.data_ptr(), st)
        hk_row = HF * 6   # K-plane bytes per row
        cap = call("rg_flash_topk_cap")
        for r0 in range(0, B, aw.Bc):
            bc = min(aw.Bc, B - r0)
            call("rg_flash_amax_screen", Hk.data_ptr() + r0 * hk_row, Wk.data_ptr(), bias_pad.data_ptr(), bc, A, HF,
                 aw.nsplit, SCREEN_TERMS, aw.pbest.data_ptr(), aw.parg.data_ptr(), aw.cmax.data_ptr(), st)
            call("rg_flash_argmax", aw.pbest.data_ptr(), aw.parg.data_ptr(), aw.nsplit, bc,
                 out_idx.data_ptr() + 4 * r0, out_val.data_ptr() + 4 * r0, st)
            call("rg_flash_argmax_exact", aw.cmax.data_ptr(), bc, A, h.data_ptr() + 4 * r0 * HF, W, b, HF,
                 aw.wnorm.data_ptr(), _f32(SCREEN_TOL if SCREEN_TERMS == 3 else SCREEN_TOL_1),
                 aw.lim.data_ptr() + 4 * r0,
                 aw.cand.data_ptr() + 4 * r0 * cap, aw.ncand.data_ptr() + 4 * r0,
                 out_idx.data_ptr() + 4 * r0, out_val.data_ptr() + 4 * r0, self.top_scanned.data_ptr(), st)

    # ---- evaluation scoring without logits (evaluate / update_train_metrics) ----
    def score_topk(self, h, K, tgt=None, slot="eval", screen=False):
        """Canonical top-K (value desc, index asc) of the fp32 logits h·Wᵀ + b
        of every row and, with ``tgt``, the per-row CE (lse − z_target),
        without a (B, A) logit buffer (reference eval_protocol.py:123-359
        scores the full (B, A) predictions).  Rows run in chunks of R (cmax
        ≤ EVAL_CMAX_BYTES): rg_flash_score (pass 1's S-part at 6 plane
        products: lse partials + chunk maxima), rg_flash_lse (lse, fp32
        target logit), rg_flash_topk (every item of the candidate chunks
        re-scored in fp32, fmaf chain + bias).  Returns (idx (B, K) int32,
        vals (B, K), loss_row (B,) or None); a row past the candidate cap
        (massive ties) is scanned whole (counted in ``top_scanned``).  HF must
        be in {32, 64, 128, 256}, K <= 32.  screen (no tgt): the chunk maxima
        come from the 3-product screening pass (rg_flash_amax_screen) and the
        candidates are taken within its error bound (rg_flash_topk_screened) —
        the same exact lists at half the MFMA work."""
        B, A, HF = h.shape[0], self.A, self.HF
        if K > min(32, A) or HF not in (32, 64, 128, 256):
            raise ValueError(f"score_topk: K={K} (<= 32 and <= A) and HF={HF} in {{32, 64, 128, 256}}")
        w = _ScoreWS.get(self, slot, B, K)
        st = stream_ptr()
        Wp, bp = self.params_ro()
        Wk, bias_pad = self._eval_planes(Wp, bp, st)
        R = w.R
        screen = screen and tgt is None
        if screen:
            call("rg_row_norm_max", Wp.p.data_ptr(), A, HF, w.wnorm.data_ptr(), st)
        for r0 in range(0, B, R):
            n = min(R, B - r0)
            hs = w.h if n < R else h[r0:r0 + R]
            if n < R:   # ragged tail: zero-padded rows (pass 1 scores them; the top-k takes only the n real rows)
                w.h.zero_()
                w.h[:n].copy_(h[r0:r0 + n])
            call("rg_head_planes", hs.data_ptr(), R, HF, w.Hk.data_ptr(), None, None, None, st)
            if screen:
                call("rg_flash_amax_screen", w.Hk.data_ptr(), Wk.data_ptr(), bias_pad.data_ptr(), R, A, HF, w.nsplit,
                     3, w.pbest.data_ptr(), w.parg.data_ptr(), w.cmax.data_ptr(), st)
                call("rg_flash_topk_screened", w.cmax.data_ptr(), R, n, A, K, _f32(SCREEN_TOL), w.wnorm.data_ptr(),
                     hs.data_ptr(), Wp.p.data_ptr(), bp.p.data_ptr(), HF, w.cand.data_ptr(), w.ncand.data_ptr(),
                     w.idx.data_ptr() + 4 * r0 * K, w.vals.data_ptr() + 4 * r0 * K, self.top_scanned.data_ptr(),
                     w.tk_work.data_ptr(), st)
                continue
            call("rg_flash_score", w.Hk.data_ptr(), Wk.data_ptr(), bias_pad.data_ptr(), R, A, HF, 6, w.nsplit,
                 w.pm.data_ptr(), w.pl.data_ptr(), w.pbest.data_ptr(), w.parg.data_ptr(), w.cmax.data_ptr(), st)
            if tgt is not None:
                ts = w.t if n < R else tgt[r0:r0 + R]
                if n < R:
                    w.t.zero_()
                    w.t[:n].copy_(tgt[r0:r0 + n])
                call("rg_flash_lse", w.pm.data_ptr(), w.pl.data_ptr(), w.nsplit, hs.data_ptr(), Wp.p.data_ptr(),
                     bp.p.data_ptr(), ts.data_ptr(), 0, A, A, R, HF, w.lse.data_ptr(), w.zt.data_ptr(), st)
                call("rg_sub", w.lse.data_ptr(), w.zt.data_ptr(), n, w.loss_row.data_ptr() + 4 * r0, st)
            call("rg_flash_topk", w.cmax.data_ptr(), R, n, A, K, _f32(self.TOP_TOL_ABS), _f32(self.TOP_TOL_REL),
                 hs.data_ptr(), Wp.p.data_ptr(), bp.p.data_ptr(), HF, w.cand.data_ptr(), w.ncand.data_ptr(),
                 w.idx.data_ptr() + 4 * r0 * K, w.vals.data_ptr() + 4 * r0 * K, self.top_scanned.data_ptr(),
                 w.tk_work.data_ptr(), st)
        return w.idx[:B], w.vals[:B], (w.loss_row[:B] if tgt is not None else None)

    def _eval_planes(self, Wp, bp, st):
        """W's K-planes and padded bias for the current W: a training
        workspace's (pass 2 left them current) when one matches, else the
        head's own evaluation copy, rebuilt when W changed."""
        for fw in self._fws.values():
            if fw.wgen == self._wgen:
                return fw.Wk, fw.bias_pad
        ep = getattr(self, "_eplanes", None)
        if ep is None or ep[0] != self._wgen:
            Wk = ep[1] if ep is not None else torch.empty(call("rg_head_plane_bytes", self.A, self.HF),
                                                           dtype=torch.uint8, device=self.device)
            bias_pad = ep[2] if ep is not None else torch.empty(_round_up(self.A, 32), device=self.device)
            call("rg_head_planes", Wp.p.data_ptr(), self.A, self.HF, Wk.data_ptr(), None, bp.p.data_ptr(),
                 bias_pad.data_ptr(), st)
            ep = self._eplanes = (self._wgen, Wk, bias_pad)
        return ep[1], ep[2]

    def release_eval(self):
        """Drop the evaluation workspaces (row-chunk buffers, W planes copy)."""
        self._eplanes = None
        getattr(self, "_sws_eval", {}).clear()

    def check_top_err(self):
        """Raise if a stored-logit top-k with K > 32 (rg_topk) of this head
        overflowed its candidate buffer since the last check (massive exact
        ties); every other top-k path scans such a row whole instead."""
        if int(self.top_err.item()):
            self.top_err.zero_()
            raise RuntimeError(f"{self.name}: top-k candidate overflow (massive ties in the logits)")

    def flash_dh(self, w, tgt, lse, g, dh_out):
        """dh_out := this head's ∂loss/∂h given the (all-rank) lse."""
        st = stream_ptr()
        call("rg_flash_rows", lse.data_ptr(), tgt.data_ptr(), self.lo, self.A, w.B, w.rows.data_ptr(), st)
        with region("head_dh"):
            call("rg_flash_dh", w.pm.data_ptr(), w.pO.data_ptr(), w.rows.data_ptr(), w.nsplit,
                 self.params_ro()[0].p.data_ptr(), g, w.B, self.HF, dh_out.data_ptr(), st)

    def join(self):
        """Order the current stream after an overlapped pass 2 (backward_step(overlap=True))."""
        if not getattr(self, "_joined", True):   # (heads built with __new__ never overlap)
            self._joined = True
            torch.cuda.current_stream(self.device).wait_stream(self._side)

    def flash_dw_adam_async(self, w, g, adam6):
        """Pass 2 on this head's side stream, ordered after everything issued so
        far; the head joins it on the next access of W / b or its workspace."""
        if getattr(self, "_side", None) is None:
            self._side = torch.cuda.Stream(device=self.device, priority=PASS2_STREAM_PRIORITY)
        self._side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(self._side):
            self.flash_dw_adam(w, g, adam6)
        self._joined = False

    def flash_dw_adam(self, w, g, adam6):
        """Pass 2: dW, db and the Adam step of W / b (after flash_dh); the
        updated W / b also leave as this workspace's operand planes and padded
        bias (the next flash_forward on it skips rg_head_planes for W)."""
        Wp, bp = self._Wp, self._bp   # not the joining properties: this may run on the side stream
        with region("head_dw_adam"):
            call("rg_flash_dw_adam_planes", w.Hk.data_ptr(), w.Hr.data_ptr(), w.Wk.data_ptr(),
                 w.bias_pad.data_ptr(), w.rows.data_ptr(), g, w.B, self.A, self.HF, w.terms, Wp.p.data_ptr(),
                 Wp.m.data_ptr(), Wp.v.data_ptr(), bp.p.data_ptr(), bp.m.data_ptr(), bp.v.data_ptr(), adam6, None,
                 None, w.Wk.data_ptr(), w.Wr.data_ptr(), w.bias_pad.data_ptr(), w.dw_work.data_ptr(),
                 w.dw_work_bytes, w.zs.data_ptr() if w.zs_live else None, stream_ptr())
        w.zs_live = False
        self._wgen += 1
        w.wgen = self._wgen

    def ws(self, slot, B, store_z):
        key = (slot, B, store_z)
        w = self._ws.get(key)
        if w is None:
            for k in [k for k in self._ws if k[0] == slot]:
                del self._ws[k]
            w = _HeadWS(B, self.A, self.HF, store_z, self.device)
            self._ws[key] = w
        return w

    def logits_T(self, h, slot=None):
        """Zᵀ (A × ldz) for h; returns (workspace, the (B, A) logical view, no
        copy).  slot=None: a fresh buffer owned by the returned tensors (the
        model's forward(), for callers that index the logits — freed when they
        drop it); a named slot keeps it cached in the head."""
        B = h.shape[0]
        w = self.ws(slot, B, True) if slot is not None else _HeadWS(B, self.A, self.HF, True, self.device)
        Wp, bp = self.params_ro()
        call("rg_head_fwd", h.data_ptr(), Wp.p.data_ptr(), bp.p.data_ptr(), B, self.A, self.HF,
             w.ZT.data_ptr(), w.ldz, w.pmax.data_ptr(), w.psum.data_ptr(), w.parg.data_ptr(), 1, stream_ptr())
        return w, w.ZT[:, :B].t()

    def forward_loss(self, h, tgt, slot="main", h_planes=None):
        """CE(mean) of Z = h·Wᵀ + b against tgt; keeps Zᵀ / lse for backward.
        Returns the device loss tensor (1,) and the workspace.  (h_planes:
        used by the sampled head only.)"""
        B = h.shape[0]
        st = stream_ptr()
        terms = self.flash_terms(B)
        if terms:  # fused split-bf16 head: no logits stored
            w = self.flash_forward(h, tgt, slot, terms)
            call("rg_sub", w.lse.data_ptr(), w.zt.data_ptr(), B, w.loss_row.data_ptr(), st)
            call("rg_sum_scale", w.loss_row.data_ptr(), B, _f32(1.0 / B), w.loss.data_ptr(), None, st)
            return w.loss, w
        w = self.ws(slot, B, True)
        with region("head_fwd"):
            call("rg_head_fwd", h.data_ptr(), self.W.p.data_ptr(), self.b.p.data_ptr(), B, self.A, self.HF,
                 w.ZT.data_ptr(), w.ldz, w.pmax.data_ptr(), w.psum.data_ptr(), w.parg.data_ptr(), 1, st)
        call("rg_lse_combine", w.pmax.data_ptr(), w.psum.data_ptr(), w.parg.data_ptr(), B, w.nJ, w.work.data_ptr(),
             w.ZT.data_ptr(), w.ldz, tgt.data_ptr(), self.A, w.lse.data_ptr(), w.amax.data_ptr(),
             w.loss_row.data_ptr(), None, st)
        call("rg_sum_scale", w.loss_row.data_ptr(), B, _f32(1.0 / B), w.loss.data_ptr(), None, st)
        return w.loss, w

    def backward_step(self, h, tgt, dh_out, adam6, slot="main", gscale=None, overlap=False):
        """dh_out (B, HF) := ∂loss/∂h (overwrites); then the fused dW/db + Adam.
        overlap (fused head): pass 2 runs on a side stream, so the caller's
        trunk backward (which needs only dh) fills the CUs pass 2's last,
        partial round of workgroups leaves idle; the caller must ``join()``
        before anything reads W / b again."""
        B = h.shape[0]
        g = _f32(1.0 / B) if gscale is None else gscale
        if self.flash_terms(B):
            w = self.fws(slot, B)
            self.flash_dh(w, tgt, w.lse, g, dh_out)
            if overlap:   # joined lazily: by the next access of W / b or of the workspace
                self.flash_dw_adam_async(w, g, adam6)
            else:
                self.flash_dw_adam(w, g, adam6)
            return
        w = self.ws(slot, B, True)
        st = stream_ptr()
        with region("head_dh"):
            n = call("rg_head_dh", w.ZT.data_ptr(), w.ldz, w.lse.data_ptr(), tgt.data_ptr(), g, self.W.p.data_ptr(),
                     B, self.A, self.HF, w.dh_splits, w.dh_slabs.data_ptr(), st)
        call("rg_reduce_slabs", w.dh_slabs.data_ptr(), n, B * self.HF, dh_out.data_ptr(), None, self.HF, 0, st)
        with region("head_dw_adam"):
            call("rg_head_dw_adam", w.ZT.data_ptr(), w.ldz, w.lse.data_ptr(), tgt.data_ptr(), g, h.data_ptr(), B,
                 self.A, self.HF, self.W.p.data_ptr(), self.W.m.data_ptr(), self.W.v.data_ptr(),
                 self.b.p.data_ptr(), self.b.m.data_ptr(), self.b.v.data_ptr(), adam6, None, None, st)

    def amax_ws(self, slot, B):
        """The screening-argmax workspace of ``slot`` for B rows."""
        w = self._aws.get(slot) if hasattr(self, "_aws") else None
        if w is None or w.B != B:
            if not hasattr(self, "_aws"):
                self._aws = {}
            self._aws.pop(slot, None)
            w = self._aws[slot] = _AmaxWS(B, self.A, self.HF, self.device, True)
        return w

    def argmax(self, h, slot="argmax", planes_ready=False):
        """argmax_j (h·Wᵀ + b)[b, j] without storing Z (first maximum); the
        row maxima are left in ``self.argmax_mx``.  With a split-bf16
        precision the contraction runs on bf16 MFMAs (csrc/head_flash.hip
        k_flash_amax: pass 1's S-part with first-maximum tracking).
        planes_ready: the slot's workspace already holds W's K-planes, padded
        bias and max row norm (QNet.argmax_q's rg_qcomb)."""
        B = h.shape[0]
        st = stream_ptr()
        terms = self.flash_terms(B)
        if terms:
            # screening (3 plane products) + exact fp32 re-scoring of the
            # chunks within the error bound (rows in chunks when the chunk
            # maxima would not fit SCREEN_CMAX_BYTES)
            w = self.amax_ws(slot, B)
            Wp, bp = self.W, self.b
            call("rg_head_planes", h.data_ptr(), B, self.HF, w.Hk.data_ptr(), None, None, None, st)
            if not planes_ready:
                call("rg_head_planes", Wp.p.data_ptr(), self.A, self.HF, w.Wk.data_ptr(), None, bp.p.data_ptr(),
                     w.bias_pad.data_ptr(), st)
            self._screened_argmax(w, w.Hk, w.Wk, w.bias_pad, h, Wp, bp, w.amax, w.mx, wnorm_ready=planes_ready)
            self.argmax_mx = w.mx
            return w.amax
        w = self.ws(slot, B, False)
        self.argmax_mx = w.mx
        call("rg_head_fwd", h.data_ptr(), self.W.p.data_ptr(), self.b.p.data_ptr(), B, self.A, self.HF, None, 0,
             w.pmax.data_ptr(), w.psum.data_ptr(), w.parg.data_ptr(), 0, st)
        call("rg_lse_combine", w.pmax.data_ptr(), w.psum.data_ptr(), w.parg.data_ptr(), B, w.nJ, w.work.data_ptr(),
             None, 0, None, self.A, None, w.amax.data_ptr(), None, w.mx.data_ptr(), st)
        return w.amax


# --------------------------------------------------------- sampled head ----
class _SampledWS:
    def __init__(self, B, S, HF, device, terms=0):
        z = lambda *s, dt=torch.float32: torch.empty(*s, dtype=dt, device=device)
        self.B, self.S = B, S
        self.terms = terms  # 0: native fp32 forward, 6 / 9: split-bf16 (rg_sampled_logits / rg_sampled_fwd_x)
        self.nT = call("rg_sampled_nparts", B, S, terms)  # (max, Σexp) partials per row
        # logits layout: the fused one-launch split forward (csrc/sampled.hip
        # k_sampled_logits, HF <= 256) stores Z row-major (B × ldz, negatives
        # contiguous); the native fp32 forward stores Zᵀ (S × ldz, rows contiguous)
        self.zrow = terms != 0 and HF <= 256
        self.ldz = _round_up(S, 4) if self.zrow else _round_up(B, 4)
        self.ZT = z(B, self.ldz) if self.zrow else z(S, self.ldz)
        # (stride over batch rows, stride over negatives) of the logits
        self.zs_b, self.zs_s = (self.ldz, 1) if self.zrow else (1, self.ldz)
        self.dbslabs = z((B + 127) // 128, S)
        self.pmax = z(self.nT, B)
        self.psum = z(self.nT, B)
        self.lse = z(B)
        self.loss_row = z(B)
        self.loss = torch.zeros(1, device=device)
        # scatter lists: rows [0, S) = the negatives, [S, S+B) = the targets
        self.ids = z(S + B, dt=torch.int32)
        self.grows = z(S + B, HF)       # ∂/∂W rows
        self.gb = z(S + B)              # ∂/∂bias entries
        self.nrows = torch.full((1,), S + B, dtype=torch.int32, device=device)
        self.Wg = z(S, HF)
        self.bg = z(S)
        self.Wp = None    # the negatives' bf16 planes from rg_gather_neg (allocated on first use)
        self.pre_draw = -1   # draw index whose ids / bg / Wg / Wp the gather launch already wrote
        self.pre_fmt = 0     # Wp's format then (rg_gather_neg wfmt)
        self.work = None  # split-bf16 operand planes (allocated on first use)
        self.dh_splits = max(1, min(8, S // 256))
        self.dw_splits = max(1, min(16, B // 256))
        # slab 0 = the positive part of dh (written by rg_sampled_lse)
        self.dh_slabs = z(self.dh_splits + 1, B, HF)
        self.dw_slabs = z(self.dw_splits, S, HF)


class SampledSoftmaxHead(SoftmaxHead):
    """Linear(HF→A) trained with a sampled softmax: CE over the target and
    ``n_neg`` negatives shared by the batch, drawn uniformly with replacement
    from a counter-based stream (``seed``, draw index) — csrc/sampled.hip.
    Build-defined (SURVEY §8 A7 ext., config C3); evaluation (``logits_T``,
    ``argmax``) still scores every item.  Same parameters, init order and
    state_dict keys as SoftmaxHead; Adam stays dense (rows the step did not
    touch see g = 0, as torch.optim.Adam would)."""

    LOSSES = ("ce", "bpr")

    def __init__(self, name, A, HF, device, n_neg, seed=0, loss="ce", shard=None):
        if HF % 32 or HF > 256:
            raise ValueError(f"sampled softmax needs head width in {{32, 64, 128, 256}}, got {HF}")
        if n_neg <= 0:
            raise ValueError("n_negatives must be positive")
        if loss not in self.LOSSES:
            raise ValueError(f"sampled loss must be one of {self.LOSSES}, got {loss!r}")
        super().__init__(name, A, HF, device, shard=shard)
        # "ce": CE over [target ‖ negatives]; "bpr": mean_s −log σ(z_pos − z_neg_s)
        self.loss = loss
        self.S = int(n_neg)
        self.seed = int(seed) & (2**64 - 1)
        self.draws = 0
        self.G = torch.zeros_like(self._Wp.p)
        self.Gb = torch.zeros_like(self._bp.p)
        self.tags = torch.zeros(self.A, dtype=torch.int32, device=device)
        self.tag = 0
        self.scatter = SegScatter(device)
        self._sws = {}
        # catch-up Adam of W / b (one GPU; the item-sharded head keeps the eager sweeps): a
        # step's targets and negatives are caught up before they are read (prepare_rows),
        # every row before any other read — the W / b properties, named_params, evaluation
        self.lazy = LazyRows(self.A, device) if LAZY_ADAM and shard is None else None
        self._ready_draw = -1
        self._neg_draw = -1   # the draw whose negatives catch_up_async already queued

    # the step's own kernels use _Wp / _bp (their rows are caught up by
    # prepare_rows); every other access goes through these properties
    @property
    def W(self):
        self.materialize()
        return SoftmaxHead.W.fget(self)

    @W.setter
    def W(self, v):
        SoftmaxHead.W.fset(self, v)

    @property
    def b(self):
        self.materialize()
        return SoftmaxHead.b.fget(self)

    @b.setter
    def b(self, v):
        SoftmaxHead.b.fset(self, v)

    def params_ro(self):
        self.materialize()
        return SoftmaxHead.params_ro(self)

    def _lazy_tab(self):
        W, b = self._Wp, self._bp
        return (W.p.data_ptr(), W.m.data_ptr(), W.v.data_ptr(), self.HF, None, b.p.data_ptr(), b.m.data_ptr(),
                b.v.data_ptr())

    def materialize(self):
        lz = self.__dict__.get("lazy")
        if lz is not None:
            lz.materialize(self._lazy_tab())

    def prepare_rows(self, tgt, B, early=False):
        """Catch up the rows the next forward_loss reads: its B targets (device
        int64) and the S negatives of draw ``self.draws``.  ``early`` (neg_job,
        before the trunk's forward): when the negatives were already caught up
        by the last backward, the targets' catch-up goes to the side stream
        and runs beside the trunk's forward; forward_loss joins it."""
        if self.lazy is not None and self._ready_draw != self.draws:
            S = 0 if self._neg_draw == self.draws else self.S   # (the negatives: queued by the last backward)
            if early and S == 0 and TARGETS_ASYNC:
                self.lazy.catch_up_async(self._lazy_tab(), 0, 0, 0, ids=tgt.data_ptr(), n_ids=B)
            else:
                self.lazy.catch_up(self._lazy_tab(), tgt.data_ptr(), B, self.seed, self.draws, S)
            self._ready_draw = self.draws

    @staticmethod
    def _dz_gemms(w, h, B, S, HF, st):
        """dh slabs 1.. = dZ · Wg and dw slabs = dZᵀ · h (split-K): at a split
        precision on the bf16 planes of exact 3-way splits (rg_gemm_x6_sk, 6 or
        9 products, the logits' arithmetic), else fp32 MFMA (rg_gemm_f32)."""
        if w.terms and w.zrow:
            t = 9 if w.terms == 9 else 6
            call("rg_gemm_x6_sk", w.ZT.data_ptr(), w.ldz, 1, w.Wg.data_ptr(), HF, 0,
                 w.dh_slabs.data_ptr() + 4 * B * HF, HF, B * HF, B, HF, S, w.dh_splits, t, st)
            call("rg_gemm_x6_sk", w.ZT.data_ptr(), w.ldz, 0, h.data_ptr(), HF, 0, w.dw_slabs.data_ptr(), HF, S * HF,
                 S, HF, B, w.dw_splits, t, st)
        else:
            call("rg_gemm_f32", w.ZT.data_ptr(), w.zs_b, w.zs_s, w.Wg.data_ptr(), HF, 1,
                 w.dh_slabs.data_ptr() + 4 * B * HF, HF, None, B, None, HF, S, None, w.dh_splits, st)
            call("rg_gemm_f32", w.ZT.data_ptr(), w.zs_s, w.zs_b, h.data_ptr(), HF, 1, w.dw_slabs.data_ptr(), HF, None,
                 S, None, HF, B, None, w.dw_splits, st)

    def split_terms(self, B):
        """bf16 terms of the forward for batch B (0: native fp32 MFMA)."""
        if self.precision == "f32" or B % 32 or self.S % 32:
            return 0
        return LOGIT_TERMS[self.precision]

    def sws(self, slot, B):
        w = self._sws.get(slot)
        terms = self.split_terms(B)
        if w is None or w.B != B or w.terms != terms:
            w = _SampledWS(B, self.S, self.HF, self.device, terms)
            self._sws[slot] = w
        return w

    def neg_job(self, slot, B, tgt=None):
        """The negatives' row gather of the next forward_loss(slot, B), to run
        inside the trunk's embedding-gather launch (Trunk.neg_job ->
        rg_gather_neg): ids, biases, rows and their fragment-order bf16 planes
        of draw ``self.draws``.  None where the one-launch split logits do not
        run (native fp32 forward).  ``tgt``: the step's targets, whose rows (and
        the negatives') are caught up here, before the trunk's gather launch
        reads the negatives (catch-up Adam)."""
        if tgt is not None:
            self.prepare_rows(tgt, B, early=True)
        w = self.sws(slot, B)
        if w.terms == 0 or not w.zrow:
            return None
        if w.Wp is None:
            w.Wp = torch.empty(self.S * self.HF * 6, dtype=torch.uint8, device=self.device)
        head, draw = self, self.draws
        wfmt = 1 if NEG_FP32_FRAGS and self.HF <= 128 else 0

        class _Job:
            @staticmethod
            def args():
                return (head._Wp.p.data_ptr(), head._bp.p.data_ptr(), head.seed, draw, head.A, head.S, head.HF,
                        w.ids.data_ptr(), w.Wg.data_ptr(), w.bg.data_ptr(), w.Wp.data_ptr(), wfmt)

            @staticmethod
            def done():
                w.pre_draw = draw
                w.pre_fmt = wfmt
        return _Job()

    def forward_loss(self, h, tgt, slot="main", h_planes=None):
        """h_planes: h's bf16 K-planes from the GRU forward (Trunk.emit_planes),
        consumed by the one-launch split logits at HF <= 128.  When the trunk's
        gather launch already gathered this draw's negatives (neg_job), the
        logits read their planes (draw = 2)."""
        B = h.shape[0]
        self.prepare_rows(tgt, B)   # (a no-op when neg_job already did it for this draw)
        if self.lazy is not None:
            self.lazy.join()        # (the targets' catch-up queued by neg_job on the side stream)
        w = self.sws(slot, B)
        st = stream_ptr()
        g = _f32(1.0 / B)
        split = w.terms != 0
        pre = w.pre_draw == self.draws
        W, bb = (self._Wp, self._bp) if self.lazy is not None else (self.W, self.b)
        w.pre_draw = -1
        # the negatives' row gather is part of the timed logits step (or of the
        # gather launch, pre); with the one-launch kernel the region is kernel-exact
        with region("sampled_fwd", exact=bool(split and w.zrow)):
            if split and w.zrow:  # one launch: [draw, row gather, operand split,] logits, partials
                hp = h_planes.data_ptr() if h_planes is not None else None
                call("rg_sampled_logits", h.data_ptr(), W.p.data_ptr(), bb.p.data_ptr(), w.ids.data_ptr(),
                     (3 if w.pre_fmt else 2) if pre else 1, self.seed, self.draws, self.A, B, self.S, self.HF, w.terms, w.ZT.data_ptr(),
                     w.ldz, w.pmax.data_ptr(), w.psum.data_ptr(), w.Wg.data_ptr(), w.bg.data_ptr(), hp,
                     w.Wp.data_ptr() if pre else None, st)
            elif split:  # draw + gather + operand split fused into one prep launch
                if w.work is None:
                    w.work = torch.empty(call("rg_sampled_work_bytes", B, self.S, self.HF), dtype=torch.uint8,
                                         device=self.device)
                call("rg_sampled_fwd_x", h.data_ptr(), W.p.data_ptr(), bb.p.data_ptr(), w.ids.data_ptr(),
                     1, self.seed, self.draws, self.A, B, self.S, self.HF, w.terms,
                     w.ZT.data_ptr(), w.ldz, w.pmax.data_ptr(), w.psum.data_ptr(), w.Wg.data_ptr(),
                     w.bg.data_ptr(), w.work.data_ptr(), st)
            else:
                call("rg_sample_uniform", self.seed, self.draws, self.S, self.A, w.ids.data_ptr(), st)
                call("rg_sampled_fwd", h.data_ptr(), W.p.data_ptr(), bb.p.data_ptr(), w.ids.data_ptr(),
                     B, self.S, self.HF, w.ZT.data_ptr(), w.ldz, w.pmax.data_ptr(), w.psum.data_ptr(),
                     w.Wg.data_ptr(), w.bg.data_ptr(), st)
        self.draws += 1
        if self.loss == "bpr":   # w.lse holds z_pos for the backward
            call("rg_bpr_rows", h.data_ptr(), W.p.data_ptr(), bb.p.data_ptr(), tgt.data_ptr(), B, self.A,
                 self.HF, w.ZT.data_ptr(), w.zs_b, w.zs_s, self.S, g, w.lse.data_ptr(), w.loss_row.data_ptr(),
                 w.ids.data_ptr() + 4 * self.S, w.gb.data_ptr() + 4 * self.S,
                 w.grows.data_ptr() + 4 * self.S * self.HF, w.dh_slabs.data_ptr(), st)
        else:
            call("rg_sampled_lse", h.data_ptr(), W.p.data_ptr(), bb.p.data_ptr(), tgt.data_ptr(), B,
                 self.A, self.HF, w.pmax.data_ptr(), w.psum.data_ptr(), w.nT, g, w.lse.data_ptr(),
                 w.loss_row.data_ptr(), w.ids.data_ptr() + 4 * self.S, w.gb.data_ptr() + 4 * self.S,
                 w.grows.data_ptr() + 4 * self.S * self.HF, w.dh_slabs.data_ptr(), st)
        call("rg_sum_scale", w.loss_row.data_ptr(), B, g, w.loss.data_ptr(), None, st)
        return w.loss, w

    def backward_step(self, h, tgt, dh_out, adam6, slot="main", gscale=None, overlap=False):
        B = h.shape[0]   # (overlap: no side-stream pass here; the sampled backward is short)
        w = self.sws(slot, B)
        st = stream_ptr()
        S, HF = self.S, self.HF
        g = _f32(1.0 / B)
        if gscale is not None and gscale != g:
            raise NotImplementedError("sampled softmax: the loss scale is fixed at 1/B (set in forward_loss)")
        with region("sampled_bwd"):
            if self.loss == "bpr":
                call("rg_bpr_dz", w.ZT.data_ptr(), w.zs_b, w.zs_s, w.lse.data_ptr(), B, S, g, w.dbslabs.data_ptr(),
                     w.gb.data_ptr(), st)
            elif w.zrow:
                call("rg_sampled_dz_rows", w.ZT.data_ptr(), w.ldz, w.lse.data_ptr(), B, S, g, w.dbslabs.data_ptr(),
                     w.gb.data_ptr(), st)
            else:
                call("rg_sampled_dz", w.ZT.data_ptr(), w.ldz, w.lse.data_ptr(), B, S, g, w.gb.data_ptr(), st)
            # dh = dZ · Wg (+ the positive part already in slab 0); dWg = dZᵀ · h -> rows [0, S) of the
            # scatter list.  Split precisions: the logits' split-bf16 planes (rg_gemm_x6_sk), else fp32 MFMA
            self._dz_gemms(w, h, B, S, HF, st)
            call("rg_reduce_slabs", w.dh_slabs.data_ptr(), w.dh_splits + 1, B * HF, dh_out.data_ptr(), None, HF, 0,
                 st)
            call("rg_reduce_slabs", w.dw_slabs.data_ptr(), w.dw_splits, S * HF, w.grows.data_ptr(), None, HF, 0,
                 st)
            self.tag += 1
            self.scatter(w.ids.data_ptr(), w.grows.data_ptr(), HF, w.nrows.data_ptr(), S + B, -1, self.G.data_ptr(),
                         self.A, self.tags.data_ptr(), self.tag, st)
            self.scatter(w.ids.data_ptr(), w.gb.data_ptr(), 1, w.nrows.data_ptr(), S + B, -1, self.Gb.data_ptr(),
                         self.A, self.tags.data_ptr(), self.tag, st, reuse_sort=True)
        with region("sampled_adam"):
            if self.lazy is not None:   # the touched rows only (catch-up Adam)
                self.lazy.adam(self._lazy_tab(), self.G.data_ptr(), self.Gb.data_ptr(), self.tags.data_ptr(),
                               self.tag, adam6)
                if PREFETCH_NEGATIVES:   # the next draw's negatives, caught up under the rest of the step
                    self.lazy.catch_up_async(self._lazy_tab(), self.seed, self.draws, self.S)
                    self._neg_draw = self.draws
                return
            call("rg_adam_rows", self.W.p.data_ptr(), self.W.m.data_ptr(), self.W.v.data_ptr(), self.G.data_ptr(),
                 self.tags.data_ptr(), self.tag, self.A, HF, adam6, st)
            call("rg_adam_rows", self.b.p.data_ptr(), self.b.m.data_ptr(), self.b.v.data_ptr(), self.Gb.data_ptr(),
                 self.tags.data_ptr(), self.tag, self.A, 1, adam6, st)


class ShardedSampledHead(SampledSoftmaxHead):
    """SampledSoftmaxHead item-sharded over the ranks (multi-GPU; SURVEY §8e,
    csrc/sampled_shard.hip): this rank holds output rows [lo, hi) and their
    Adam moments and trains its own B session rows of the global batch.  Rows
    move to the data, never logits or an item-sized gradient:

      forward   the S shared negatives (the same counter-based draw on every
                rank): each rank writes the rows it owns, one SUM all-reduce
                of S·(HF+1) floats (1 MB at HF 128, S 2048) gives every rank
                all of them, cut into the logits' bf16 planes; the rank's
                targets' rows come from their owners by all-to-all; then the
                one-launch split logits and the CE exactly as on one GPU
      backward  dZ, dh local; the negatives' row gradients (summed over the
                rank's rows) SUM all-reduced, each owner scatters the rows it
                holds; the targets' row gradients go back to their owners by
                all-to-all; row-sparse dense-semantics Adam on the local rows.

    The loss is the mean over all world·B rows (gscale = 1/(world·B)), the
    one-GPU step on the concatenated batch up to fp32 summation order."""

    def __init__(self, name, A, HF, device, n_neg, seed, loss, comm, shard):
        if loss != "ce":
            raise NotImplementedError("item-sharded sampled head: the CE loss only")
        super().__init__(name, A, HF, device, n_neg, seed, loss, shard=shard)
        self.comm = comm

    def neg_job(self, slot, B, tgt=None):
        return None   # the negatives' rows come from their owners (forward_loss)

    def sws(self, slot, B):
        w = super().sws(slot, B)
        if getattr(w, "wgb", None) is None:
            S, HF, dev = self.S, self.HF, self.device
            z = lambda *sh, dt=torch.float32: torch.empty(*sh, dtype=dt, device=dev)  # noqa: E731
            w.wgb = z(S * HF + S)   # the negatives' rows and biases, one all-reduce
            w.Wg, w.bg = w.wgb[:S * HF].view(S, HF), w.wgb[S * HF:]
            w.Wp = torch.empty(S * HF * 6, dtype=torch.uint8, device=dev)
            w.nloc = z(S, dt=torch.int32)
            w.nS = torch.full((1,), S, dtype=torch.int32, device=dev)
            w.troute = z(3 * B, dt=torch.int32)   # t32 | slot | send (one host → device copy)
            w.t32, w.tslot, w.tsend = w.troute[:B], w.troute[B:2 * B], w.troute[2 * B:]
            w.nt = z(1, dt=torch.int32)
            from .dist import HostStage
            w.tstage = HostStage()
            w.tcounts = z(self.comm.world, dt=torch.int32)
            w.tW, w.tb = z(B, HF), z(B)
            w.trow = z(B, dt=torch.int64)
            w.nR = torch.zeros(1, dtype=torch.int32, device=dev)
            w.gsend = z(B, HF + 4)   # target row + bias gradients, one all-to-all
            w.xb = {}
        return w

    def _xb(self, w, name, rows, cols=None, dtype=torch.float32):
        """Exchange buffer of at least ``rows`` rows (grown ×1.25 when needed)."""
        t = w.xb.get(name)
        if t is None or t.shape[0] < rows:
            n = max(16, int(rows * 1.25))
            t = w.xb[name] = torch.empty((n,) if cols is None else (n, cols), dtype=dtype, device=self.device)
        return t

    def forward_loss(self, h, tgt, slot="main", h_planes=None, gscale=None, route=None):
        """route: the targets' (send_splits, recv_splits) from the host batch
        (dist.host_routes); None routes on the device and reads the counts back."""
        B = h.shape[0]
        w = self.sws(slot, B)
        if w.terms == 0 or not w.zrow:
            raise NotImplementedError("item-sharded sampled head: split-bf16 logits only (B % 32 == 0, "
                                      "S % 32 == 0, a split matmul_precision)")
        comm, st = self.comm, stream_ptr()
        S, HF = self.S, self.HF
        g = _f32(1.0 / B) if gscale is None else gscale
        W, b = self.W.p.data_ptr(), self.b.p.data_ptr()
        with region("neg_exchange"):
            call("rg_neg_pick", self.seed, self.draws, self.A_full, S, HF, self.lo, self.hi, W, b, w.ids.data_ptr(),
                 w.nloc.data_ptr(), w.Wg.data_ptr(), w.bg.data_ptr(), st)
            comm.all_reduce(w.wgb)
            call("rg_neg_planes", w.Wg.data_ptr(), S, HF, w.Wp.data_ptr(), st)
            # the rank's targets' rows and biases from their owners
            plan = route[2] if route is not None and len(route) > 2 else None
            if plan is not None:   # t32 | slot | send from the host batch (dist.target_route)
                w.tstage.to_device(plan, w.troute)
            else:
                call("rg_target_ids", tgt.data_ptr(), B, self.A_full, w.t32.data_ptr(), w.nt.data_ptr(), st)
                call("rg_shard_route", w.t32.data_ptr(), w.nt.data_ptr(), self.A_full, comm.world,
                     w.tslot.data_ptr(), w.tsend.data_ptr(), w.tcounts.data_ptr(), st)
            if route is not None:
                w.send_splits, w.recv_splits = list(route[0]), list(route[1])
            else:
                allc = torch.zeros(comm.world * comm.world, dtype=torch.int32, device=self.device)
                comm.all_gather(allc, w.tcounts)
                M = allc.view(comm.world, comm.world).cpu()     # one sync
                w.send_splits, w.recv_splits = M[comm.rank].tolist(), M[:, comm.rank].tolist()
            R = w.R = sum(w.recv_splits)
            ld = HF + 4   # row, bias, pad: one all-to-all carries both
            recv_ids = self._xb(w, "recv_ids", max(R, 1), dtype=torch.int32)
            comm.all_to_all(recv_ids[:R], w.tsend[:B], w.recv_splits, w.send_splits)
            rows_out = self._xb(w, "rows_out", max(R, 1), ld)
            w.local_ids = self._xb(w, "local_ids", max(R, 1), dtype=torch.int32)
            call("rg_head_rows_gather", recv_ids.data_ptr(), R, self.lo, self.A, W, b, HF, ld, rows_out.data_ptr(),
                 w.local_ids.data_ptr(), st)
            rows_in = self._xb(w, "rows_in", B, ld)
            comm.all_to_all(rows_in[:B], rows_out[:R], w.send_splits, w.recv_splits)
            call("rg_rows_unslot", rows_in.data_ptr(), ld, w.tslot.data_ptr(), w.t32.data_ptr(), B, HF,
                 w.tW.data_ptr(), w.tb.data_ptr(), w.trow.data_ptr(), st)
        hp = h_planes.data_ptr() if h_planes is not None else None
        with region("sampled_fwd", exact=True):   # the one-launch logits on the exchanged planes (draw = 2)
            call("rg_sampled_logits", h.data_ptr(), W, b, w.ids.data_ptr(), 2, self.seed, self.draws, self.A_full,
                 B, S, HF, w.terms, w.ZT.data_ptr(), w.ldz, w.pmax.data_ptr(), w.psum.data_ptr(), w.Wg.data_ptr(),
                 w.bg.data_ptr(), hp, w.Wp.data_ptr(), st)
        self.draws += 1
        # CE with the fetched target rows (row b's target is row b of tW / tb; −1 for an invalid
        # target: NaN loss row, zero gradients, as on one GPU)
        call("rg_sampled_lse", h.data_ptr(), w.tW.data_ptr(), w.tb.data_ptr(), w.trow.data_ptr(), B, B, HF,
             w.pmax.data_ptr(), w.psum.data_ptr(), w.nT, g, w.lse.data_ptr(), w.loss_row.data_ptr(),
             w.ids.data_ptr() + 4 * S, w.gb.data_ptr() + 4 * S, w.grows.data_ptr() + 4 * S * HF,
             w.dh_slabs.data_ptr(), st)
        call("rg_sum_scale", w.loss_row.data_ptr(), B, g, w.loss.data_ptr(), None, st)
        comm.all_reduce(w.loss)
        return w.loss, w

    def backward_step(self, h, tgt, dh_out, adam6, slot="main", gscale=None, overlap=False):
        B = h.shape[0]
        w = self.sws(slot, B)
        comm, st = self.comm, stream_ptr()
        S, HF = self.S, self.HF
        g = _f32(1.0 / B) if gscale is None else gscale
        with region("sampled_bwd"):
            call("rg_sampled_dz_rows", w.ZT.data_ptr(), w.ldz, w.lse.data_ptr(), B, S, g, w.dbslabs.data_ptr(),
                 w.gb.data_ptr(), st)
            self._dz_gemms(w, h, B, S, HF, st)
            call("rg_reduce_slabs", w.dh_slabs.data_ptr(), w.dh_splits + 1, B * HF, dh_out.data_ptr(), None, HF, 0,
                 st)
            call("rg_reduce_slabs", w.dw_slabs.data_ptr(), w.dw_splits, S * HF, w.grows.data_ptr(), None, HF, 0,
                 st)
        R = w.R
        with region("neg_grad_exchange"):
            comm.all_reduce(w.grows[:S])   # every rank's rows' part of the negatives' gradients
            comm.all_reduce(w.gb[:S])
            ld = HF + 4
            call("rg_rows_slot", w.grows.data_ptr() + 4 * S * HF, w.gb.data_ptr() + 4 * S, w.tslot.data_ptr(), B,
                 HF, ld, w.gsend.data_ptr(), st)
            grecv = self._xb(w, "grecv", max(R, 1), ld)
            comm.all_to_all(grecv[:R], w.gsend[:B], w.recv_splits, w.send_splits)
        self.tag += 1
        with region("sampled_bwd"):
            G, Gb, tags = self.G.data_ptr(), self.Gb.data_ptr(), self.tags.data_ptr()
            self.scatter(w.nloc.data_ptr(), w.grows.data_ptr(), HF, w.nS.data_ptr(), S, -1, G, self.A, tags,
                         self.tag, st)
            self.scatter(w.nloc.data_ptr(), w.gb.data_ptr(), 1, w.nS.data_ptr(), S, -1, Gb, self.A, tags, self.tag,
                         st, reuse_sort=True)
            if R > 0:
                w.nR.fill_(R)
                self.scatter(w.local_ids.data_ptr(), grecv.data_ptr(), HF, w.nR.data_ptr(), R, -1, G, self.A, tags,
                             self.tag, st, ld=ld)
                self.scatter(w.local_ids.data_ptr(), grecv.data_ptr() + 4 * HF, 1, w.nR.data_ptr(), R, -1, Gb, self.A,
                             tags, self.tag, st, reuse_sort=True, ld=ld)
        with region("sampled_adam"):
            call("rg_adam_rows", self.W.p.data_ptr(), self.W.m.data_ptr(), self.W.v.data_ptr(), self.G.data_ptr(),
                 self.tags.data_ptr(), self.tag, self.A, HF, adam6, st)
            call("rg_adam_rows", self.b.p.data_ptr(), self.b.m.data_ptr(), self.b.v.data_ptr(), self.Gb.data_ptr(),
                 self.tags.data_ptr(), self.tag, self.A, 1, adam6, st)
