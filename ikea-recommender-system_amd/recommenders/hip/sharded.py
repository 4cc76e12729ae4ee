"""Multi-GPU supervised step: batch-sharded trunk, item-sharded head.

Weak scaling: every rank trains its own B-row batch shard; the job's
objective is the mean CE over all world·B rows (= one reference step on the
concatenated batch).  Per step:

  trunk (replicated params)      local fwd on the rank's B rows
  all_gather   h  (B·HF floats), targets (B int64)        -> world·B rows
  head shard   logits of all world·B rows over items [lo, hi)  (same FLOPs
               as one GPU at batch B), online LSE partials
  all_gather   per-rank lse (world·B floats) -> merged LSE
  all_reduce   target logit (owner rank contributes)
  backward     dH_all = dZ·W_shard (world·B × HF) -> reduce_scatter -> own dh
               BPTT, dX, dW_ih/dW_hh, embedding scatter (local)
  all_reduce   GRU grads (~0.4 MB) and the embedding grad table (async,
               overlapped with the head's fused dW + Adam kernel)
  Adam         head rows: local (each rank owns its items' W, b, m, v);
               trunk: identical dense Adam on every replica.

The output layer's gradient (A × H, 512 MB at C2) is never communicated.
"""
from __future__ import annotations

import torch

from . import call, stream_ptr
from .engine import _f32
from .timing import region


def _buf(net, name, shape, dtype=torch.float32):
    b = getattr(net, "_sbuf", None)
    if b is None:
        b = net._sbuf = {}
    t = b.get(name)
    if t is None or tuple(t.shape) != tuple(shape) or t.dtype != dtype:
        t = b[name] = torch.empty(*shape, dtype=dtype, device=net.device)
    return t


def sharded_supervised_step(net, clock, s, a, true_len):
    comm = net.comm
    dev = net.device
    s = s.to(dev, non_blocking=True)
    a = a.to(dev, non_blocking=True).contiguous()
    head = next(iter(net.heads.values()))
    W_, HF = comm.world, net.hf
    st = stream_ptr()
    h = net.trunk.forward(s, true_len, slot="main", save=True)
    B = h.shape[0]
    Bg = W_ * B
    mask = None
    h_in = h
    if net.training and net.dropout_p > 0:
        mask = net.dropout_mask(B)
        h_in = net.apply_mask(h, mask, _buf(net, "hd", (B, HF)))
    with region("comm_fwd"):
        H_all = comm.all_gather(_buf(net, "H_all", (Bg, HF)), h_in)
        a_all = comm.all_gather(_buf(net, "a_all", (Bg,), torch.int64), a)
    w = head.ws("main", Bg, True)
    with region("head_fwd"):
        call("rg_head_fwd", H_all.data_ptr(), head.W.p.data_ptr(), head.b.p.data_ptr(), Bg, head.A, HF,
             w.ZT.data_ptr(), w.ldz, w.pmax.data_ptr(), w.psum.data_ptr(), w.parg.data_ptr(), 1, st)
    call("rg_lse_combine", w.pmax.data_ptr(), w.psum.data_ptr(), w.parg.data_ptr(), Bg, w.nJ, w.work.data_ptr(),
         None, 0, None, head.A, w.lse.data_ptr(), None, None, st)
    zt = _buf(net, "zt", (Bg,))
    tgt_loc = _buf(net, "tgt_loc", (Bg,), torch.int64)
    call("rg_shard_targets", w.ZT.data_ptr(), w.ldz, a_all.data_ptr(), head.lo, head.hi, Bg, zt.data_ptr(),
         tgt_loc.data_ptr(), st)
    with region("comm_lse"):
        lse_r = comm.all_gather(_buf(net, "lse_r", (W_ * Bg,)), w.lse)
        comm.all_reduce(zt)
    lse = _buf(net, "lse_g", (Bg,))
    call("rg_lse_merge_ranks", lse_r.data_ptr(), W_, Bg, lse.data_ptr(), st)
    call("rg_sub", lse.data_ptr(), zt.data_ptr(), Bg, w.loss_row.data_ptr(), st)
    call("rg_sum_scale", w.loss_row.data_ptr(), Bg, _f32(1.0 / Bg), w.loss.data_ptr(), None, st)
    # ---- backward ----
    adam6 = clock.next_args()
    net.trunk_tag = getattr(net, "trunk_tag", 0) + 1
    g = _f32(1.0 / Bg)
    dH_all = _buf(net, "dH_all", (Bg, HF))
    with region("head_dh"):
        n = call("rg_head_dh", w.ZT.data_ptr(), w.ldz, lse.data_ptr(), tgt_loc.data_ptr(), g, head.W.p.data_ptr(),
                 Bg, head.A, HF, w.dh_splits, w.dh_slabs.data_ptr(), st)
    call("rg_reduce_slabs", w.dh_slabs.data_ptr(), n, Bg * HF, dH_all.data_ptr(), None, HF, 0, st)
    dh = net.dh_buffer(B)
    with region("comm_dh"):
        comm.reduce_scatter(dh, dH_all)
    if mask is not None:
        net.apply_mask(dh, mask, dh)
    net.trunk.backward(dh, slot="main")
    net.trunk.grads_for_allreduce(net.trunk_tag)
    works = net.trunk.allreduce_start(comm)
    with region("head_dw_adam"):
        call("rg_head_dw_adam", w.ZT.data_ptr(), w.ldz, lse.data_ptr(), tgt_loc.data_ptr(), g, H_all.data_ptr(),
             Bg, head.A, HF, head.W.p.data_ptr(), head.W.m.data_ptr(), head.W.v.data_ptr(), head.b.p.data_ptr(),
             head.b.m.data_ptr(), head.b.v.data_ptr(), adam6, None, None, st)
    with region("comm_wait"):
        for wk in works:
            if wk is not None:
                wk.wait()
    net.trunk.adam_after_allreduce(adam6)
    return w.loss
