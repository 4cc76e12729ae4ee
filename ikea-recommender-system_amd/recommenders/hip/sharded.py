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

import numpy as np
import torch

from . import call, stream_ptr
from .engine import _f32
from .dist import host_routes
from .qlearn import q_heads_backward, q_side_stream
from .remap import raise_if_unmapped, remap_ids
from .timing import region


def _buf(net, name, shape, dtype=torch.float32):
    b = getattr(net, "_sbuf", None)
    if b is None:
        b = net._sbuf = {}
    t = b.get(name)
    if t is None or tuple(t.shape) != tuple(shape) or t.dtype != dtype:
        t = b[name] = torch.empty(*shape, dtype=dtype, device=net.device)
    return t


def _sharded_ce_forward(net, head, H_all, a_all, st, want_argmax=False):
    """CE(mean over world·B rows) of the item-sharded head: local logits over
    items [lo, hi) for every gathered row, per-rank LSE merged across ranks,
    target logit summed from its owner.  Keeps Zᵀ/lse for the backward.  With
    want_argmax the native head leaves the local (row max, argmax) in
    w.mx / w.amax; the fused head computes its top entries in pass 1
    (head.top_k, read with head.top_entries)."""
    comm = net.comm
    W_, HF = comm.world, net.hf
    Bg = H_all.shape[0]
    terms = head.flash_terms(Bg)
    if terms:
        # fused split-bf16 head (csrc/head_flash.hip): local lse and the
        # owner's target logit, no logits stored; targets stay global ids
        w = head.flash_forward(H_all, a_all, "main", terms)
        zt, tgt_loc = w.zt, a_all
    else:
        w = head.ws("main", Bg, True)
        with region("head_fwd"):
            call("rg_head_fwd", H_all.data_ptr(), head.W.p.data_ptr(), head.b.p.data_ptr(), Bg, head.A, HF,
                 w.ZT.data_ptr(), w.ldz, w.pmax.data_ptr(), w.psum.data_ptr(), w.parg.data_ptr(), 1, st)
        call("rg_lse_combine", w.pmax.data_ptr(), w.psum.data_ptr(), w.parg.data_ptr(), Bg, w.nJ, w.work.data_ptr(),
             None, 0, None, head.A, w.lse.data_ptr(), w.amax.data_ptr() if want_argmax else None, None,
             w.mx.data_ptr() if want_argmax else None, st)
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
    return w, lse, tgt_loc


def _sharded_ce_dh(net, head, w, lse, tgt_loc, dH_all, st):
    """dH_all (world·B × HF) := dZ · W_shard for every gathered row."""
    Bg = dH_all.shape[0]
    if getattr(w, "terms", 0):  # fused head: tgt_loc holds the global target ids
        head.flash_dh(w, tgt_loc, lse, _f32(1.0 / Bg), dH_all)
        return
    with region("head_dh"):
        n = call("rg_head_dh", w.ZT.data_ptr(), w.ldz, lse.data_ptr(), tgt_loc.data_ptr(), _f32(1.0 / Bg),
                 head.W.p.data_ptr(), Bg, head.A, net.hf, w.dh_splits, w.dh_slabs.data_ptr(), st)
    call("rg_reduce_slabs", w.dh_slabs.data_ptr(), n, Bg * net.hf, dH_all.data_ptr(), None, net.hf, 0, st)




def _sharded_ce_dw_adam(net, head, w, lse, tgt_loc, H_all, adam6, st):
    Bg = H_all.shape[0]
    if getattr(w, "terms", 0):
        head.flash_dw_adam(w, _f32(1.0 / Bg), adam6)
        return
    with region("head_dw_adam"):
        call("rg_head_dw_adam", w.ZT.data_ptr(), w.ldz, lse.data_ptr(), tgt_loc.data_ptr(), _f32(1.0 / Bg),
             H_all.data_ptr(), Bg, head.A, net.hf, head.W.p.data_ptr(), head.W.m.data_ptr(), head.W.v.data_ptr(),
             head.b.p.data_ptr(), head.b.m.data_ptr(), head.b.v.data_ptr(), adam6, None, None, st)


def _gather_rows(comm, net, name, x):
    """all_gather of a local (B, ...) tensor into (world·B, ...), rank-major."""
    out = _buf(net, name, (comm.world * x.shape[0],) + tuple(x.shape[1:]), x.dtype)
    return comm.all_gather(out, x.contiguous())


def sharded_sampled_step(net, clock, s, a, true_len, host=None):
    """GRU4Rec with the item-sharded sampled head (engine.ShardedSampledHead)
    over the global batch: each rank's trunk on its own rows (row-sharded item
    table, id / row exchange), the head's rows moved to the data (negatives by
    one all-reduce, targets by all-to-all), trunk gradients all-reduced.  The
    mean CE over all world·B rows = the one-GPU sampled step on the
    concatenated batch (same negatives) up to fp32 summation order."""
    comm = net.comm
    dev = net.device
    head = next(iter(net.heads.values()))
    routes = host_routes(comm, net.trunk, [(s, true_len)], targets=(a, head.A_full))
    route, troute = (routes[0], routes[1]) if routes else (None, None)
    s = s.to(dev, non_blocking=True)
    a = a.to(dev, non_blocking=True).contiguous()
    h = net.trunk.forward(s, true_len, slot="main", save=True, route=route)
    B = h.shape[0]
    Bg = comm.world * B
    g = _f32(1.0 / Bg)
    mask = None
    h_in = h
    if net.training and net.dropout_p > 0:
        mask = net.dropout_mask(B)
        h_in = net.apply_mask(h, mask, _buf(net, "hd", (B, net.hf)))
    loss, _ = head.forward_loss(h_in, a, slot="main", h_planes=net.trunk.h_planes if mask is None else None,
                                gscale=g, route=troute)
    if host is not None:
        host.capture(loss)
    adam6 = clock.next_args()
    net.trunk_tag = getattr(net, "trunk_tag", 0) + 1
    dh = net.dh_buffer(B)
    head.backward_step(h_in, a, dh, adam6, slot="main", gscale=g)
    if mask is not None:
        net.apply_mask(dh, mask, dh)
    net.trunk.backward(dh, slot="main")
    net.trunk.grads_for_allreduce(net.trunk_tag)
    works = net.trunk.allreduce_start(comm)
    net.trunk.adam_after_allreduce(adam6, works)
    return loss


def sharded_supervised_step(net, clock, s, a, true_len, host=None):
    if hasattr(next(iter(net.heads.values())), "neg_job"):   # sampled head
        return sharded_sampled_step(net, clock, s, a, true_len, host=host)
    comm = net.comm
    dev = net.device
    # the id / row exchange's splits from the host batch (no device read-back)
    route = host_routes(comm, net.trunk, [(s, true_len)])
    s = s.to(dev, non_blocking=True)
    a = a.to(dev, non_blocking=True).contiguous()
    head = next(iter(net.heads.values()))
    HF = net.hf
    st = stream_ptr()
    h = net.trunk.forward(s, true_len, slot="main", save=True, route=route and route[0])
    B = h.shape[0]
    Bg = comm.world * B
    mask = None
    h_in = h
    if net.training and net.dropout_p > 0:
        mask = net.dropout_mask(B)
        h_in = net.apply_mask(h, mask, _buf(net, "hd", (B, HF)))
    with region("comm_fwd"):
        H_all = _gather_rows(comm, net, "H_all", h_in)
        a_all = _gather_rows(comm, net, "a_all", a)
    w, lse, tgt_loc = _sharded_ce_forward(net, head, H_all, a_all, st)
    if host is not None:
        host.capture(w.loss)
    # ---- backward ----
    adam6 = clock.next_args()
    net.trunk_tag = getattr(net, "trunk_tag", 0) + 1
    dH_all = _buf(net, "dH_all", (Bg, HF))
    _sharded_ce_dh(net, head, w, lse, tgt_loc, dH_all, st)
    fused = bool(getattr(w, "terms", 0))
    if fused:   # pass 2 on the head's side stream under the exchanges and the trunk backward
        head.flash_dw_adam_async(w, _f32(1.0 / Bg), adam6)
    dh = net.dh_buffer(B)
    with region("comm_dh"):
        comm.reduce_scatter(dh, dH_all)
    if mask is not None:
        net.apply_mask(dh, mask, dh)
    net.trunk.backward(dh, slot="main")
    net.trunk.grads_for_allreduce(net.trunk_tag)
    works = net.trunk.allreduce_start(comm)
    if not fused:
        _sharded_ce_dw_adam(net, head, w, lse, tgt_loc, H_all, adam6, st)
    net.trunk.adam_after_allreduce(adam6, works)   # (waits for the all-reduce on the trunk's side stream)
    return w.loss


# ------------------------------------------------------ double-Q (C4) ------
def _owner_q(qnet, buf_net, H_all, name, idx64=None, idx32=None):
    """Q_i(row)[idx] for every gathered row: the rank holding item idx computes
    it, the others write 0, a SUM all-reduce leaves the owner's exact value on
    every rank.  Returns (q (world·B, nh), local index (world·B) or −1)."""
    comm = buf_net.comm
    st = stream_ptr()
    Bg = H_all.shape[0]
    qh = qnet.q_heads[0]
    loc = _buf(buf_net, name + "_loc", (Bg,), torch.int64)
    call("rg_shard_index", None if idx64 is None else idx64.data_ptr(), None if idx32 is None else idx32.data_ptr(),
         Bg, qh.lo, qh.hi, loc.data_ptr(), st)
    q = qnet.gather_q(H_all, idx64=loc, out=_buf(buf_net, name, (Bg, len(qnet.q_heads))))
    comm.all_reduce(q)
    return q, loc


def _global_argmax(net, mx, am, A, name):
    """Merge every rank's (row max, local argmax) into the global first-maximum index."""
    comm = net.comm
    Bg = mx.shape[0]
    mx_r = _gather_rows(comm, net, name + "_mx", mx)
    am_r = _gather_rows(comm, net, name + "_am", am)
    out = _buf(net, name, (Bg,), torch.int32)
    call("rg_argmax_merge_ranks", mx_r.data_ptr(), am_r.data_ptr(), comm.world, Bg, A, out.data_ptr(), None,
         stream_ptr())
    return out


def _global_topk(net, head, w, K, name):
    """Canonical top-K of the supervised logits over all items, every gathered row."""
    comm = net.comm
    Bg = w.B
    st = stream_ptr()
    if getattr(w, "terms", 0):   # fused head: local top-K from pass 1's chunk maxima
        idx, vals = head.top_entries(w)
    else:
        vals = _buf(net, name + "_v", (Bg, K))
        idx = _buf(net, name + "_i", (Bg, K), torch.int32)
        call("rg_topk", w.ZT.data_ptr(), w.ldz, w.pmax.data_ptr(), Bg, head.A, K, idx.data_ptr(), vals.data_ptr(),
             head.top_err.data_ptr(), st)
    v_r = _gather_rows(comm, net, name + "_vr", vals)
    i_r = _gather_rows(comm, net, name + "_ir", idx)
    out = _buf(net, name, (Bg, K), torch.int32)
    call("rg_topk_merge_ranks", v_r.data_ptr(), i_r.data_ptr(), comm.world, Bg, K, head.A_full, out.data_ptr(), None,
         st)
    return out


def sharded_double_q_step(nets, clocks, k, s, a, r, s_next, true_len, true_next_len, is_end, *, gamma, smorl=None,
                          host=None):
    """SQN / SMORL step over the global batch (every rank's B rows) with the
    trunk replicated and every head item-sharded:

      trunks      local fwd (main on s and s', boot on s' with true_len)
      all_gather  h, h', h_boot, a (world·B rows)
      sup CE      as sharded_supervised_step
      Q(s, a)     owner computes, SUM all-reduce
      a*          local argmax of (Σ w_i) Q_main(s', ·) per shard -> all_gather
                  (max, index) -> first global maximum (rg_argmax_merge_ranks)
      Q_boot(s', a*)  owner computes, SUM all-reduce
      TD / SMORL  on the rank's own rows; losses summed over ranks
      backward    sup dH + Q-head dH accumulate in one (world·B × HF) buffer,
                  one reduce_scatter; trunk grads all-reduced; head rows and
                  their Adam moments never leave their owner.
    Returns device (sup_loss, q_loss) — the global-batch means."""
    from .qlearn import _dev
    main, boot = nets[k], nets[1 - k]
    comm = main.comm
    dev = main.device
    # splits of the three trunk passes' id / row exchanges from the host batch
    # (one host all-gather over the gloo group; no device read-back)
    routes = host_routes(comm, main.trunk, [(s, true_len), (s_next, true_next_len), (s_next, true_len)]) or [None] * 3
    s = _dev(s, dev)
    a = _dev(a, dev).contiguous()
    s_next = _dev(s_next, dev)
    end8 = _dev(is_end, dev, torch.uint8)
    B = s.shape[0]
    Bg = comm.world * B
    rows = slice(comm.rank * B, (comm.rank + 1) * B)
    nh = len(main.q_heads)
    HF = main.hf
    A = main.action_dim
    st = stream_ptr()
    sup = main.sup_head_output
    with region("sqn_trunk_main"):
        h = main.trunk.forward(s, true_len, slot="main", save=True, route=routes[0])
    with region("comm_fwd"):
        H_all = _gather_rows(comm, main, "H_all", h)
        a_all = _gather_rows(comm, main, "a_all", a)
    want_top1 = smorl is not None and max(smorl["topk_div"], smorl["topk_nov"]) == 1
    w, lse, tgt_loc = _sharded_ce_forward(main, sup, H_all, a_all, st, want_argmax=want_top1)
    sup_loss = w.loss
    q_all, a_loc = _owner_q(main, main, H_all, "q", idx64=a_all)
    with region("sqn_target"):
        h_n = main.trunk.forward(s_next, true_next_len, slot="next", save=False, route=routes[1])
        Hn_all = _gather_rows(comm, main, "Hn_all", h_n)
        am = main.argmax_q(Hn_all, None if smorl is None else smorl["w"])
        head_am = main.q_heads[0] if len(main.q_heads) == 1 else main._argmax_head
        a_star = _global_argmax(main, head_am.argmax_mx, am, A, "a_star")
        h_b = boot.trunk.forward(s_next, true_len, slot="boot", save=False,   # quirk: true_len
                                 route=routes[2])
        Hb_all = _gather_rows(comm, main, "Hb_all", h_b)
        qn_all, _ = _owner_q(boot, main, Hb_all, "qn", idx32=a_star)
    q = q_all[rows]
    qn = qn_all[rows]
    dq = _buf(main, "dq", (B, nh))
    if smorl is None:
        r64 = _dev(r, dev, torch.float64)
        sq = _buf(main, "sq", (B,), torch.float64)
        q_loss = _buf(main, "qloss64", (1,), torch.float64)
        call("rg_sqn_td", q.data_ptr(), qn.data_ptr(), r64.data_ptr(), end8.data_ptr(), _f32(gamma), B, 1.0 / Bg,
             sq.data_ptr(), dq.data_ptr(), st)
        call("rg_sum64", sq.data_ptr(), B, 1.0 / Bg, q_loss.data_ptr(), None, st)
    else:
        if want_top1 and getattr(w, "terms", 0):
            am1, mx1 = sup.top_entries(w)
            top = _global_argmax(main, mx1.view(Bg), am1.view(Bg), A, "sup_top1").view(Bg, 1)
        elif want_top1:
            top = _global_argmax(main, w.mx, w.amax, A, "sup_top1").view(Bg, 1)
        else:
            top = _global_topk(main, sup, w, max(smorl["topk_div"], smorl["topk_nov"]), "sup_topk")
        rr = _smorl_rewards_rows(main, smorl, s, r, true_next_len, top[rows].contiguous(), B)
        if smorl.get("lut") is not None:   # every rank raises together, before any update
            raise_if_unmapped(smorl["remap_err"], comm)
        row = _buf(main, "qrow", (B,))
        q_loss = _buf(main, "qloss32", (1,))
        grad_row = _f32(np.float32(smorl["alpha"]) / np.float32(Bg))
        call("rg_smorl_td", q.data_ptr(), qn.data_ptr(), rr.data_ptr(), end8.data_ptr(), smorl["w_dev"].data_ptr(),
             nh, _f32(gamma), grad_row, B, row.data_ptr(), dq.data_ptr(), st)
        call("rg_sum_scale", row.data_ptr(), B, _f32(1.0 / Bg), q_loss.data_ptr(), None, st)
    comm.all_reduce(q_loss)
    if host is not None:   # (SMORL on the native fp32 head: + rg_topk's K > 32 overflow flag)
        host.capture(sup_loss, q_loss, *([sup.top_err] if smorl is not None and not getattr(w, "terms", 0) else []))
    # ---- backward + Adam (main network, its own optimizer clock) ----
    adam6 = clocks[k].next_args()
    main.trunk_tag = getattr(main, "trunk_tag", 0) + 1
    tag = main.trunk_tag
    dH_all = _buf(main, "dH_all", (Bg, HF))
    _sharded_ce_dh(main, sup, w, lse, tgt_loc, dH_all, st)
    fused = bool(getattr(w, "terms", 0))
    if fused:   # pass 2 on the supervised head's side stream under the rest of the step
        sup.flash_dw_adam_async(w, _f32(1.0 / Bg), adam6)
    dq_all = _gather_rows(comm, main, "dq_all", dq)
    q_heads_backward(main, H_all, a_loc, Bg, dq_all, dH_all, tag, st)
    cur = torch.cuda.current_stream(main.device)
    qs = q_side_stream(main)   # the Q heads' dense Adam sweeps beside the trunk's (qlearn.double_q_step)
    qs.wait_stream(cur)
    with torch.cuda.stream(qs):
        for qh in main.q_heads:
            qh.adam(adam6, tag)
    dh = main.dh_buffer(B)
    with region("comm_dh"):
        comm.reduce_scatter(dh, dH_all)
    main.trunk.backward(dh, slot="main")
    main.trunk.grads_for_allreduce(tag)
    works = main.trunk.allreduce_start(comm)
    if not fused:
        _sharded_ce_dw_adam(main, sup, w, lse, tgt_loc, H_all, adam6, st)
    main.trunk.adam_after_allreduce(adam6, works)   # (waits for the all-reduce on the trunk's side stream)
    cur.wait_stream(qs)
    return sup_loss, q_loss


def _smorl_rewards_rows(main, smorl, s, r_acc, true_next_len, idx, B):
    """r = stack([r_acc, r_div, r_nov]) for the rank's rows from their global top-k list."""
    from .qlearn import _dev
    dev = main.device
    st = stream_ptr()
    K = idx.shape[1]
    r_div = _buf(main, "r_div", (B,))
    lens = _dev(true_next_len, dev, torch.int64)   # quirk: diversity uses true_next_len
    idx_div = idx if smorl.get("lut") is None else remap_ids(idx, smorl["lut"], smorl["remap_err"])
    call("rg_diversity", s.data_ptr(), s.shape[1], lens.data_ptr(), 1 if smorl["pad_end"] else 0,
         idx_div.data_ptr(), smorl["topk_div"], K, smorl["div_table"].data_ptr(), smorl["div_table"].shape[0],
         smorl["div_table"].shape[1],
         _f32(1e-6), B, r_div.data_ptr(), st)
    r_nov = _buf(main, "r_nov", (B,))
    call("rg_novelty", idx.data_ptr(), smorl["topk_nov"], K, smorl["bitmap"].data_ptr(), main.action_dim,
         _f32(smorl["nov_rew_sig"]),
         B, r_nov.data_ptr(), st)
    r64 = _dev(r_acc, dev, torch.float64)
    rr = _buf(main, "rr", (B, 3))
    call("rg_stack_rewards", r64.data_ptr(), r_div.data_ptr(), r_nov.data_ptr(), B, rr.data_ptr(), st)
    main._last_rewards = rr
    return rr
