"""Double-Q training steps on the MI355X.

SQN  (SQN/sqn_gru.py:183-254): supervised head + one Q head, double-Q target.
SMORL (SMORL/smorl_gru.py:233-334, 3-reward form of SURVEY §3.4): supervised
head + Q heads (acc, div, nov), weighted-argmax target, online diversity and
novelty rewards.

Per step: trunk(s) with saved state; sup head CE (Zᵀ kept for backward);
Q(s, a) as B dot products; trunk(s') of the main net -> argmax of the
(weighted) Q head without storing Z; trunk(s') of the boot net with
``true_len`` (reference quirk) -> Q_boot(s', a*) gathers; TD loss;
backward: sup head (dh + fused dW/Adam), Q-head row scatter, BPTT, Adam
sweeps of every main-net parameter (dense semantics).
"""
from __future__ import annotations

import numpy as np
import torch

from . import call, engine, host_floats, host_ptr_array, stream_ptr
from .engine import SegScatter, SoftmaxHead, _f32
from .nets import HipNet
from .remap import raise_if_unmapped, remap_ids
from .timing import region


class QHead(SoftmaxHead):
    """Linear(H -> A) used through row gathers, argmax (fused GEMM pass, no Z
    stored) and row-sparse gradients; logits_T for evaluation."""

    def __init__(self, name, A, HF, device, shard=None):
        super().__init__(name, A, HF, device, shard=shard)
        self.G = torch.zeros_like(self.W.p)
        self.Gb = torch.zeros_like(self.b.p)
        self.tags = torch.zeros(self.A, dtype=torch.int32, device=device)

    def adam(self, adam6, tag):
        st = stream_ptr()
        call("rg_adam_rows", self.W.p.data_ptr(), self.W.m.data_ptr(), self.W.v.data_ptr(), self.G.data_ptr(),
             self.tags.data_ptr(), tag, self.A, self.HF, adam6, st)
        call("rg_adam_rows", self.b.p.data_ptr(), self.b.m.data_ptr(), self.b.v.data_ptr(), self.Gb.data_ptr(),
             self.tags.data_ptr(), tag, self.A, 1, adam6, st)


class _T:
    """Bare parameter holder (.p) for derived device tensors."""

    def __init__(self, t):
        self.p = t


class QNet(HipNet):
    """Trunk + supervised softmax head + Q heads (reference key names)."""

    def __init__(self, *, q_names, **kw):
        super().__init__(head_names=["sup_head_output"], **kw)
        self.q_heads = [QHead(n, self.action_dim, self.hf, self.device, shard=self.shard) for n in q_names]
        for q in self.q_heads:
            setattr(self, q.name, q)
        self._argmax_head = None
        self._buf = {}

    def set_matmul_precision(self, precision):
        """Also the Q heads' argmax contraction (the double-Q target a*): on
        split-bf16 MFMAs with f32x6 / f32x9; their row gathers stay fp32."""
        super().set_matmul_precision(precision)
        for q in self.q_heads:
            q.set_matmul_precision(precision)
        if self._argmax_head is not None:
            self._argmax_head.precision = precision
        return self

    def named_param_objs(self):
        out = list(self.trunk.named_params()) + self.sup_head_output.named_params()
        for q in self.q_heads:
            out += q.named_params()
        return out

    def buf(self, name, shape, dtype=torch.float32):
        t = self._buf.get(name)
        if t is None or tuple(t.shape) != tuple(shape) or t.dtype != dtype:
            t = torch.empty(*shape, dtype=dtype, device=self.device)
            self._buf[name] = t
        return t

    def forward(self, s, lengths):
        """(sup (B, A), q (B, A)) for SQN; (sup, q_all (B, heads, A)) for SMORL,
        as the reference's nn.Module forward returns (sqn_gru.py:87-112)."""
        if self.comm is not None:
            raise NotImplementedError("forward() of an item-sharded model: each rank holds a slice of the items")
        h = self.hidden(s, lengths, slot="eval", save=False)
        _, sup = self.sup_head_output.logits_T(h)
        outs = [q.logits_T(h)[1] for q in self.q_heads]
        if len(outs) == 1:
            return sup, outs[0]
        return sup, torch.stack(outs, dim=1)

    def argmax_q(self, h, weights=None):
        """argmax_a Σ_i w_i Q_i(s, a) via one fused GEMM+argmax pass over the
        combined head (W_c = Σ w_i W_i, b_c = Σ w_i b_i)."""
        if len(self.q_heads) == 1:
            return self.q_heads[0].argmax(h, slot="argmax")
        if self._argmax_head is None:
            hd = SoftmaxHead.__new__(SoftmaxHead)
            hd.name, hd.A, hd.HF, hd.device, hd._ws = "qcomb", self.q_heads[0].A, self.hf, self.device, {}
            hd.precision = self.q_heads[0].precision
            hd.W = _T(torch.empty_like(self.q_heads[0].W.p))
            hd.b = _T(torch.empty_like(self.q_heads[0].b.p))
            self._argmax_head = hd
        hd = self._argmax_head
        wts = host_floats(weights)
        st = stream_ptr()
        B = h.shape[0]
        if hd.flash_terms(B):
            # one pass over the Q heads: W_c, b_c, W_c's K-planes, padded bias and
            # max row norm for the screening argmax (csrc/misc.hip rg_qcomb)
            w = hd.amax_ws("argmax", B)
            call("rg_qcomb", host_ptr_array([q.W.p for q in self.q_heads]),
                 host_ptr_array([q.b.p for q in self.q_heads]), wts, len(self.q_heads), hd.A, hd.HF,
                 1 if engine.SCREEN_TERMS == 1 else 3, hd.W.p.data_ptr(), hd.b.p.data_ptr(), w.Wk.data_ptr(),
                 w.bias_pad.data_ptr(), w.wnorm.data_ptr(), st)
            return hd.argmax(h, slot="argmax", planes_ready=True)
        call("rg_weighted_sum", host_ptr_array([q.W.p for q in self.q_heads]), wts, len(self.q_heads),
             hd.W.p.numel(), hd.W.p.data_ptr(), st)
        call("rg_weighted_sum", host_ptr_array([q.b.p for q in self.q_heads]), wts, len(self.q_heads),
             hd.b.p.numel(), hd.b.p.data_ptr(), st)
        return hd.argmax(h, slot="argmax")

    def gather_q(self, h, idx64=None, idx32=None, out=None):
        B = h.shape[0]
        nh = len(self.q_heads)
        q = out if out is not None else torch.empty(B, nh, device=self.device)
        call("rg_q_gather", h.data_ptr(), self.hf, host_ptr_array([x.W.p for x in self.q_heads]),
             host_ptr_array([x.b.p for x in self.q_heads]), nh, None if idx64 is None else idx64.data_ptr(),
             None if idx32 is None else idx32.data_ptr(), B, q.data_ptr(), stream_ptr())
        return q


def q_side_stream(net):
    """The stream a Q network's head Adam sweeps run on (created once)."""
    if getattr(net, "_qstream", None) is None:
        net._qstream = torch.cuda.Stream(device=net.device)
    return net._qstream


# the double-Q target (the next-state trunk forwards, the combined Q head,
# the screening argmax, Q_boot(s', a*)) on its own stream beside the main
# state's forward and the supervised head's pass 1, joined before the TD loss
TARGET_SIDE_STREAM = True
# (round 6: starting it only after the previous step's pass 2, so that it shares the CUs with
# pass 1 instead, measured 214.5K vs 215.1K session-steps/s at C4 — not kept,
# profiles/r07/ab_c4_target_after_pass2.txt)
# queue the target on the host after the supervised head's pass 1 (device order
# unchanged: after the step's catch-up), so the main state's trunk forward and
# pass 1 are dispatched first and the target fills in beside pass 2: neutral at C4
# (228.5K vs 228.3K session-steps/s over three same-box pairs,
# profiles/r07/ab_c4_target_after_pass1.txt), so the target stays queued first
TARGET_AFTER_PASS1 = False


def target_stream(net):
    """The stream a network's double-Q target runs on when it is main (created once)."""
    if getattr(net, "_tstream", None) is None:
        net._tstream = torch.cuda.Stream(device=net.device)
    return net._tstream


def q_heads_backward(main, h, idx, B, dq, dh, tag, st):
    """Backward of the Q heads' gathered Q(s, a) (sqn_gru.py:221-222): dh +=
    Σ_i dq_i W_i[a], and G_i[a] += dq_i h, Gb_i[a] += dq_i summed per action in
    row order through one sort shared by every head (csrc/segsum.hip) — rows of
    a batch share actions, so atomic adds would make the step
    order-dependent.  idx: int64 action per row, -1 = not held here."""
    nh, HF = len(main.q_heads), main.hf
    rows = main.buf("q_grows", (nh, B, HF))
    rows_b = main.buf("q_grows_b", (nh, B))
    ids = main.buf("q_ids", (B,), torch.int32)
    n = main.buf("q_n", (1,), torch.int32)
    call("rg_q_backward", h.data_ptr(), HF, host_ptr_array([x.W.p for x in main.q_heads]), nh, idx.data_ptr(), B,
         dq.data_ptr(), dh.data_ptr(), rows.data_ptr(), rows_b.data_ptr(), ids.data_ptr(), n.data_ptr(), st)
    if getattr(main, "_qscatter", None) is None:
        main._qscatter = SegScatter(main.device)
    sc = main._qscatter
    for i, qh in enumerate(main.q_heads):
        sc(ids.data_ptr(), rows[i].data_ptr(), HF, n.data_ptr(), B, -1, qh.G.data_ptr(), qh.A, qh.tags.data_ptr(),
           tag, st, reuse_sort=i > 0)
        sc(ids.data_ptr(), rows_b[i].data_ptr(), 1, n.data_ptr(), B, -1, qh.Gb.data_ptr(), qh.A, qh.tags.data_ptr(),
           tag, st, reuse_sort=True)


def _dev(x, dev, dtype=None):
    x = x.to(dev, non_blocking=True)
    return x if dtype is None else x.to(dtype)




def double_q_step(nets, clocks, k, s, a, r, s_next, true_len, true_next_len, is_end, *, gamma, smorl=None,
                  host=None):
    """One SQN (smorl=None) or SMORL step with main = nets[k].  Returns device
    (sup_loss (1,) f32, q_loss (1,) f64 for SQN / f32 for SMORL)."""
    main, boot = nets[k], nets[1 - k]
    dev = main.device
    s = _dev(s, dev)
    a = _dev(a, dev)
    s_next = _dev(s_next, dev)
    end8 = _dev(is_end, dev, torch.uint8)
    B = s.shape[0]
    nh = len(main.q_heads)
    st = stream_ptr()
    cur = torch.cuda.current_stream(dev)

    # catch-up Adam: every embedding row the three trunk passes read is brought up to
    # date here, on the current stream, before the target pass forks onto its own
    main.trunk.catch_up_rows(s, s_next)
    boot.trunk.catch_up_rows(s_next)

    def target():
        with region("sqn_target"):
            h_n = main.trunk.forward(s_next, true_next_len, slot="next", save=False, catch_up=False)
            a_star = main.argmax_q(h_n, None if smorl is None else smorl["w"])
            h_b = boot.trunk.forward(s_next, true_len, slot="boot", save=False, catch_up=False)   # quirk: true_len
            return boot.gather_q(h_b, idx32=a_star, out=main.buf("qn", (B, nh)))

    # the double-Q target needs neither the supervised head nor its workspace
    # (nor the main state's trunk pass: its own trunk slots, the combined Q
    # head's workspace), so it runs on its own stream, ordered after
    # everything queued so far — the previous steps' updates — and beside the
    # main state's forward and pass 1, instead of ahead of pass 1 on the
    # serial chain; joined before the TD loss reads qn
    ts = target_stream(main) if TARGET_SIDE_STREAM else None
    late = ts is not None and TARGET_AFTER_PASS1
    if ts is not None:
        ts.wait_stream(cur)
        if not late:
            with torch.cuda.stream(ts):
                qn = target()
    with region("sqn_trunk_main"):
        h = main.trunk.forward(s, true_len, slot="main", save=True, catch_up=False)
    if ts is None:
        qn = target()
    sup_loss, _ = main.sup_head_output.forward_loss(h, a, slot="main")
    if late:   # queued behind pass 1 on the host, ordered on the device only after the catch-up above
        with torch.cuda.stream(ts):
            qn = target()
    q = main.gather_q(h, idx64=a, out=main.buf("q", (B, nh)))
    dq = main.buf("dq", (B, nh))
    if smorl is not None:   # the rewards' top-k re-scores pass 1's candidates with W: before pass 2 moves it
        rr = smorl_rewards(main, smorl, s, a, r, true_next_len, B)
        if smorl.get("lut") is not None:   # the reference raises in the reward, before any update
            raise_if_unmapped(smorl["remap_err"])
    # ---- backward + Adam (main network, its own optimizer clock) ----
    adam6 = clocks[k].next_args()
    main.trunk_tag = getattr(main, "trunk_tag", 0) + 1
    tag = main.trunk_tag
    dh = main.dh_buffer(B)
    # the supervised head's dh and pass 2 (side stream) need pass 1 only, not the double-Q
    # target: launched before the target is joined, so pass 2 never waits behind it (a target
    # whose kernels found the CUs busy with pass 1 used to run between pass 1 and pass 2,
    # profiles/r06/c4_timeline_target_stream.txt); pass 2 overlaps the target's tail, the TD
    # loss, the Q heads' backward / Adam and the trunk
    # (same box, C4: 225.3-227.1K vs 214.2-215.9K session-steps/s with pass 2 after the
    # join, profiles/r07/ab_c4_pass2_before_target.txt)
    main.sup_head_output.backward_step(h, a, dh, adam6, slot="main", overlap=True)
    if ts is not None:
        cur.wait_stream(ts)
    if smorl is None:
        r64 = _dev(r, dev, torch.float64)
        sq = main.buf("sq", (B,), torch.float64)
        q_loss = main.buf("qloss64", (1,), torch.float64)
        call("rg_sqn_td", q.data_ptr(), qn.data_ptr(), r64.data_ptr(), end8.data_ptr(), _f32(gamma), B, 1.0 / B,
             sq.data_ptr(), dq.data_ptr(), st)
        call("rg_sum64", sq.data_ptr(), B, 1.0 / B, q_loss.data_ptr(), None, st)
    else:
        row = main.buf("qrow", (B,))
        q_loss = main.buf("qloss32", (1,))
        grad_row = _f32(np.float32(smorl["alpha"]) / np.float32(B))
        call("rg_smorl_td", q.data_ptr(), qn.data_ptr(), rr.data_ptr(), end8.data_ptr(), smorl["w_dev"].data_ptr(),
             nh, _f32(gamma), grad_row, B, row.data_ptr(), dq.data_ptr(), st)
        call("rg_sum_scale", row.data_ptr(), B, _f32(1.0 / B), q_loss.data_ptr(), None, st)
    if host is not None:   # (SMORL on the native fp32 head: + rg_topk's K > 32 overflow flag; the
        # fused head never raises it — its overflowing rows are scanned whole, counted in top_scanned)
        fused = bool(main.sup_head_output.flash_terms(B))
        host.capture(sup_loss, q_loss, *([main.sup_head_output.top_err] if smorl is not None and not fused else []))
    q_heads_backward(main, h, a, B, dq, dh, tag, st)
    # the Q heads' dense Adam sweeps on their own stream beside the trunk
    # backward (they read only the Q heads' G rows, written above); joined
    # before the step ends
    qs = q_side_stream(main)
    qs.wait_stream(cur)
    with torch.cuda.stream(qs):
        for qh in main.q_heads:
            qh.adam(adam6, tag)
    main.trunk.backward(dh, slot="main")
    main.trunk.step(adam6, tag)
    cur.wait_stream(qs)
    return sup_loss, q_loss


def smorl_rewards(main, smorl, s, a, r_acc, true_next_len, B):
    """r = stack([r_acc, r_div, r_nov]).float32."""
    dev = main.device
    st = stream_ptr()
    head = main.sup_head_output
    k_div, k_nov = smorl["topk_div"], smorl["topk_nov"]
    K = max(k_div, k_nov)
    if head.flash_terms(B):   # fused head: top-K from pass 1, no logits stored
        idx, _ = head.top_entries(head.fws("main", B))
    elif K == 1:
        w = head.ws("main", B, True)
        idx = w.amax  # argmax of the supervised logits = topk(sup, 1)
    else:
        w = head.ws("main", B, True)
        idx = main.buf("topk_idx", (B, K), torch.int32)
        call("rg_topk", w.ZT.data_ptr(), w.ldz, w.pmax.data_ptr(), B, head.A, K, idx.data_ptr(), None,
             head.top_err.data_ptr(), st)
    r_div = main.buf("r_div", (B,))
    lens = _dev(true_next_len, dev, torch.int64)   # quirk: diversity uses true_next_len
    idx_div = idx if smorl.get("lut") is None else remap_ids(idx, smorl["lut"], smorl["remap_err"])
    call("rg_diversity", s.data_ptr(), s.shape[1], lens.data_ptr(), 1 if smorl["pad_end"] else 0,
         idx_div.data_ptr(), k_div, K, smorl["div_table"].data_ptr(), smorl["div_table"].shape[0],
         smorl["div_table"].shape[1], _f32(1e-6), B,
         r_div.data_ptr(), st)
    r_nov = main.buf("r_nov", (B,))
    call("rg_novelty", idx.data_ptr(), k_nov, K, smorl["bitmap"].data_ptr(), head.A, _f32(smorl["nov_rew_sig"]), B,
         r_nov.data_ptr(), st)
    r64 = _dev(r_acc, dev, torch.float64)
    rr = main.buf("rr", (B, 3))
    call("rg_stack_rewards", r64.data_ptr(), r_div.data_ptr(), r_nov.data_ptr(), B, rr.data_ptr(), st)
    main._last_rewards = rr
    return rr


_BITMAPS = {}


def unpopular_bitmap(unpopular, n_actions, device, fresh=False):
    """The unpopular set (novelty.py:12-47, item_frequency.py:8-24) as a device
    bitmap over the actions.  fresh=False (the per-batch update_train_metrics,
    which the harness calls with the same set every batch): cached per (set
    object, size, n_actions, device), so a set changed in place without a
    change of size must be passed as a new object (or a frozenset); evaluate()
    and the SMORL trainer's construction build it fresh."""
    key = (id(unpopular), len(unpopular), int(n_actions), str(device))
    hit = None if fresh else _BITMAPS.get(key)
    if hit is not None and hit[0] is unpopular:
        return hit[1]
    j = np.fromiter((int(x) for x in unpopular), dtype=np.int64, count=len(unpopular))
    j = j[(j >= 0) & (j < n_actions)]
    bm = np.zeros((n_actions + 31) // 32, dtype=np.uint32)
    np.bitwise_or.at(bm, j >> 5, (np.uint32(1) << (j & 31).astype(np.uint32)))
    t = torch.from_numpy(bm.view(np.int32)).to(device)
    if len(_BITMAPS) > 8:
        _BITMAPS.clear()
    _BITMAPS[key] = (unpopular, t)
    return t
