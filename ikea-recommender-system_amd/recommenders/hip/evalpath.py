"""Device path of evaluation.

The reference scores every batch as a full (B, A) prediction matrix, copies
it to the host and runs torch.topk there (recommenders/evaluate/
eval_protocol.py:179-214, :303-318).  Here no (B, A) buffer exists:
``SoftmaxHead.score_topk`` runs pass 1's S-part (rg_flash_score: lse
partials and 32-item chunk maxima, row-chunked), the CE from rg_flash_lse,
and the canonical top-K by re-scoring the candidate chunks' items in fp32
(rg_flash_topk); HR/NDCG sums, diversity and novelty are kernels, and only
the (B, K) top-K index matrix reaches the host.  Heads the fused scorer does
not take (HF outside {32, 64, 128, 256}, or K > 32) score row chunks of
stored logits (rg_head_fwd + rg_topk), each chunk's Zᵀ bounded by
EVAL_ZT_BYTES and released after the batch.
"""
from __future__ import annotations

import ctypes

import torch

from . import call, stream_ptr
from .engine import _f32

# row chunk of the stored-logit fallback: Zᵀ (A x rows floats) at most this many bytes
EVAL_ZT_BYTES = 1 << 30


class EvalBatch:
    __slots__ = ("idx", "idx_in", "vals", "loss", "div", "nov", "hits", "ndcg", "reps")


def head_for(model, head_idx):
    heads = list(model.heads.values())
    if head_idx == 0:
        return heads[0]
    qh = getattr(model, "q_heads", [])
    if head_idx == 1 and len(qh) == 1:
        return qh[0]
    raise NotImplementedError(f"head_idx={head_idx} for {type(model).__name__}")


def topk_device(head, ws, B, K):
    """rg_topk over a stored Zᵀ (native head workspace)."""
    idx = torch.empty(B, K, dtype=torch.int32, device=head.device)
    vals = torch.empty(B, K, dtype=torch.float32, device=head.device)
    err = torch.zeros(1, dtype=torch.int32, device=head.device)
    call("rg_topk", ws.ZT.data_ptr(), ws.ldz, ws.pmax.data_ptr(), B, head.A, K, idx.data_ptr(), vals.data_ptr(),
         err.data_ptr(), stream_ptr())
    return idx, vals, err


def fused_scoring(head, K):
    return head.HF in (32, 64, 128, 256) and K <= min(32, head.A)


def score_rows(head, h, K, tgt=None, screen=True):
    """(idx (B, K) int32, vals (B, K), loss_row (B,) or None, err flag tensor
    or None): the canonical top-K and per-row CE of h's logits without a
    (B, A) buffer.  Without targets (update_train_metrics) the chunk maxima
    come from the 3-product screening pass; a row whose candidate band holds
    more chunks than the cap is scanned whole on the device, so the fused path
    has no error flag.  The stored-logit fallback's flag (rg_topk, K > 32 on
    massive ties) is read by the caller once at its end."""
    B = h.shape[0]
    if fused_scoring(head, K):
        idx, vals, loss_row = head.score_topk(h, K, tgt, screen=screen and tgt is None)
        return idx, vals, loss_row, None
    # stored-logit fallback, row-chunked
    st = stream_ptr()
    dev = head.device
    rows = max(4, min(B, EVAL_ZT_BYTES // (4 * head.A) // 4 * 4))
    idx = torch.empty(B, K, dtype=torch.int32, device=dev)
    vals = torch.empty(B, K, device=dev)
    loss_row = torch.empty(B, device=dev) if tgt is not None else None
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    W, b = head.params_ro()
    for r0 in range(0, B, rows):
        n = min(rows, B - r0)
        w = head.ws("eval_chunk", n, True)
        hs = h[r0:r0 + n]
        call("rg_head_fwd", hs.data_ptr(), W.p.data_ptr(), b.p.data_ptr(), n, head.A, head.HF, w.ZT.data_ptr(),
             w.ldz, w.pmax.data_ptr(), w.psum.data_ptr(), w.parg.data_ptr(), 1, st)
        if tgt is not None:
            call("rg_lse_combine", w.pmax.data_ptr(), w.psum.data_ptr(), w.parg.data_ptr(), n, w.nJ,
                 w.work.data_ptr(), w.ZT.data_ptr(), w.ldz, tgt[r0:r0 + n].data_ptr(), head.A, w.lse.data_ptr(),
                 w.amax.data_ptr(), loss_row.data_ptr() + 4 * r0, None, st)
        call("rg_topk", w.ZT.data_ptr(), w.ldz, w.pmax.data_ptr(), n, head.A, K, idx.data_ptr() + 4 * r0 * K,
             vals.data_ptr() + 4 * r0 * K, err.data_ptr(), st)
    # no Zᵀ stays cached after the batch (the caching allocator reuses the block)
    for k in [k for k in head._ws if k[0] == "eval_chunk"]:
        del head._ws[k]
    return idx, vals, loss_row, err


def eval_batch(model, s, s_len, a, *, head_idx=0, K=20, ks=(20,), padding_pos="end", div_table=None, k_div=1,
               bitmap=None, k_nov=1, nov_reward=1.0, want_loss=True, lut=None, rep_ks=None, screen=True):
    """CE loss, top-K, HR/NDCG sums and reward sums of one batch, on the
    device.  ``lut`` (recommenders/hip/remap.py): the top-K ids are mapped to
    the input vocabulary for the diversity reward and returned as ``idx_in``
    (for the host repetition count), as the reference's tokenizer branch
    does; an id without an input token raises RemapError (the reference's
    stoi KeyError) — its diversity entry is NaN and never reads the table."""
    dev = model.device
    s = s.to(dev)
    a = a.to(dev)
    B = s.shape[0]
    st = stream_ptr()
    h = model.hidden(s, s_len, slot="eval", save=False)
    head = head_for(model, head_idx)
    idx, vals, loss_row, top_err = score_rows(head, h, K, a if want_loss else None, screen=screen)
    out = EvalBatch()
    out.loss = None
    if want_loss:
        loss = torch.empty(1, device=dev)
        call("rg_sum_scale", loss_row.data_ptr(), B, _f32(1.0 / B), loss.data_ptr(), None, st)
        out.loss = loss
    out.idx, out.vals = idx, vals
    out.idx_in = idx
    rerr = None
    if lut is not None:
        from .remap import remap_ids
        rerr = torch.zeros(1, dtype=torch.int32, device=dev)
        out.idx_in = remap_ids(idx, lut, rerr)
    sums = torch.zeros(2 * len(ks), dtype=torch.float64, device=dev)
    ks_host = (ctypes.c_int * len(ks))(*[int(k) for k in ks])
    call("rg_hits_ndcg", idx.data_ptr(), K, a.data_ptr(), B, ks_host, len(ks), sums.data_ptr(), st)
    out.hits, out.ndcg = sums[:len(ks)], sums[len(ks):]
    out.div = out.nov = None
    if div_table is not None:
        lens = torch.as_tensor(s_len).to(dev, torch.int64)
        div = torch.empty(B, device=dev)
        call("rg_diversity", s.data_ptr(), s.shape[1], lens.data_ptr(), 1 if padding_pos == "end" else 0,
             out.idx_in.data_ptr(), k_div, K, div_table.data_ptr(), div_table.shape[0], div_table.shape[1],
             _f32(1e-6), B, div.data_ptr(), st)
        out.div = div
    if bitmap is not None:
        nov = torch.empty(B, device=dev)
        call("rg_novelty", idx.data_ptr(), k_nov, K, bitmap.data_ptr(), head.A, _f32(nov_reward), B, nov.data_ptr(),
             st)
        out.nov = nov
    out.reps = None
    if rep_ks is not None:   # repetitions (repetitiveness.py:21-57) on the input-vocabulary ids
        reps = torch.zeros(len(rep_ks), dtype=torch.int64, device=dev)
        kh = (ctypes.c_int * len(rep_ks))(*[int(k) for k in rep_ks])
        call("rg_repetitions", s.data_ptr(), s.shape[1], out.idx_in.data_ptr(), K, B, kh, len(rep_ks),
             reps.data_ptr(), st)
        out.reps = reps
    if top_err is not None and int(top_err.item()):   # stored-logit fallback only (rg_topk, K > 32)
        raise RuntimeError("top-k candidate overflow (massive exact ties in the logits)")
    if rerr is not None and int(rerr.item()):
        from .remap import RemapError
        raise RemapError("a predicted id has no input-vocabulary token (input_tokenizer.stoi(output_tokenizer.itos(id)))")
    return out
