"""Device path of evaluation: per batch the logits
stay in HBM (Zᵀ from the head forward), the top-k runs on the MI355X
(rg_topk), CE / diversity / novelty / HR-NDCG sums are kernels, and only the
(B, K) top-k index matrix reaches the host — the reference copies the whole
(B, A) logit matrix there (recommenders/evaluate/eval_protocol.py:199, :318).
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import call, stream_ptr
from .engine import _f32


class EvalBatch:
    __slots__ = ("idx", "idx_in", "vals", "loss", "div", "nov", "hits", "ndcg")


def head_for(model, head_idx):
    heads = list(model.heads.values())
    if head_idx == 0:
        return heads[0]
    qh = getattr(model, "q_heads", [])
    if head_idx == 1 and len(qh) == 1:
        return qh[0]
    raise NotImplementedError(f"head_idx={head_idx} for {type(model).__name__}")


def topk_device(head, ws, B, K):
    idx = torch.empty(B, K, dtype=torch.int32, device=head.device)
    vals = torch.empty(B, K, dtype=torch.float32, device=head.device)
    err = torch.zeros(1, dtype=torch.int32, device=head.device)
    call("rg_topk", ws.ZT.data_ptr(), ws.ldz, ws.pmax.data_ptr(), B, head.A, K, idx.data_ptr(), vals.data_ptr(),
         err.data_ptr(), stream_ptr())
    return idx, vals, err


def eval_batch(model, s, s_len, a, *, head_idx=0, K=20, ks=(20,), padding_pos="end", div_table=None, k_div=1,
               bitmap=None, k_nov=1, nov_reward=1.0, want_loss=True, lut=None):
    """Logits, CE loss, top-K and reward sums of one batch, on the device.
    ``lut`` (recommenders/hip/remap.py): the top-K ids are mapped to the input
    vocabulary for the diversity reward and returned as ``idx_in`` (for the
    host repetition count), as the reference's tokenizer branch does."""
    dev = model.device
    s = s.to(dev)
    a = a.to(dev)
    B = s.shape[0]
    st = stream_ptr()
    h = model.hidden(s, s_len, slot="eval", save=False)
    head = head_for(model, head_idx)
    ws, _ = head.logits_T(h, slot="eval")
    out = EvalBatch()
    if want_loss:
        call("rg_lse_combine", ws.pmax.data_ptr(), ws.psum.data_ptr(), ws.parg.data_ptr(), B, ws.nJ,
             ws.work.data_ptr(), ws.ZT.data_ptr(), ws.ldz, a.data_ptr(), head.A, ws.lse.data_ptr(),
             ws.amax.data_ptr(), ws.loss_row.data_ptr(), None, st)
        loss = torch.empty(1, device=dev)
        call("rg_sum_scale", ws.loss_row.data_ptr(), B, _f32(1.0 / B), loss.data_ptr(), None, st)
        out.loss = loss
    idx, vals, err = topk_device(head, ws, B, K)
    out.idx, out.vals = idx, vals
    out.idx_in = idx
    if lut is not None:
        from .remap import remap_ids
        out.idx_in = remap_ids(idx, lut, err)
    sums = torch.zeros(2 * len(ks), dtype=torch.float64, device=dev)
    ks_host = (ctypes.c_int * len(ks))(*[int(k) for k in ks])
    call("rg_hits_ndcg", idx.data_ptr(), K, a.data_ptr(), B, ks_host, len(ks), sums.data_ptr(), st)
    out.hits, out.ndcg = sums[:len(ks)], sums[len(ks):]
    out.div = out.nov = None
    if div_table is not None:
        lens = torch.as_tensor(s_len).to(dev, torch.int64)
        div = torch.empty(B, device=dev)
        call("rg_diversity", s.data_ptr(), s.shape[1], lens.data_ptr(), 1 if padding_pos == "end" else 0,
             out.idx_in.data_ptr(), k_div, K, div_table.data_ptr(), div_table.shape[1], _f32(1e-6), B, div.data_ptr(),
             st)
        out.div = div
    if bitmap is not None:
        nov = torch.empty(B, device=dev)
        call("rg_novelty", idx.data_ptr(), k_nov, K, bitmap.data_ptr(), _f32(nov_reward), B, nov.data_ptr(), st)
        out.nov = nov
    e = int(err.item())
    if e & 2:
        raise RuntimeError("rg_topk candidate overflow (massive exact ties in the logits)")
    if e & 1:
        from .remap import RemapError
        raise RemapError("a predicted id has no input-vocabulary token (input_tokenizer.stoi(output_tokenizer.itos(id)))")
    return out
