"""CPU restatement of the loss-side helpers and eval metrics (TEST INFRA ONLY).

* ``gather_heads``      <- recommenders/utils/tensor_operations.py:4-33 (gather_from_3d)
* ``weighted_q_loss``   <- tensor_operations.py:36-47
* ``weighted_heads``    <- tensor_operations.py:50-70 (get_weighted_q_target)
* ``max_action``        <- tensor_operations.py:73-84
* ``last_action``       <- recommenders/evaluate/diversity.py:4-12
* ``batch_diversity_rewards`` <- diversity.py:15-73
* ``batch_novelty_rewards``   <- recommenders/evaluate/novelty.py:12-47
* ``hits_for_batch``    <- recommenders/evaluate/eval_protocol.py:26-100
"""
from __future__ import annotations

import numpy as np
import torch


def gather_heads(q, idx):
    """(B, heads, A), (B,) -> (B, heads): Q_i(s, idx_b) for every head i."""
    ix = idx.view(-1, 1, 1).expand(q.shape[0], q.shape[1], 1)
    return torch.gather(q, 2, ix).squeeze(2)


def weighted_q_loss(per_head, w):
    return torch.matmul(per_head, w)


def weighted_heads(q, w):
    """sum_i w_i Q_i -> (B, A), summed over the head axis like the reference."""
    return torch.sum(q * w.to(q.device).view(1, -1, 1), dim=1)


def max_action(q):
    return torch.argmax(q, dim=1)


def last_action(s, padding_pos, s_len=None):
    if padding_pos == "end":
        return s.gather(1, (s_len - 1).unsqueeze(1)).squeeze(1)
    return s[:, -1]


def batch_diversity_rewards(s, preds, len_states, padding_pos, topk, div_table):
    """1 - mean_k cos(D[last], D[topk_k]) with CosineSimilarity(eps=1e-6)."""
    last = last_action(s, padding_pos, len_states)
    _, idx = torch.topk(preds, k=topk)
    e_last = div_table[last].unsqueeze(1)
    e_pred = div_table[idx]
    sim = torch.nn.functional.cosine_similarity(e_last, e_pred, dim=2, eps=1e-6)
    return 1 - sim.mean(dim=1)


def batch_novelty_rewards(preds, unpopular, reward=1, topk=1):
    """mean_k [topk_k in U] * reward, float64 numpy (B,)."""
    _, idx = torch.topk(preds, k=topk)
    idx = idx.cpu().numpy()
    flags = np.isin(idx, np.fromiter(unpopular, dtype=np.int64, count=len(unpopular)))
    return (flags.astype(int) * reward).mean(axis=1)


def hits_for_batch(preds, true_idx, top_k=(5, 10, 20)):
    """Per k: number of hits and sum of 1/log2(rank+1) (rank 1-based)."""
    max_k = max(top_k)
    _, idx = torch.topk(preds, k=max_k)
    idx = idx.numpy()
    tgt = true_idx.numpy().reshape(-1, 1)
    hits = np.zeros(len(top_k))
    ndcg = np.zeros(len(top_k))
    for i, k in enumerate(top_k):
        eq = idx[:, :k] == tgt
        found = eq.any(1)
        rank = np.zeros(len(tgt))
        rank[found] = np.argmax(eq[found], axis=1) + 1
        hits[i] = found.sum()
        ndcg[i] = (1.0 / np.log2(rank[found] + 1)).sum()
    return hits, ndcg


def canonical_topk_fast(values, k):
    """canonical_topk for wide rows (A ~ 1M): argpartition down to the
    candidates >= the k-th largest value (ties at the boundary included),
    then the (value desc, index asc) order among them."""
    v = np.asarray(values)
    part = np.argpartition(-v, k - 1, axis=1)[:, :k]
    kth = np.take_along_axis(v, part, 1).min(1)
    out = np.empty((v.shape[0], k), dtype=np.int64)
    for i in range(v.shape[0]):
        cand = np.nonzero(v[i] >= kth[i])[0]
        order = np.lexsort((cand, -v[i, cand]))
        out[i] = cand[order[:k]]
    return out


def hits_from_lists(idx, true_idx, top_k=(5, 10, 20)):
    """hits_for_batch on given (B, max_k) top-k index lists (rank = first
    position of the target among the first k, eval_protocol.py:26-59, 84-98)."""
    idx = np.asarray(idx)
    tgt = np.asarray(true_idx).reshape(-1, 1)
    hits = np.zeros(len(top_k))
    ndcg = np.zeros(len(top_k))
    for i, k in enumerate(top_k):
        eq = idx[:, :k] == tgt
        found = eq.any(1)
        rank = np.zeros(len(tgt))
        rank[found] = np.argmax(eq[found], axis=1) + 1
        hits[i] = found.sum()
        ndcg[i] = (1.0 / np.log2(rank[found] + 1)).sum()
    return hits, ndcg


def target_ranks(idx, true_idx):
    """1-based position of the target in each top-k list, 0 if absent."""
    eq = np.asarray(idx) == np.asarray(true_idx).reshape(-1, 1)
    found = eq.any(1)
    r = np.zeros(len(eq), dtype=np.int64)
    r[found] = np.argmax(eq[found], axis=1) + 1
    return r


def topk_flip_report(z_ref, idx_got, idx_ref, bound):
    """Compare two canonical top-k lists of the same rows scored by z_ref (the
    reference-side logits): wherever the lists differ, the item the checked
    side put at rank j must score (under z_ref) within ``bound`` of the item
    the reference put there — a flip is allowed only between items whose
    reference logits are closer than the logit error bound.
    Returns (rows that differ, max |gap| over differing positions)."""
    z = np.asarray(z_ref, dtype=np.float64)
    vg = np.take_along_axis(z, np.asarray(idx_got, dtype=np.int64), 1)
    vr = np.take_along_axis(z, np.asarray(idx_ref, dtype=np.int64), 1)
    diff = np.asarray(idx_got) != np.asarray(idx_ref)
    gap = np.abs(vg - vr)
    worst = float(gap[diff].max()) if diff.any() else 0.0
    if worst > bound:
        raise AssertionError(f"top-k flip between items {worst:.3g} apart (bound {bound:.3g})")
    return int(diff.any(1).sum()), worst


def canonical_topk(values, k):
    """Top-k indices of each row ordered by (value desc, index asc) — the tie
    policy used when comparing against GPU top-k (SURVEY.md §7 hard parts)."""
    v = np.asarray(values)
    order = np.lexsort((np.broadcast_to(np.arange(v.shape[1]), v.shape), -v), axis=1)
    return order[:, :k]
