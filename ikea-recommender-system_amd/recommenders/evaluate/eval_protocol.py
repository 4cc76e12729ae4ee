"""Drop-in ``recommenders.evaluate.eval_protocol`` (reference
``recommenders/evaluate/eval_protocol.py:1-359``).

``get_hits_for_batch`` keeps the reference's host semantics for host tensors
(HR@k = target within the first k of top-max(k); NDCG@k = 1/log2(rank+1)).
``evaluate`` / ``update_train_metrics`` take the device path for the MI355X
models: logits, CE, top-k, HR/NDCG sums, diversity and novelty run as
kernels, and only the (B, K) top-k indices are copied to the host, where
coverage and repetitions are accumulated exactly as the reference does on
its top-k lists.
"""
from __future__ import annotations

import numpy as np
import torch

from recommenders.evaluate.coverage import get_coverage, update_coverage_from_indices
from recommenders.hip.evalpath import eval_batch
from recommenders.hip.nets import HipNet
from recommenders.hip.qlearn import unpopular_bitmap


def compare_elements(array_to_check, vals_to_find):
    return np.asarray(array_to_check) == np.asarray(vals_to_find)


def check_existence_and_rank(array_to_check, vals_to_find):
    """(mask, rank) with rank = 1 + position of the target, 0 if absent."""
    eq = compare_elements(array_to_check, vals_to_find)
    mask = eq.any(1)
    rank = np.zeros(shape=len(vals_to_find))
    rank[mask] = np.argmax(eq[mask], axis=1) + 1
    return mask, rank


def hits_from_topk(idx, true_idx, top_k):
    """HR/NDCG sums from a (B, max_k) top-k index matrix (host numpy)."""
    idx = np.asarray(idx)
    tgt = np.asarray(true_idx).reshape(-1, 1)
    hits = np.zeros(len(top_k))
    ndcg = np.zeros(len(top_k))
    for i, k in enumerate(top_k):
        found, rank = check_existence_and_rank(idx[:, :k], tgt)
        hits[i] = found.sum()
        denom = np.log2(rank + 1)
        ndcg[i] = np.divide(found, denom, out=np.zeros_like(denom), where=denom != 0).sum()
    return hits, ndcg


def get_hits_for_batch(predictions, true_idx, top_k=[5, 10, 20]):
    """Reference semantics on a host (B, A) prediction tensor."""
    _, idx = torch.topk(predictions, k=max(top_k))
    return hits_from_topk(idx.numpy(), true_idx.numpy(), top_k)


def get_preds(states, true_len, model, head_idx):
    out = model(states, true_len)
    return out[head_idx] if isinstance(out, tuple) else out


_DIV = {}


def _div_table(diversity_embedding, device):
    """The frozen diversity table on the device, cached per (tensor, in-place
    version, device): the harness passes the same embedding every batch
    (trainGRU.py:199-224), a 1M x 64 table is 256 MB of H2D per call."""
    if diversity_embedding is None:
        return None
    t = diversity_embedding.weight if hasattr(diversity_embedding, "weight") else diversity_embedding
    key = (id(t), t._version, str(device))
    hit = _DIV.get(key)
    if hit is not None and hit[0] is t:
        return hit[1]
    d = t.detach().to(device, torch.float32).contiguous()
    _DIV.clear()
    _DIV[key] = (t, d)
    return d


def _lut(input_tokenizer, output_tokenizer, device):
    from recommenders.hip.remap import remap_table, tokenizers
    return remap_table(input_tokenizer, output_tokenizer, device) if tokenizers(input_tokenizer,
                                                                                output_tokenizer) else None


def _require_hip(model):
    if not isinstance(model, HipNet):
        raise TypeError("evaluate() runs the MI355X device path; pass a recommenders.models.* model")


def _check_loss_function(loss_function):
    """The device path computes mean CE (the trainers' ``cross_entropy_loss``,
    reference eval_protocol.py:182 calls ``loss_function(preds, a)``); any
    other loss is refused rather than silently replaced."""
    if loss_function is None:
        return
    ok = (isinstance(loss_function, torch.nn.CrossEntropyLoss) and loss_function.weight is None
          and loss_function.reduction == "mean" and loss_function.ignore_index == -100
          and loss_function.label_smoothing == 0.0)
    if not ok:
        raise NotImplementedError(f"evaluate(): only CrossEntropyLoss(reduction='mean') runs on the device path, "
                                  f"got {loss_function!r}")


def evaluate(evaluation_data_loader, model, device, loss_function, padding_pos, diversity_embedding,
             unpopular_actions_set, head_idx=0, topk_hr_ndcg=[5, 10, 20], topk_to_consider_div=1,
             topk_to_consider_nov=1, topk_to_consider_cov=[1, 5, 10], novelty_rew_signal=1, input_tokenizer=None,
             output_tokenizer=None):
    """Same 7-tuple as the reference (eval_protocol.py:123-263):
    (loss, hr, ndcg, coverage_res, avg_diversity_rew, avg_novelty_rew, repetitions)."""
    _require_hip(model)
    _check_loss_function(loss_function)
    model.eval()
    dev = model.device
    lut = _lut(input_tokenizer, output_tokenizer, dev)
    table = _div_table(diversity_embedding, dev)
    bitmap = unpopular_bitmap(unpopular_actions_set, model.action_dim, dev, fresh=True)
    K = max(max(topk_hr_ndcg), topk_to_consider_div, topk_to_consider_nov, max(topk_to_consider_cov))
    hr = np.zeros(len(topk_hr_ndcg))
    ndcg = np.zeros(len(topk_hr_ndcg))
    reps = np.zeros(len(topk_hr_ndcg))
    covered = {k: set() for k in topk_to_consider_cov}
    tot_div = 0.0
    tot_nov = 0.0
    loss = 0.0
    n = 0
    nb = 0
    with torch.no_grad():
        for s, a, s_len in evaluation_data_loader:
            r = eval_batch(model, s, s_len, a, head_idx=head_idx, K=K, ks=topk_hr_ndcg, padding_pos=padding_pos,
                           div_table=table, k_div=topk_to_consider_div, bitmap=bitmap, k_nov=topk_to_consider_nov,
                           nov_reward=novelty_rew_signal, lut=lut, rep_ks=topk_hr_ndcg)
            idx = r.idx.cpu().numpy()
            loss += float(r.loss.item())
            hr += r.hits.cpu().numpy()
            ndcg += r.ndcg.cpu().numpy()
            tot_div += float(r.div.double().sum().item()) if r.div is not None else 0.0
            tot_nov += float(r.nov.double().sum().item())
            covered = update_coverage_from_indices(idx, covered, topk_to_consider_cov)
            reps += r.reps.cpu().numpy()
            n += len(a)
            nb += 1
    coverage_res = get_coverage(covered, set(unpopular_actions_set), model.action_dim, topk_to_consider_cov)
    return (torch.tensor(loss / nb), hr / n, ndcg / n, coverage_res, torch.tensor(tot_div / n), tot_nov / n,
            reps / n)


def update_train_metrics(s, a, s_len, model, device, padding_pos, diversity_embedding, unpopular_actions_set,
                         actions_covered_topk_dict, head_idx=0, topk_hr_ndcg=[5, 10, 20], topk_to_consider_div=1,
                         topk_to_consider_nov=1, topk_to_consider_cov=[1, 5, 10], novelty_rew_signal=1,
                         input_tokenizer=None, output_tokenizer=None):
    """Per-batch metric update (eval_protocol.py:266-359), device path."""
    _require_hip(model)
    model.eval()
    dev = model.device
    K = max(max(topk_hr_ndcg), topk_to_consider_div, topk_to_consider_nov, max(topk_to_consider_cov))
    with torch.no_grad():
        r = eval_batch(model, s, s_len, a, head_idx=head_idx, K=K, ks=topk_hr_ndcg, padding_pos=padding_pos,
                       div_table=_div_table(diversity_embedding, dev), k_div=topk_to_consider_div,
                       bitmap=unpopular_bitmap(unpopular_actions_set, model.action_dim, dev),
                       k_nov=topk_to_consider_nov, nov_reward=novelty_rew_signal, want_loss=False,
                       lut=_lut(input_tokenizer, output_tokenizer, dev), rep_ks=topk_hr_ndcg)
        idx = r.idx.cpu().numpy()
        covered = update_coverage_from_indices(idx, actions_covered_topk_dict, topk_to_consider_cov)
        reps = r.reps.cpu().numpy().astype(np.float64)
        return (r.hits.cpu().numpy(), r.ndcg.cpu().numpy(), covered, r.div.sum(), float(r.nov.double().sum()),
                reps)
