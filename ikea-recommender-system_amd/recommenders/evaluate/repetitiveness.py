"""Repetition counts (reference ``recommenders/evaluate/repetitiveness.py:21-57``):
per k, the number of (state item, top-k prediction) equal pairs summed over
the batch, fed from a top-k index matrix."""
import numpy as np
import torch


def repetitions_from_indices(s, idx, topk):
    s = np.asarray(s)[:, :, None]
    idx = np.asarray(idx)
    out = np.zeros(len(topk))
    for i, k in enumerate(topk):
        out[i] = (s == idx[:, None, :k]).sum()
    return out


def get_batch_repetitions(s, preds, topk=[1], input_tokenizer=None, output_tokenizer=None):
    _, idx = torch.topk(preds, k=max(topk))
    if input_tokenizer is not None:   # predicted ids back to the input vocabulary
        from recommenders.evaluate.diversity import map_ids_host
        idx = map_ids_host(idx, input_tokenizer, output_tokenizer)
    return repetitions_from_indices(s.cpu().numpy(), idx.cpu().numpy(), topk)
