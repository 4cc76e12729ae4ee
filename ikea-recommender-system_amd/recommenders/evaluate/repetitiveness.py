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
    return repetitions_from_indices(s.cpu().numpy(), idx.cpu().numpy(), topk)
