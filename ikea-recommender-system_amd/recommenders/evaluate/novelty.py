"""Novelty reward (reference ``recommenders/evaluate/novelty.py:12-47``).
Device form: ``rg_novelty`` over top-k indices and an unpopular-item bitmap."""
import numpy as np
import torch


def is_unpopular(array_element, unpopular_items):
    return array_element in unpopular_items


def get_batch_novelty_rewards(predictions, unpopular_items, reward=1, topk_to_consider=1):
    """mean over the top-k predictions of [item in unpopular set] * reward (float64, (B,))."""
    _, idx = torch.topk(predictions, k=topk_to_consider)
    idx = idx.cpu().numpy()
    flags = np.isin(idx, np.fromiter((int(x) for x in unpopular_items), dtype=np.int64))
    return (flags.astype(int) * reward).mean(axis=1)
