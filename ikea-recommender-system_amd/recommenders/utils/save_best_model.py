"""``SaveBestModel`` of the reference (``recommenders/utils/save_best_model.py:
4-41``): the same ``best_model.pt`` dictionary, so the unchanged harness reads
it back (``torch.load(...)["model_state_dict"]`` into ``load_state_dict``,
GRU4Rec/train.py:309-311).

Kept as the reference behaves: the comparison branch tests the builtin ``max``
(always true), so a checkpoint is written whenever the metric exceeds the best
seen (``self.max`` is stored but not consulted); the first best is 0.  On an
item-sharded (multi-GPU) model the item tables are all-gathered
(``full_state_dict``) and rank 0 writes the file.
"""
from __future__ import annotations

import torch


class SaveBestModel:
    def __init__(self, out_dir, max=True, metric_name=""):  # noqa: A002 (reference keyword)
        self.max = max
        self.best_valid_metric = 0
        self.out_dir = f"{out_dir}/best_model.pt"
        self.metric_name = metric_name

    def __call__(self, curr_valid_metric, epoch, model, model_idx=1):
        if not curr_valid_metric > self.best_valid_metric:
            return
        self.best_valid_metric = curr_valid_metric
        full = getattr(model, "full_state_dict", None)
        sd = full() if full is not None else model.state_dict()
        comm = getattr(model, "comm", None)
        if comm is not None and comm.rank != 0:
            return
        torch.save({"epoch": epoch, "model_idx": model_idx, "hidden_dim": model.hidden_dim,
                    "item_num": model.item_num, "action_dim": model.action_dim, "state_size": model.state_size,
                    "embedding_dim": model.embedding_dim, "model_state_dict": sd}, self.out_dir)
