"""Drop-in ``BidirGRU4Rec`` / ``BidirGRU4Rec_trainer`` for the MI355X
(reference ``recommenders/models/BidirGRU4Rec/model.py:7-194``).

Both directions run the same persistent GRU kernel; the backward direction
reads each row's valid prefix back to front (packed semantics) and writes its
final state into columns [H, 2H) of the (B, 2H) head input, so
``cat(h[0], h[1])`` (:90) costs nothing.  Dropout (:60,93) draws its mask from
the CPU generator exactly like the reference's CPU ``F.dropout``.
"""
import random

import torch
import torch.nn as nn

from recommenders.hip import require_gpu
from recommenders.hip.engine import AdamClock
from recommenders.hip.hostsync import HostScalars
from recommenders.hip.supervised import SupervisedNet, supervised_step
from recommenders.models.GRU4Rec.model import _AdamFacade


class BidirGRU4Rec(SupervisedNet):
    def __init__(self, hidden_size, embedding_dim, item_num, state_size, action_dim, gru_layers=1, dropout=0,
                 use_packed_seq=True, train_pad_embed=True, padding_idx=None, device="cuda", n_negatives=None,
                 neg_seed=0, fp16_embeddings=False, sampled_loss="ce"):
        super().__init__(trunk_attr="gru", head_names=["output"], hidden_dim=hidden_size,
                         embedding_dim=embedding_dim, item_num=item_num, state_size=state_size,
                         action_dim=action_dim, gru_layers=gru_layers, use_packed_seq=use_packed_seq,
                         train_pad_embed=train_pad_embed, padding_idx=padding_idx, bidir=True, device=device,
                         dropout=dropout, n_negatives=n_negatives, neg_seed=neg_seed,
                         fp16_embeddings=fp16_embeddings, sampled_loss=sampled_loss)


class BidirGRU4Rec_trainer:
    def __init__(self, hidden_dim, embedding_dim, gru_layers, dropout, train_pad_embed, use_packed_seq,
                 learning_rate, item_num, state_size, action_dim, device, padding_idx=None, torch_rand_seed=118,
                 python_rand_seed=999, n_negatives=None, neg_seed=0, fp16_embeddings=False,
                 matmul_precision="f32x6d3", sampled_loss="ce"):
        torch.manual_seed(torch_rand_seed)
        random.seed(python_rand_seed)
        self.device = require_gpu(device)
        self.gru_model = BidirGRU4Rec(hidden_size=hidden_dim, embedding_dim=embedding_dim, item_num=item_num,
                                      state_size=state_size, action_dim=action_dim, gru_layers=gru_layers,
                                      dropout=dropout, use_packed_seq=use_packed_seq,
                                      train_pad_embed=train_pad_embed, padding_idx=padding_idx,
                                      device=self.device, n_negatives=n_negatives, neg_seed=neg_seed,
                                      fp16_embeddings=fp16_embeddings, sampled_loss=sampled_loss)
        self.gru_model.set_matmul_precision(matmul_precision)
        self.learning_rate = learning_rate
        self.cross_entropy_loss = nn.CrossEntropyLoss(weight=None, reduction="mean")
        self.clock = AdamClock(learning_rate)
        self.optimizer = _AdamFacade(self.clock, [self.gru_model])

    def train_step(self, s, a, true_len):
        # the loss is read back as soon as it is final (hip/hostsync.py)
        hs = self.__dict__.setdefault("_host_scalars", HostScalars())
        supervised_step(self.gru_model, self.clock, s, a, true_len, host=hs)
        return hs.get()[0]

    def train_step_async(self, s, a, true_len):
        return supervised_step(self.gru_model, self.clock, s, a, true_len)

    def set_train(self):
        self.gru_model.train()

    def set_eval(self):
        self.gru_model.eval()

    def send_to_device(self):
        self.gru_model.to(self.device)
