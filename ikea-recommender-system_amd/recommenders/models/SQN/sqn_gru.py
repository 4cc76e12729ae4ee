"""Drop-in ``SQN_Network`` / ``SQN_trainer`` for the MI355X
(reference ``recommenders/models/SQN/sqn_gru.py:10-277``).

Double-Q: the main/boot choice is the reference's ``random.uniform(0, 1) <= 0.5``
on Python's global RNG (seeded at construction, :137, :207-216); only the main
network's optimizer steps; the bootstrap net runs on ``s_next`` with
``true_len`` (reference quirk, :231); the TD loss is evaluated in float64 like
the reference's float64-reward promotion.
"""
import random

import torch
import torch.nn as nn

from recommenders.hip import require_gpu
from recommenders.hip.engine import AdamClock
from recommenders.hip.hostsync import HostScalars
from recommenders.hip.dist import Comm
from recommenders.hip.qlearn import QNet, double_q_step
from recommenders.hip.sharded import sharded_double_q_step
from recommenders.models.GRU4Rec.model import _AdamFacade


class SQN_Network(QNet):
    def __init__(self, hidden_dim, item_num, state_size, action_dim, gamma, gru_layers, embedding_dim=50,
                 random_embed_init=True, train_pad_embed=True, use_packed_seq=False, padding_idx=None,
                 name="DQNetwork", device="cuda", comm=None, fp16_embeddings=False):
        if not random_embed_init:
            raise NotImplementedError("TODO: Pretrained embedings.")  # as the reference (:67-68)
        if use_packed_seq:
            train_pad_embed = True  # sqn_gru.py:45-48
        super().__init__(q_names=["q_head_output"], trunk_attr="base_model", hidden_dim=hidden_dim,
                         embedding_dim=embedding_dim, item_num=item_num, state_size=state_size,
                         action_dim=action_dim, gru_layers=gru_layers, use_packed_seq=use_packed_seq,
                         train_pad_embed=train_pad_embed, padding_idx=padding_idx, bidir=False, device=device,
                         comm=comm, fp16_embeddings=fp16_embeddings)
        self.gamma = gamma
        self.name = name
        self.random_embed_init = random_embed_init


class SQN_trainer:
    def __init__(self, hidden_dim, embedding_dim, train_pad_embed, use_packed_seq, learning_rate, item_num,
                 state_size, action_dim, gamma, gru_layers, device, padding_idx=None, torch_rand_seed=118,
                 python_rand_seed=999, name_1="SQN_1", name_2="SQN_2", shard_items=False, process_group=None,
                 fp16_embeddings=False, matmul_precision="f32x6d3"):
        torch.manual_seed(torch_rand_seed)
        random.seed(python_rand_seed)
        self.device = require_gpu(device)
        # shard_items (build extension, off by default): multi-GPU weak scaling,
        # every head item-sharded over the ranks (recommenders/hip/sharded.py)
        self.comm = Comm(process_group) if shard_items else None
        mk = lambda name: SQN_Network(hidden_dim=hidden_dim, item_num=item_num, state_size=state_size,
                                      action_dim=action_dim, gamma=gamma, gru_layers=gru_layers,
                                      embedding_dim=embedding_dim, train_pad_embed=train_pad_embed,
                                      use_packed_seq=use_packed_seq, padding_idx=padding_idx, name=name,
                                      device=self.device, comm=self.comm, fp16_embeddings=fp16_embeddings)
        self.DQN_1 = mk(name_1)
        self.DQN_2 = mk(name_2)
        # matmul_precision (build extension): arithmetic of the supervised head
        # and the Q argmax, split-bf16 "f32x6d3" (default, fp32-class) / "f32x6" /
        # "f32x9", or "f32" native fp32 MFMA (GRU4Rec/model.py)
        for net in (self.DQN_1, self.DQN_2):
            net.set_matmul_precision(matmul_precision)
        self.gamma = gamma
        self.learning_rate = learning_rate
        self.cross_entropy_loss = nn.CrossEntropyLoss(weight=None, reduction="mean")
        self.clock_1 = AdamClock(learning_rate)
        self.clock_2 = AdamClock(learning_rate)
        self.optimizer_1 = _AdamFacade(self.clock_1, [self.DQN_1])
        self.optimizer_2 = _AdamFacade(self.clock_2, [self.DQN_2])
        self.last_main = None

    def train_step_async(self, s, a, r, s_next, true_len, true_next_len, is_end, host=None):
        k = 0 if random.uniform(0, 1) <= 0.5 else 1
        self.last_main = k
        step = sharded_double_q_step if self.comm is not None else double_q_step
        return step([self.DQN_1, self.DQN_2], [self.clock_1, self.clock_2], k, s, a, r, s_next, true_len,
                    true_next_len, is_end, gamma=self.gamma, host=host)

    def train_step(self, s, a, r, s_next, true_len, true_next_len, is_end):
        """One double-Q step; returns (sup_loss, q_loss) as Python floats, read
        back as soon as they are final (hip/hostsync.py)."""
        hs = self.__dict__.setdefault("_host_scalars", HostScalars())
        self.train_step_async(s, a, r, s_next, true_len, true_next_len, is_end, host=hs)
        sup, q = hs.get()
        return sup, q

    def set_train(self):
        self.DQN_1.train()
        self.DQN_2.train()

    def set_eval(self):
        self.DQN_1.eval()
        self.DQN_2.eval()

    def send_to_device(self):
        self.DQN_1.to(self.device)
        self.DQN_2.to(self.device)
