"""Drop-in ``SMORL_GRU_Net`` / ``SMORL_trainer`` for the MI355X
(reference ``recommenders/models/SMORL/smorl_gru.py:14-359``).

The shipped reference step stacks two rewards against three Q heads and
raises (:311 vs :137).  This step implements the 3-reward form it was written
for: r = stack([r_acc, r_div, r_nov]).float32 with the novelty
reward of ``recommenders/evaluate/novelty.py:12-47``; the stubbed kwargs
``topk_nov`` / ``nov_rew_sig`` (:219-220) are accepted.  Weighted target
argmax over Σ w_i Q_i(s', ·) runs as one fused GEMM+argmax pass over the
combined head.  Parity is pinned to the reference helpers composed in that
order (tests/golden/smorl_composed.npz).
"""
import random

import torch
import torch.nn as nn

from recommenders.hip import require_gpu
from recommenders.hip.engine import AdamClock
from recommenders.hip.hostsync import HostScalars
from recommenders.hip.dist import Comm
from recommenders.hip.qlearn import QNet, double_q_step, unpopular_bitmap
from recommenders.hip.sharded import sharded_double_q_step
from recommenders.hip.remap import RemapError, remap_table, tokenizers  # noqa: F401 (RemapError re-exported)
from recommenders.models.GRU4Rec.model import _AdamFacade


class SMORL_GRU_Net(QNet):
    def __init__(self, hidden_dim, embedding_dim, item_num, state_size, action_dim, q_weights, gamma, gru_layers=1,
                 random_embed_init=True, train_pad_embed=True, use_packed_seq=False, padding_idx=None,
                 name="SMORL_GRU_Network", device="cuda", comm=None, fp16_embeddings=False):
        if not random_embed_init:
            raise NotImplementedError("TODO: Pretrained embedings.")
        if use_packed_seq:
            train_pad_embed = True
        super().__init__(q_names=["q_head_acc", "q_head_div", "q_head_nov"], trunk_attr="base_model",
                         hidden_dim=hidden_dim, embedding_dim=embedding_dim, item_num=item_num,
                         state_size=state_size, action_dim=action_dim, gru_layers=gru_layers,
                         use_packed_seq=use_packed_seq, train_pad_embed=train_pad_embed, padding_idx=padding_idx,
                         bidir=False, device=device, comm=comm, fp16_embeddings=fp16_embeddings)
        self.q_weights = q_weights
        self.gamma = gamma
        self.name = name


class SMORL_trainer:
    def __init__(self, hidden_dim, embedding_dim, padding_pos, train_pad_embed, use_packed_seq, learning_rate,
                 item_num, state_size, action_dim, gamma, gru_layers, q_weights, alpha, div_embedding,
                 unpopular_actions_set, topk_div, device, input_tokenizer=None, output_tokenizer=None,
                 padding_idx=None, torch_rand_seed=118, python_rand_seed=999, name_1="SMORL_1", name_2="SMORL_2",
                 topk_nov=1, nov_rew_sig=1, shard_items=False, process_group=None, fp16_embeddings=False,
                 matmul_precision="f32x6d3"):
        torch.manual_seed(torch_rand_seed)
        random.seed(python_rand_seed)
        self.device = require_gpu(device)
        self.comm = Comm(process_group) if shard_items else None   # item-sharded heads (multi-GPU)
        mk = lambda name: SMORL_GRU_Net(hidden_dim=hidden_dim, item_num=item_num, state_size=state_size,
                                        action_dim=action_dim, gru_layers=gru_layers, gamma=gamma,
                                        q_weights=q_weights, embedding_dim=embedding_dim,
                                        train_pad_embed=train_pad_embed, use_packed_seq=use_packed_seq,
                                        padding_idx=padding_idx, name=name, device=self.device, comm=self.comm,
                                        fp16_embeddings=fp16_embeddings)
        self.SMORL_1 = mk(name_1)
        self.SMORL_2 = mk(name_2)
        # matmul_precision (build extension): arithmetic of the supervised head
        # and the Q argmax, split-bf16 "f32x6d3" (default, fp32-class) / "f32x6" /
        # "f32x9", or "f32" native fp32 MFMA (GRU4Rec/model.py)
        for net in (self.SMORL_1, self.SMORL_2):
            net.set_matmul_precision(matmul_precision)
            # the rewards read the supervised logits' top-k after the CE forward
            net.sup_head_output.top_k = max(int(topk_div), int(topk_nov))
        self.gamma = gamma
        self.alpha = alpha
        self.q_weights = q_weights
        self.padding_pos = padding_pos
        self.learning_rate = learning_rate
        self.cross_entropy_loss = nn.CrossEntropyLoss(weight=None, reduction="mean")
        self.input_tokenizer = input_tokenizer
        self.output_tokenizer = output_tokenizer
        self.div_embedding = div_embedding
        self.topk_div = topk_div
        self.topk_nov = topk_nov
        self.nov_rew_signal = nov_rew_sig
        self.unpopular_actions_set = unpopular_actions_set
        table = div_embedding.weight if hasattr(div_embedding, "weight") else div_embedding
        w = torch.as_tensor(q_weights, dtype=torch.float32).flatten()
        self._smorl = {
            "w": [float(x) for x in w.tolist()],
            "w_dev": w.to(self.device),
            "alpha": float(alpha),
            "topk_div": int(topk_div),
            "topk_nov": int(topk_nov),
            "nov_rew_sig": float(nov_rew_sig),
            "pad_end": padding_pos == "end",
            "div_table": table.detach().to(self.device, torch.float32).contiguous(),
            "bitmap": unpopular_bitmap(unpopular_actions_set, action_dim, self.device, fresh=True),
            # tokenizer remap of the predicted ids for the diversity reward
            # (diversity.py:55-60), tabulated once (recommenders/hip/remap.py)
            "lut": (remap_table(input_tokenizer, output_tokenizer, self.device)
                    if tokenizers(input_tokenizer, output_tokenizer) else None),
            "remap_err": torch.zeros(1, dtype=torch.int32, device=self.device),
        }
        self.clock_1 = AdamClock(learning_rate)
        self.clock_2 = AdamClock(learning_rate)
        self.optimizer_1 = _AdamFacade(self.clock_1, [self.SMORL_1])
        self.optimizer_2 = _AdamFacade(self.clock_2, [self.SMORL_2])
        self.last_main = None

    def train_step_async(self, s, a, r_acc, s_next, true_len, true_next_len, is_end, host=None):
        k = 0 if random.uniform(0, 1) <= 0.5 else 1
        self.last_main = k
        step = sharded_double_q_step if self.comm is not None else double_q_step
        return step([self.SMORL_1, self.SMORL_2], [self.clock_1, self.clock_2], k, s, a, r_acc, s_next,
                    true_len, true_next_len, is_end, gamma=self.gamma, smorl=self._smorl, host=host)

    def train_step(self, s, a, r_acc, s_next, true_len, true_next_len, is_end):
        # losses and the rewards' top-k overflow flag read back as soon as they
        # are final (hip/hostsync.py); the backward is still queued on return
        hs = self.__dict__.setdefault("_host_scalars", HostScalars())
        self.train_step_async(s, a, r_acc, s_next, true_len, true_next_len, is_end, host=hs)
        vals = hs.get()
        if len(vals) > 2 and vals[2]:   # (native fp32 head only: rg_topk's K > 32 overflow)
            (self.SMORL_1, self.SMORL_2)[self.last_main].sup_head_output.check_top_err()
        return vals[0], vals[1]

    @property
    def last_rewards(self):
        net = self.SMORL_1 if self.last_main == 0 else self.SMORL_2
        return net._last_rewards

    def set_train(self):
        self.SMORL_1.train()
        self.SMORL_2.train()

    def set_eval(self):
        self.SMORL_1.eval()
        self.SMORL_2.eval()

    def send_to_device(self):
        self.SMORL_1.to(self.device)
        self.SMORL_2.to(self.device)
