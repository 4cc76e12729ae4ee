"""CPU restatement of the reference's four training steps (TEST INFRA ONLY).

See ``oracle/__init__.py`` for the rules.  Reference anchors:

* GRU4Rec net + step:      recommenders/models/GRU4Rec/model.py:6-82, 129-155
* BidirGRU4Rec net + step: recommenders/models/BidirGRU4Rec/model.py:7-101, 150-176
* SQN double-Q step:       recommenders/models/SQN/sqn_gru.py:10-112, 183-254
* SMORL 3-reward step:     recommenders/models/SMORL/smorl_gru.py:14-139, 233-334
  (shipped step is broken at :311 — 2 rewards vs 3 heads — so the 3-reward
  step here is *composed* from the reference's helpers)

The nets are plain ``nn.Module`` containers whose state_dict keys equal the
reference's (``embedding.weight``, ``gru.*`` / ``base_model.*``, head names),
constructed in the same order after the same seeding so that initial weights
are bit-identical to the reference's.
"""
from __future__ import annotations

import math
import random

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from .metrics import (
    batch_diversity_rewards,
    batch_novelty_rewards,
    gather_heads,
    weighted_heads,
)

HEADS = {
    "gru4rec": ("gru", ["output"]),
    "bidir": ("gru", ["output"]),
    "sqn": ("base_model", ["sup_head_output", "q_head_output"]),
    "smorl": ("base_model", ["sup_head_output", "q_head_acc", "q_head_div", "q_head_nov"]),
}


class _Fp16Storage(torch.autograd.Function):
    """Forward: the table as stored in fp16 (round to nearest even), widened
    back to fp32.  Backward: the fp32 gradient unchanged (it lands on the fp32
    master weights).  Build-defined C5 option; no reference counterpart."""

    @staticmethod
    def forward(ctx, w):
        return w.half().float()

    @staticmethod
    def backward(ctx, g):
        return g


class Net(nn.Module):
    """Embedding -> GRU -> layer-0 final hidden -> linear heads.

    Construction order (hence RNG consumption) follows the reference:
    embedding (N(0,1) default init, then ``normal_(0, 0.01)``,
    ``GRU4Rec/model.py:36-47``), then the GRU (``:49-55``), then the heads in
    declaration order (``:58-60``; ``sqn_gru.py:78-85``; ``smorl_gru.py:85-102``).
    """

    def __init__(self, kind, item_num, action_dim, embedding_dim, hidden_dim,
                 gru_layers=1, train_pad_embed=True, use_packed_seq=True,
                 padding_idx=None, dropout=0.0, emb_fp16=False):
        super().__init__()
        self.emb_fp16 = emb_fp16
        self.kind = kind
        self.item_num = int(item_num)
        self.action_dim = action_dim
        self.use_packed_seq = use_packed_seq
        pad = self.item_num if padding_idx is None else padding_idx
        # SQN/SMORL force a trainable pad row when packing (sqn_gru.py:45-48).
        if kind in ("sqn", "smorl") and use_packed_seq:
            train_pad_embed = True
        self.pad = pad
        self.embedding = nn.Embedding(self.item_num + 1, embedding_dim,
                                      padding_idx=None if train_pad_embed else pad)
        self.embedding.weight.data.normal_(mean=0, std=0.01)
        if not train_pad_embed:
            with torch.no_grad():
                self.embedding.weight[pad] = torch.zeros(embedding_dim)
        trunk_name, head_names = HEADS[kind]
        bidir = kind == "bidir"
        setattr(self, trunk_name, nn.GRU(embedding_dim, hidden_dim, num_layers=gru_layers,
                                         bias=True, batch_first=True, bidirectional=bidir))
        self.trunk_name = trunk_name
        self.dropout = nn.Dropout(p=dropout) if bidir else None
        feat = hidden_dim * (2 if bidir else 1)
        self.head_names = head_names
        for name in head_names:
            setattr(self, name, nn.Linear(feat, action_dim))

    def hidden(self, s, lengths):
        """Final layer-0 hidden (``GRU4Rec/model.py:62-77``; Bidir cat ``:86-93``)."""
        if self.emb_fp16:
            emb = F.embedding(s, _Fp16Storage.apply(self.embedding.weight),
                              padding_idx=self.embedding.padding_idx)
        else:
            emb = self.embedding(s)
        if self.use_packed_seq:
            emb = nn.utils.rnn.pack_padded_sequence(emb, lengths=lengths, batch_first=True,
                                                    enforce_sorted=False)
        _, h = getattr(self, self.trunk_name)(emb)
        if self.kind == "bidir":
            h = torch.cat([h[0], h[1]], dim=1)
            return self.dropout(h)
        return h[0]  # quirk: layer 0 even when gru_layers=2

    def forward(self, s, lengths):
        h = self.hidden(s, lengths)
        outs = [getattr(self, n)(h) for n in self.head_names]
        if self.kind in ("gru4rec", "bidir"):
            return outs[0]
        if self.kind == "sqn":
            return outs[0], outs[1]
        return outs[0], torch.stack(outs[1:], dim=1)


def make_adam(net, lr):
    # GRU4Rec/model.py:124-127 — torch.optim.Adam defaults (0.9, 0.999), 1e-8.
    return torch.optim.Adam(net.parameters(), lr=lr)


_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _mix64(z):
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def sample_uniform(seed, counter, S, A):
    """Negatives of draw ``counter`` (csrc/sampled.hip:k_sample_uniform):
    hi64(splitmix64(seed + φ·(counter·S + s + 1)) · A), s < S.  Build-defined:
    the reference has no sampled softmax."""
    with np.errstate(over="ignore"):
        i = np.arange(S, dtype=np.uint64) + np.uint64(counter) * np.uint64(S) + np.uint64(1)
        x = _mix64(np.uint64(seed) + np.uint64(0x9E3779B97F4A7C15) * i)
        A = np.uint64(A)
        hi, lo = x >> np.uint64(32), x & np.uint64(0xFFFFFFFF)
        r = (hi * A + ((lo * A) >> np.uint64(32))) >> np.uint64(32)
    return r.astype(np.int64)


def sampled_ce(h, weight, bias, a, neg):
    """mean_b [logsumexp(z_pos, z_neg) − z_pos] with z = h·W[·] + b[·] over the
    target and the shared negatives (duplicates kept, no logQ correction)."""
    zpos = (h * weight[a]).sum(1) + bias[a]
    zneg = h @ weight[neg].t() + bias[neg]
    logits = torch.cat([zpos[:, None], zneg], 1)
    return F.cross_entropy(logits, torch.zeros(h.shape[0], dtype=torch.long))


def sampled_bpr(h, weight, bias, a, neg):
    """Sampled BPR (Rendle et al. 2009; build-defined, no reference counterpart):
    mean_b (1/S) Σ_s −log σ(z_pos − z_neg_s) over the shared negatives
    (duplicates and target collisions kept)."""
    zpos = (h * weight[a]).sum(1) + bias[a]
    zneg = h @ weight[neg].t() + bias[neg]
    return -F.logsigmoid(zpos[:, None] - zneg).mean()


class OracleSupervised:
    """GRU4Rec / BidirGRU4Rec trainer restatement (``GRU4Rec/model.py:86-155``).
    ``n_negatives``: the build-defined sampled softmax (config C3)."""

    def __init__(self, kind, hidden_dim, embedding_dim, gru_layers, train_pad_embed,
                 use_packed_seq, learning_rate, item_num, state_size, action_dim,
                 dropout=0.0, padding_idx=None, torch_rand_seed=118, python_rand_seed=999,
                 n_negatives=None, neg_seed=0, fp16_embeddings=False, sampled_loss="ce"):
        torch.manual_seed(torch_rand_seed)
        random.seed(python_rand_seed)
        self.sampled_loss = {"ce": sampled_ce, "bpr": sampled_bpr}[sampled_loss]
        self.net = Net(kind, item_num, action_dim, embedding_dim, hidden_dim, gru_layers,
                       train_pad_embed, use_packed_seq, padding_idx, dropout, emb_fp16=fp16_embeddings)
        self.opt = make_adam(self.net, learning_rate)
        self.n_negatives, self.neg_seed, self.draws = n_negatives, neg_seed, 0

    def step(self, s, a, true_len):
        if self.n_negatives:
            neg = torch.from_numpy(sample_uniform(self.neg_seed, self.draws, self.n_negatives,
                                                  self.net.action_dim))
            self.draws += 1
            head = getattr(self.net, self.net.head_names[0])
            loss = self.sampled_loss(self.net.hidden(s, true_len), head.weight, head.bias, a, neg)
        else:
            preds = self.net(s, true_len)
            loss = F.cross_entropy(preds, a)  # CrossEntropyLoss(reduction="mean")
        self.opt.zero_grad()
        loss.backward()
        self.opt.step()
        return loss.item()


class OracleSQN:
    """SQN double-Q trainer restatement (``sqn_gru.py:115-254``)."""

    def __init__(self, hidden_dim, embedding_dim, train_pad_embed, use_packed_seq,
                 learning_rate, item_num, state_size, action_dim, gamma, gru_layers,
                 padding_idx=None, torch_rand_seed=118, python_rand_seed=999, fp16_embeddings=False):
        torch.manual_seed(torch_rand_seed)
        random.seed(python_rand_seed)
        mk = lambda: Net("sqn", item_num, action_dim, embedding_dim, hidden_dim, gru_layers,
                         train_pad_embed, use_packed_seq, padding_idx, emb_fp16=fp16_embeddings)
        self.nets = [mk(), mk()]
        self.opts = [make_adam(n, learning_rate) for n in self.nets]
        self.gamma = gamma

    def step(self, s, a, r, s_next, true_len, true_next_len, is_end):
        r = r.unsqueeze(1)
        k = 0 if random.uniform(0, 1) <= 0.5 else 1          # sqn_gru.py:207-216
        main, boot, opt = self.nets[k], self.nets[1 - k], self.opts[k]
        sup, q_out = main(s, true_len)
        q = q_out.gather(1, a.unsqueeze(1))
        with torch.no_grad():
            _, q_next_main = main(s_next, true_next_len)
            a_star = torch.argmax(q_next_main, dim=1).unsqueeze(1)
            _, q_next_boot_all = boot(s_next, true_len)       # quirk: true_len (:231)
            q_next = q_next_boot_all.gather(1, a_star)
            q_next[is_end] = 0.0
        q_loss = torch.mean((r + self.gamma * q_next - q) ** 2)  # f64 when r is f64
        sup_loss = F.cross_entropy(sup, a)
        opt.zero_grad()
        (q_loss + sup_loss).backward()
        opt.step()
        self.last_main = k
        return sup_loss.item(), q_loss.item()


class OracleSMORL:
    """SMORL 3-reward trainer, composed from the reference helpers.

    Sequencing follows ``smorl_gru.py:247-332`` with the third (novelty)
    reward added as SURVEY.md §3.4 step 6 specifies:
    r = stack([r_acc, r_div, r_nov]).float32.  The novelty reward uses
    ``novelty.py:12-47`` with ``topk_nov`` / ``nov_rew_sig``.  This
    composition is build-defined: parity is pinned to the reference helpers,
    not to a runnable reference step (the shipped one raises).
    """

    def __init__(self, hidden_dim, embedding_dim, padding_pos, train_pad_embed,
                 use_packed_seq, learning_rate, item_num, state_size, action_dim, gamma,
                 gru_layers, q_weights, alpha, div_embedding, unpopular_actions_set,
                 topk_div, topk_nov=1, nov_rew_sig=1.0, padding_idx=None,
                 torch_rand_seed=118, python_rand_seed=999, fp16_embeddings=False):
        torch.manual_seed(torch_rand_seed)
        random.seed(python_rand_seed)
        mk = lambda: Net("smorl", item_num, action_dim, embedding_dim, hidden_dim, gru_layers,
                         train_pad_embed, use_packed_seq, padding_idx, emb_fp16=fp16_embeddings)
        self.nets = [mk(), mk()]
        self.opts = [make_adam(n, learning_rate) for n in self.nets]
        self.gamma, self.alpha = gamma, alpha
        self.w = torch.as_tensor(q_weights, dtype=torch.float32)
        self.div_embedding = div_embedding  # (N+1, E_div) float tensor, frozen
        self.unpopular = unpopular_actions_set
        self.topk_div, self.topk_nov, self.nov_rew_sig = topk_div, topk_nov, nov_rew_sig
        self.padding_pos = padding_pos

    def step(self, s, a, r_acc, s_next, true_len, true_next_len, is_end):
        k = 0 if random.uniform(0, 1) <= 0.5 else 1          # smorl_gru.py:261-266
        main, boot, opt = self.nets[k], self.nets[1 - k], self.opts[k]
        sup, q_all = main(s, true_len)
        sup_loss = F.cross_entropy(sup, a)
        q = gather_heads(q_all, a)                            # tensor_operations.py:4-33
        with torch.no_grad():
            _, q_next_all = main(s_next, true_next_len)
            a_star = torch.argmax(weighted_heads(q_next_all, self.w), dim=1)
            _, q_boot_all = boot(s_next, true_len)           # quirk: true_len (:291)
            q_next = gather_heads(q_boot_all, a_star)
            q_next[is_end, :] = 0.0
            r_div = batch_diversity_rewards(s, sup, true_next_len, self.padding_pos,
                                            self.topk_div, self.div_embedding)
            r_nov = torch.from_numpy(batch_novelty_rewards(sup, self.unpopular,
                                                           self.nov_rew_sig, self.topk_nov))
            r = torch.stack([r_acc.to(torch.float64), r_div.to(torch.float64),
                             r_nov.to(torch.float64)], dim=1).to(torch.float32)
        per_head = (r + self.gamma * q_next - q) ** 2
        q_loss = torch.mean(per_head @ self.w)               # tensor_operations.py:36-47
        loss = sup_loss + self.alpha * q_loss
        opt.zero_grad()
        loss.backward()
        opt.step()
        self.last_main = k
        self.last_rewards = r
        return sup_loss.item(), q_loss.item()
