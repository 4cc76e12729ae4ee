"""Drop-in ``GRU4Rec`` / ``GRU4Rec_trainer`` for the MI355X.

Same import path, constructor signatures and methods as the reference
(``recommenders/models/GRU4Rec/model.py:6-173``); the step runs as HIP kernels
through the C ABI (recommenders/hip).  Reference quirks kept: final hidden is
``h[0]`` (layer 0) for any ``gru_layers``; init RNG order = nn.Embedding,
normal_(0, 0.01), nn.GRU, nn.Linear after ``torch.manual_seed``.
"""
import random

import torch
import torch.nn as nn

from recommenders.hip import require_gpu
from recommenders.hip.engine import AdamClock
from recommenders.hip.hostsync import HostScalars
from recommenders.hip.dist import Comm
from recommenders.hip.sharded import sharded_supervised_step
from recommenders.hip.supervised import SupervisedNet, supervised_step


class GRU4Rec(SupervisedNet):
    """embedding -> GRU -> h[0] -> Linear(H -> A) (reference ``:6-82``)."""

    def __init__(self, hidden_size, embedding_dim, item_num, state_size, action_dim, gru_layers=1,
                 use_packed_seq=True, train_pad_embed=True, padding_idx=None, device="cuda", comm=None,
                 n_negatives=None, neg_seed=0, fp16_embeddings=False, sampled_loss="ce"):
        super().__init__(trunk_attr="gru", head_names=["output"], hidden_dim=hidden_size,
                         embedding_dim=embedding_dim, item_num=item_num, state_size=state_size,
                         action_dim=action_dim, gru_layers=gru_layers, use_packed_seq=use_packed_seq,
                         train_pad_embed=train_pad_embed, padding_idx=padding_idx, bidir=False, device=device,
                         comm=comm, n_negatives=n_negatives, neg_seed=neg_seed, fp16_embeddings=fp16_embeddings,
                         sampled_loss=sampled_loss)


class _AdamFacade:
    """Stands where the reference keeps its torch.optim.Adam (``:124-127``).
    ``state_dict()`` / ``load_state_dict()`` use torch.optim.Adam's format
    (parameters indexed in registration order, per-parameter step / exp_avg /
    exp_avg_sq), so a reference optimizer loads the state of a HIP trainer and
    vice versa (true resume); item tables are whole (rows
    all-gathered on an item-sharded model)."""

    def __init__(self, clock, nets):
        self.clock = clock
        self.nets = nets

    @property
    def param_groups(self):
        c = self.clock
        return [{"lr": c.lr, "betas": (c.b1, c.b2), "eps": c.eps, "weight_decay": 0, "amsgrad": False}]

    def zero_grad(self, set_to_none=True):
        pass  # gradients never persist between steps on the HIP path

    def _params(self):
        return [(net, p) for net in self.nets for p in net.named_param_objs()]

    def state_dict(self):
        c = self.clock
        ps = self._params()
        # this torch's own Adam defaults, so torch.optim.Adam.load_state_dict accepts the groups
        group = torch.optim.Adam([torch.zeros(1, requires_grad=True)], lr=c.lr, betas=(c.b1, c.b2),
                                 eps=c.eps).state_dict()["param_groups"][0]
        group["params"] = list(range(len(ps)))
        state = {}
        if c.t > 0:
            for i, (net, p) in enumerate(ps):
                state[i] = {"step": torch.tensor(float(c.t)), "exp_avg": net.gather_rows(p.name, p.m.detach()),
                            "exp_avg_sq": net.gather_rows(p.name, p.v.detach())}
        return {"state": state, "param_groups": [group]}

    def load_state_dict(self, sd):
        ps = self._params()
        groups = sd["param_groups"]
        if len(groups) != 1 or len(groups[0]["params"]) != len(ps):
            raise ValueError("loaded state dict has a different number of parameter groups / parameters")
        g = groups[0]
        if g.get("weight_decay", 0) or g.get("amsgrad", False) or g.get("maximize", False):
            raise NotImplementedError("only plain Adam (no weight decay / amsgrad / maximize) is on the HIP path")
        c = self.clock
        c.lr, (c.b1, c.b2), c.eps = float(g["lr"]), tuple(g["betas"]), float(g["eps"])
        steps = set()
        with torch.no_grad():
            for key, (net, p) in zip(g["params"], ps):
                st = sd["state"].get(key)
                if st is None:
                    p.m.zero_()
                    p.v.zero_()
                    continue
                steps.add(int(float(st["step"])))
                for dst, src in ((p.m, st["exp_avg"]), (p.v, st["exp_avg_sq"])):
                    t = torch.as_tensor(src)
                    if tuple(t.shape) != tuple(dst.shape):
                        lo, hi = net.shard_ranges().get(p.name, (0, t.shape[0]))
                        t = t[lo:hi]
                    if tuple(t.shape) != tuple(dst.shape):
                        raise RuntimeError(f"optimizer state size mismatch for {p.name}")
                    dst.copy_(t.to(dst.device, torch.float32))
        if len(steps) > 1:
            raise NotImplementedError("per-parameter Adam step counts differ; the HIP path keeps one clock")
        c.t = steps.pop() if steps else 0


class GRU4Rec_trainer:
    def __init__(self, hidden_dim, embedding_dim, gru_layers, train_pad_embed, use_packed_seq, learning_rate,
                 item_num, state_size, action_dim, device, padding_idx=None, torch_rand_seed=118,
                 python_rand_seed=999, shard_items=False, process_group=None, n_negatives=None, neg_seed=0,
                 fp16_embeddings=False, matmul_precision="f32x6d3", sampled_loss="ce"):
        torch.manual_seed(torch_rand_seed)
        random.seed(python_rand_seed)
        self.device = require_gpu(device)
        # shard_items (build extension, off by default): multi-GPU weak scaling —
        # this rank trains its own batch shard, the output layer is split over
        # the ranks by item id (recommenders/hip/sharded.py).
        self.comm = Comm(process_group) if shard_items else None
        # n_negatives (build extension, off by default): sampled softmax over the
        # target and n_negatives shared uniform negatives instead of the full
        # softmax (config C3; recommenders/hip/engine.py:SampledSoftmaxHead);
        # sampled_loss "bpr" trains the same logits with the pairwise BPR loss.
        # fp16_embeddings (build extension, off by default): the gather reads an
        # fp16 copy of the item table, Adam keeps the fp32 master (config C5).
        self.gru_model = GRU4Rec(hidden_size=hidden_dim, embedding_dim=embedding_dim, item_num=item_num,
                                 state_size=state_size, action_dim=action_dim, gru_layers=gru_layers,
                                 use_packed_seq=use_packed_seq, train_pad_embed=train_pad_embed,
                                 padding_idx=padding_idx, device=self.device, comm=self.comm,
                                 n_negatives=n_negatives, neg_seed=neg_seed, fp16_embeddings=fp16_embeddings,
                                 sampled_loss=sampled_loss)
        # matmul_precision (build extension): "f32x6d3" (default: the fused
        # split-bf16 head, fp32-class — every output within 2x of the reference
        # CPU fp32 path's error against fp64), "f32x6" / "f32x9", or
        # "f32" (native fp32 MFMA, logits stored) (hip/engine.py)
        self.gru_model.set_matmul_precision(matmul_precision)
        self.learning_rate = learning_rate
        self.cross_entropy_loss = nn.CrossEntropyLoss(weight=None, reduction="mean")
        self.clock = AdamClock(learning_rate)
        self.optimizer = _AdamFacade(self.clock, [self.gru_model])

    def train_step(self, s, a, true_len):
        """One step on (s, a, true_len); returns the CE loss as a Python float
        (with shard_items: the mean over every rank's rows).  The loss is read
        back as soon as it is final (hip/hostsync.py): the backward and the
        Adam sweeps are still queued when this returns."""
        hs = self.__dict__.setdefault("_host_scalars", HostScalars())
        if self.comm is not None:
            sharded_supervised_step(self.gru_model, self.clock, s, a, true_len, host=hs)
        else:
            supervised_step(self.gru_model, self.clock, s, a, true_len, host=hs)
        return hs.get()[0]

    def train_step_async(self, s, a, true_len):
        """Same step without the host sync; returns the device loss tensor."""
        if self.comm is not None:
            return sharded_supervised_step(self.gru_model, self.clock, s, a, true_len)
        return supervised_step(self.gru_model, self.clock, s, a, true_len)

    def set_train(self):
        self.gru_model.train()

    def set_eval(self):
        self.gru_model.eval()

    def send_to_device(self):
        self.gru_model.to(self.device)
