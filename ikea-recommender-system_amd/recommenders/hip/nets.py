"""Model objects mirroring the reference nn.Modules' public surface
(``forward(s, lengths)``, ``.action_dim`` / ``.hidden_dim`` / ``.item_num`` /
``.state_size`` / ``.embedding_dim``, ``train()/eval()/.training``,
``state_dict()/load_state_dict()`` with the reference key names — SURVEY §8b),
backed by the HIP trunk and heads of engine.py.
"""
from __future__ import annotations

from collections import OrderedDict

import numpy as np
import torch

from . import call, stream_ptr
from .engine import SampledSoftmaxHead, ShardedSampledHead, SoftmaxHead, Trunk



_LOGGED_PRECISIONS = set()


def _log_precision_once(precision):
    """Say once per process which head arithmetic the trainers run (the
    default "f32x6d3" runs dh on three bf16 plane products)."""
    if precision not in _LOGGED_PRECISIONS:
        _LOGGED_PRECISIONS.add(precision)
        import logging
        logging.getLogger("recommenders").info(
            "head matmul_precision=%s (f32: native fp32 MFMA; f32x9 / f32x6: fp32 operands split into bf16 planes; "
            "f32x6d3: f32x6 with dh on three plane products)", precision)


class HipNet:
    """Embedding + GRU trunk + linear heads, parameters on one MI355X."""

    kind = "gru4rec"

    def __init__(self, *, trunk_attr, head_names, hidden_dim, embedding_dim, item_num, state_size, action_dim,
                 gru_layers, use_packed_seq, train_pad_embed, padding_idx, bidir, device, dropout=0.0,
                 comm=None, n_negatives=None, neg_seed=0, fp16_embeddings=False, sampled_loss="ce"):
        self.hidden_dim = hidden_dim
        self.embedding_dim = embedding_dim
        self.item_num = int(item_num)
        self.state_size = state_size
        self.action_dim = action_dim
        self.use_packed_seq = use_packed_seq
        self.gru_layers = gru_layers
        self.layers = gru_layers
        self.device = torch.device(device)
        self.padding_idx = self.item_num if padding_idx is None else padding_idx
        self.dropout_p = float(dropout)
        self.training = True
        # with comm (multi-GPU) the item table is row-sharded across the ranks
        # (csrc/emb_shard.hip) and every head item-sharded (sharded.py)
        self.trunk = Trunk(trunk_attr, self.item_num, embedding_dim, hidden_dim, gru_layers, train_pad_embed,
                           use_packed_seq, self.padding_idx, bidir, self.device, fp16_embeddings=fp16_embeddings,
                           comm=comm)
        self.hf = hidden_dim * (2 if bidir else 1)
        self.comm = comm
        shard = None
        if comm is not None:
            from .dist import item_shard
            shard = item_shard(action_dim, comm.world, comm.rank)
        self.shard = shard
        if n_negatives:
            if comm is not None:   # item-sharded sampled head (rows move to the data, engine.ShardedSampledHead)
                self.heads = OrderedDict((n, ShardedSampledHead(n, action_dim, self.hf, self.device, n_negatives,
                                                                neg_seed, sampled_loss, comm, shard))
                                         for n in head_names)
            else:
                self.heads = OrderedDict((n, SampledSoftmaxHead(n, action_dim, self.hf, self.device, n_negatives,
                                                                neg_seed, loss=sampled_loss)) for n in head_names)
            # the split logits read h as bf16 planes written by the GRU forward
            self.trunk.emit_planes = self.hf <= 256
        else:
            self.heads = OrderedDict((n, SoftmaxHead(n, action_dim, self.hf, self.device, shard=shard))
                                     for n in head_names)
        for n, hd in self.heads.items():
            setattr(self, n, hd)
        self._dh = {}
        self._hd = {}

    # ------------------------------------------------------- nn.Module-ish --
    def set_matmul_precision(self, precision):
        """Arithmetic of the trained heads' GEMMs ("f32" native fp32 MFMA,
        "f32x9" / "f32x6" split-bf16, engine.SPLIT_TERMS): the full-softmax
        head's fused training path (csrc/head_flash.hip) or the sampled
        head's split forward (csrc/sampled.hip).  Evaluation logits and the
        Q heads' row gathers stay native fp32."""
        for hd in self.heads.values():
            hd.set_matmul_precision(precision)
        # the trunk's GEMMs (Gi, dX, the weight gradients) on the same arithmetic
        self.trunk.gemm_terms = {"f32": 0, "f32x9": 9}.get(precision, 6)
        _log_precision_once(precision)
        return self

    def named_param_objs(self):
        out = list(self.trunk.named_params())
        for hd in self.heads.values():
            out += hd.named_params()
        return out

    def state_dict(self):
        """Reference key names.  On an item-sharded (multi-GPU) model the
        item tables are this rank's rows: ``shard_ranges()`` gives them."""
        return OrderedDict((p.name, p.p.detach()) for p in self.named_param_objs())

    def shard_ranges(self):
        """name -> (lo, hi) row range this rank holds of every item-indexed
        parameter (the full range on one GPU)."""
        out = {"embedding.weight": (self.trunk.lo, self.trunk.hi)}
        for hd in list(self.heads.values()) + list(getattr(self, "q_heads", [])):
            out[hd.W.name] = out[hd.b.name] = (hd.lo, hd.hi)
        return out

    def full_size(self, name):
        """Rows of the whole item-indexed parameter ``name`` (None if not item-indexed)."""
        if name == self.trunk.emb.name:
            return self.trunk.N1
        for hd in list(self.heads.values()) + list(getattr(self, "q_heads", [])):
            if name in (hd.W.name, hd.b.name):
                return hd.A_full
        return None

    def gather_rows(self, name, local):
        """The whole tensor of item-indexed parameter ``name`` from every rank's
        rows (collective on an item-sharded model; ``local`` itself on one GPU)."""
        if self.comm is None or self.full_size(name) is None:
            return local
        from .dist import item_shard
        comm, n = self.comm, self.full_size(name)
        rows = max(item_shard(n, comm.world, q)[1] - item_shard(n, comm.world, q)[0] for q in range(comm.world))
        pad = torch.zeros((rows,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
        pad[:local.shape[0]] = local
        allr = torch.empty((comm.world * rows,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
        comm.all_gather(allr, pad)
        parts = []
        for q in range(comm.world):
            lo, hi = item_shard(n, comm.world, q)
            parts.append(allr[q * rows:q * rows + hi - lo])
        return torch.cat(parts)

    def full_state_dict(self):
        """``state_dict()`` with every item table whole: on an item-sharded
        (multi-GPU) model an all-gather of the row shards, on every rank."""
        return OrderedDict((k, self.gather_rows(k, v)) for k, v in self.state_dict().items())

    def load_state_dict(self, sd, strict=True):
        """Copies the reference-keyed tensors in; full-size item tables are
        sliced to this rank's rows on an item-sharded model."""
        objs = {p.name: p for p in self.named_param_objs()}
        missing = [k for k in objs if k not in sd]
        unexpected = [k for k in sd if k not in objs]
        if strict and (missing or unexpected):
            raise RuntimeError(f"state_dict mismatch: missing={missing} unexpected={unexpected}")
        ranges = self.shard_ranges()
        with torch.no_grad():
            for k, v in sd.items():
                if k not in objs:
                    continue
                t = torch.as_tensor(v)
                dst = objs[k].p
                if tuple(t.shape) != tuple(dst.shape) and k in ranges:
                    lo, hi = ranges[k]
                    t = t[lo:hi]
                if tuple(t.shape) != tuple(dst.shape):
                    raise RuntimeError(f"size mismatch for {k}: got {tuple(t.shape)}, model {tuple(dst.shape)}")
                dst.copy_(t.to(dst.device, torch.float32))
        self.trunk.refresh_half()
        return self

    def parameters(self):
        return [p.p for p in self.named_param_objs()]

    def named_parameters(self):
        return [(p.name, p.p) for p in self.named_param_objs()]

    def train(self, mode=True):
        self.training = mode
        return self

    def eval(self):
        return self.train(False)

    def to(self, device):
        if torch.device(device) != self.device and not (torch.device(device).type == "cuda" and
                                                         self.device.type == "cuda"):
            raise RuntimeError("HIP nets live on the MI355X they were built on")
        return self

    def __call__(self, s, lengths):
        return self.forward(s, lengths)

    # ------------------------------------------------------------ helpers --
    def dh_buffer(self, B):
        t = self._dh.get(B)
        if t is None:
            self._dh = {B: torch.empty(B, self.hf, device=self.device)}
            t = self._dh[B]
        return t

    def hidden(self, s, lengths, slot="eval", save=False):
        s = s.to(self.device)
        return self.trunk.forward(s, lengths, slot=slot, save=save)

    def dropout_mask(self, B):
        """Bernoulli(1-p) mask drawn from the CPU generator exactly like the
        reference's CPU F.dropout (noise.bernoulli_(1-p).div_(1-p))."""
        noise = torch.empty(B, self.hf).bernoulli_(1 - self.dropout_p)
        noise.div_(1 - self.dropout_p)
        return noise.to(self.device)

    def apply_mask(self, x, mask, out):
        call("rg_mask_scale", x.data_ptr(), mask.data_ptr(), 1.0, x.numel(), out.data_ptr(), stream_ptr())
        return out
