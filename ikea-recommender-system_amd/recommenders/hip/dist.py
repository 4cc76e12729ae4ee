"""Collectives for the multi-GPU step (one process per GPU, torch.distributed).

With the "nccl" backend (= RCCL on ROCm, xGMI inside a node) device tensors
go straight to the collective; with "gloo" the same calls are staged through
host memory — used to run several ranks on one GPU in tests and on CPU.
"""
from __future__ import annotations

import torch


class Comm:
    def __init__(self, group=None):
        import torch.distributed as dist
        if not dist.is_initialized():
            raise RuntimeError("item sharding needs torch.distributed to be initialised")
        self.dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.native = dist.get_backend(group) == "nccl"

    def all_gather(self, out, inp):
        """out (world·n) ← concat over ranks of inp (n), rank-major."""
        if self.native:
            self.dist.all_gather_into_tensor(out, inp.contiguous(), group=self.group)
            return out
        parts = [torch.empty(inp.shape, dtype=inp.dtype) for _ in range(self.world)]
        self.dist.all_gather(parts, inp.detach().cpu().contiguous(), group=self.group)
        out.copy_(torch.cat(parts).view(out.shape))
        return out

    def reduce_scatter(self, out, inp):
        """out (n) ← slice `rank` of the elementwise sum over ranks of inp (world·n)."""
        if self.native:
            self.dist.reduce_scatter_tensor(out, inp.contiguous(), group=self.group)
            return out
        t = inp.detach().cpu().contiguous()
        self.dist.all_reduce(t, group=self.group)
        n = out.numel()
        out.copy_(t.view(-1)[self.rank * n:(self.rank + 1) * n].view(out.shape))
        return out

    def all_to_all(self, out, inp, out_splits, in_splits):
        """Variable all-to-all along dim 0: rows [Σ in_splits[:q], +in_splits[q])
        of ``inp`` go to rank q; ``out`` receives out_splits[q] rows from q."""
        if self.native:
            self.dist.all_to_all_single(out, inp.contiguous(), list(out_splits), list(in_splits), group=self.group)
            return out
        o = torch.empty((out.shape[0],) + tuple(out.shape[1:]), dtype=out.dtype)
        self.dist.all_to_all_single(o, inp.detach().cpu().contiguous(), list(out_splits), list(in_splits),
                                    group=self.group)
        out.copy_(o)
        return out

    def all_reduce(self, t, async_op=False):
        if self.native:
            return self.dist.all_reduce(t, group=self.group, async_op=async_op)
        c = t.detach().cpu().contiguous()
        self.dist.all_reduce(c, group=self.group)
        t.copy_(c.view(t.shape))
        return None


def item_shard(A, world, rank):
    """Contiguous, balanced item range [lo, hi) owned by `rank`."""
    return (rank * A) // world, ((rank + 1) * A) // world
