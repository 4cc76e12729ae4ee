"""CPU restatement of the item-sharded softmax head (TEST INFRA ONLY).

The multi-GPU step (recommenders/hip/sharded.py) has no reference
counterpart ("parity unpinned" by the reference): it must equal ONE
reference step (GRU4Rec/model.py:129-155) on the concatenation of every
rank's batch.  This restatement checks the decomposition itself — per-rank
logits over an item shard, cross-rank LSE merge, owner-contributed target
logit, reduce-scattered dh, local dW — against the unsharded math.
"""
import torch


def sharded_ce(h_local, a_local, W_shard, b_shard, lo, hi, comm):
    world, rank = comm.world, comm.rank
    B, H = h_local.shape
    Bg = world * B
    H_all = comm.all_gather(torch.empty(Bg, H), h_local)
    a_all = comm.all_gather(torch.empty(Bg, dtype=torch.int64), a_local)
    Z = H_all @ W_shard.t() + b_shard
    lse_loc = torch.logsumexp(Z, 1)
    lse_r = comm.all_gather(torch.empty(world * Bg), lse_loc).view(world, Bg)
    lse = torch.logsumexp(lse_r, 0)
    own = (a_all >= lo) & (a_all < hi)
    zt = torch.zeros(Bg)
    zt[own] = Z[own.nonzero().squeeze(1), (a_all[own] - lo)]
    comm.all_reduce(zt)
    loss = (lse - zt).mean()
    P = torch.exp(Z - lse[:, None])
    P[own.nonzero().squeeze(1), a_all[own] - lo] -= 1.0
    dZ = P / Bg
    dW, db = dZ.t() @ H_all, dZ.sum(0)
    dh = comm.reduce_scatter(torch.empty(B, H), dZ @ W_shard)
    return loss, dh, dW, db
