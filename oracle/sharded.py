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


def sharded_argmax(scores_local, lo, comm):
    """Global first-maximum index per row from each rank's (max, local argmax)
    — the merge rule of csrc/shard.hip:k_argmax_merge_ranks (larger value wins,
    ties keep the lower rank = lower global index)."""
    world = comm.world
    n = scores_local.shape[0]
    mx, am = scores_local.max(1)                     # torch: first maximum
    mx_r = comm.all_gather(torch.empty(world * n, dtype=mx.dtype), mx).view(world, n)
    g_r = comm.all_gather(torch.empty(world * n, dtype=torch.int64), am + lo).view(world, n)
    out = g_r[0].clone()
    best = mx_r[0].clone()
    for r in range(1, world):
        upd = mx_r[r] > best
        out[upd] = g_r[r][upd]
        best[upd] = mx_r[r][upd]
    return out


def canonical_topk(scores, K):
    """(value desc, index asc) first K indices per row."""
    out = []
    for row in scores.tolist():
        out.append(sorted(range(len(row)), key=lambda j: (-row[j], j))[:K])
    return torch.tensor(out, dtype=torch.int64)


def sharded_topk(scores_local, K, lo, comm):
    """Global canonical top-K per row: merge of every rank's local canonical
    top-K (csrc/shard.hip:k_topk_merge_ranks)."""
    world = comm.world
    n = scores_local.shape[0]
    loc = canonical_topk(scores_local, K)
    v = torch.gather(scores_local, 1, loc)
    v_r = comm.all_gather(torch.empty(world * n * K, dtype=v.dtype), v.reshape(-1)).view(world, n, K)
    g_r = comm.all_gather(torch.empty(world * n * K, dtype=torch.int64), (loc + lo).reshape(-1)).view(world, n, K)
    out = torch.empty(n, K, dtype=torch.int64)
    for i in range(n):
        pos = [0] * world
        for q in range(K):
            best = None
            for r in range(world):
                if pos[r] >= K:
                    continue
                cand = (-float(v_r[r, i, pos[r]]), int(g_r[r, i, pos[r]]), r)
                if best is None or cand < best:
                    best = cand
            out[i, q] = best[1]
            pos[best[2]] += 1
    return out


def sharded_embedding(tok_local, table_shard, lo, n_rows, comm, dX_local=None):
    """Row-sharded nn.Embedding (csrc/emb_shard.hip) restated with plain
    collectives: every token's row fetched from its owner (route by owner,
    all-to-all of ids, owner gathers, all-to-all of rows back); with dX_local
    the row-gradients sent back to the owners and summed into the owner's
    rows.  Returns (X_local, dtable_shard)."""
    world, rank = comm.world, comm.rank
    own = ((tok_local + 1) * world + n_rows - 1) // n_rows - 1
    order = torch.sort(own, stable=True).indices
    send_ids = tok_local[order]
    counts = torch.bincount(own, minlength=world)
    M = comm.all_gather(torch.empty(world * world, dtype=torch.int64), counts).view(world, world)
    send, recv = M[rank].tolist(), M[:, rank].tolist()
    ids_in = torch.empty(sum(recv), dtype=torch.int64)
    comm.dist.all_to_all_single(ids_in, send_ids, recv, send)
    rows_out = table_shard[ids_in - lo]
    rows_in = torch.empty(sum(send), table_shard.shape[1], dtype=table_shard.dtype)
    comm.dist.all_to_all_single(rows_in, rows_out, send, recv)
    X = torch.empty_like(rows_in)
    X[order] = rows_in
    if dX_local is None:
        return X, None
    g_in = torch.empty(sum(recv), table_shard.shape[1], dtype=dX_local.dtype)
    comm.dist.all_to_all_single(g_in, dX_local[order].contiguous(), recv, send)
    dtab = torch.zeros_like(table_shard)
    dtab.index_add_(0, ids_in - lo, g_in)
    return X, dtab
