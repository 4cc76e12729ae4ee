"""Item-sharded multi-GPU SQN / SMORL steps (config C4, recommenders/hip/
sharded.py: sharded_double_q_step), run as 2 ranks sharing the box's GPU with
host-staged (gloo) collectives, equal the single-GPU HIP step on the
concatenated batch.  The target argmax and the SMORL top-k lists are exact
(merged across ranks with the lowest-index tie rule), so the same actions are
bootstrapped; losses and weights follow the tolerances of
tests/test_gpu_supervised.py.  Parity unpinned by the reference (it has no
multi-GPU path): pinned to the single-GPU path, itself pinned to the golden
vectors."""
import os
import socket
import sys
import tempfile

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N, L, H, B, STEPS, WORLD = 3001, 8, 32, 64, 4, 2


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


# the module's default shapes; the C4-instantiation test overrides them (cfg)
CFG = dict(N=N, L=L, H=H, B=B, STEPS=STEPS, WORLD=WORLD, seed=33, q_weights=(1.0, 0.5, 2.0), lr=0.005)


def _batches(c=CFG):
    from recommenders.data_utils.synthetic import SessionStream
    st = SessionStream(c["N"], c["L"], c["WORLD"] * c["B"] * c["STEPS"], seed=c["seed"])
    return [st.batch(i, c["WORLD"] * c["B"]) for i in range(c["STEPS"])]


def _smorl_extras(c):
    g = torch.Generator().manual_seed(7)
    table = torch.randn(c["N"] + 1, 16, generator=g) * 0.01
    return dict(padding_pos="end", q_weights=list(c["q_weights"]), alpha=1.0, div_embedding=table,
                unpopular_actions_set=set(range(0, c["N"], 3)), nov_rew_sig=1.0)


def _common(c):
    return dict(hidden_dim=c["H"], embedding_dim=c["H"], train_pad_embed=True, use_packed_seq=True,
                learning_rate=c["lr"], item_num=c["N"], state_size=c["L"], action_dim=c["N"], gamma=0.5,
                gru_layers=1)


def _make(kind, topk, c=CFG, **extra):
    if kind == "sqn":
        from recommenders.models.SQN.sqn_gru import SQN_trainer
        return SQN_trainer(**_common(c), **extra)
    from recommenders.models.SMORL.smorl_gru import SMORL_trainer
    return SMORL_trainer(topk_div=topk[0], topk_nov=topk[1], **_smorl_extras(c), **_common(c), **extra)


def _nets(tr):
    return (tr.DQN_1, tr.DQN_2) if hasattr(tr, "DQN_1") else (tr.SMORL_1, tr.SMORL_2)


def _rank(rank, port, out, kind, topk, extra, c=CFG):
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "ikea-recommender-system_amd"))
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=c["WORLD"])
    try:
        tr = _make(kind, topk, c, device="cuda:0", shard_items=True, **extra)
        losses, rewards, stored = [], [], []
        Bk = c["B"]
        for s, a, r, sn, ln, nln, e in _batches(c):
            sl = slice(rank * Bk, (rank + 1) * Bk)
            losses.append(tr.train_step(s[sl], a[sl], r[sl], sn[sl], ln[sl], nln[sl], e[sl]))
            if kind == "smorl":
                rewards.append(tr.last_rewards.cpu().numpy())
            # did the trained net's item-sharded supervised head keep its logits for pass 2?
            stored.append(bool(_nets(tr)[getattr(tr, "last_main", 0)].sup_head_output.stored_logits()))
        res = {"losses": np.array(losses), "stored": np.array(stored)}
        if rewards:
            res["rewards"] = np.stack(rewards)
        for i, net in enumerate(_nets(tr)):
            for k, v in net.state_dict().items():
                res[f"n{i}.{k}"] = v.cpu().numpy()
        np.savez(os.path.join(out, f"rank{rank}.npz"), **res)
    finally:
        dist.destroy_process_group()


def _run_ranks(kind, topk, extra, c=CFG):
    out = tempfile.mkdtemp()
    ctx = mp.get_context("spawn")
    port = _port()
    procs = [ctx.Process(target=_rank, args=(r, port, out, kind, topk, extra, c)) for r in range(c["WORLD"])]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=600)
        assert p.exitcode == 0
    return [np.load(os.path.join(out, f"rank{r}.npz")) for r in range(c["WORLD"])]


def _check_shards(ranks, ref, c=CFG):
    from recommenders.hip.dist import item_shard
    lr = c["lr"]
    for rank, g in enumerate(ranks):
        lo, hi = item_shard(c["N"], c["WORLD"], rank)
        elo, ehi = item_shard(c["N"] + 1, c["WORLD"], rank)   # the row-sharded item table (pad row included)
        for i, net in enumerate(_nets(ref)):
            for k, v in net.state_dict().items():
                got = g[f"n{i}.{k}"]
                want = v.cpu().numpy()
                if "head" in k or k.startswith("output."):
                    want = want[lo:hi]
                elif k == "embedding.weight":
                    want = want[elo:ehi]
                assert got.shape == want.shape, (rank, k)
                d = np.abs(got - want)
                assert d.max() <= 2 * lr + 1e-5, (rank, i, k, float(d.max()))
                assert (d > 1e-4).mean() < 1e-3, (rank, i, k)


F16 = {"fp16_embeddings": True}
X6 = {"matmul_precision": "f32x6"}
X6D3 = {"matmul_precision": "f32x6d3"}


@pytest.mark.parametrize("kind,topk,extra", [("sqn", None, {}), ("smorl", (1, 1), {}), ("smorl", (3, 2), {}),
                                             ("sqn", None, F16), ("smorl", (3, 2), F16),
                                             ("smorl", (1, 1), {**F16, **X6}), ("smorl", (3, 2), {**F16, **X6}),
                                             ("sqn", None, X6D3), ("smorl", (3, 2), {**F16, **X6D3})])
def test_item_sharded_double_q_equals_single_gpu_global_batch(kind, topk, extra):
    """Heads item-sharded and the item table row-sharded (ids / rows /
    row-gradients exchanged by all-to-all, csrc/emb_shard.hip); fp16 item
    table (C5); f32x6: the supervised head on the fused path, its SMORL top-k
    from pass 1 merged across ranks."""
    sys.path.insert(0, os.path.join(REPO, "ikea-recommender-system_amd"))
    ranks = _run_ranks(kind, topk, extra)
    ref = _make(kind, topk, device="cuda", **extra)
    ref_losses = np.array([ref.train_step(s, a, r, sn, ln, nln, e) for s, a, r, sn, ln, nln, e in _batches()])
    for g in ranks:
        np.testing.assert_allclose(g["losses"], ref_losses, rtol=0, atol=1e-4)
    _check_shards(ranks, ref)


@pytest.mark.parametrize("world", [2, 3, 8])
def test_item_sharded_smorl_c4_instantiation(world):
    """The benched C4 kernels item-sharded: SMORL 3-reward, H = E = 128,
    f32x6d3 (k_flash_fwd<128, 6, 3, true> with a shard offset, the rewards'
    top-1 re-scored in fp32 and merged across ranks, k_flash_amax<128, 3,
    true> screening for the double-Q target), topk_div = topk_nov = 1,
    q_weights [1, 1, 1], and an uneven split: N = 30001 items over 2, 3 or 8
    ranks (the 30002-row item table too).  2 / 3 ranks: 64 rows each, L 50;
    8 ranks (the partition of the C4 / C5 lines): 32 rows each, L 20 — 256
    gathered rows, one whole pass-1 row block, so every rank's shard of the
    head stores its logits (k_flash_fwd<128, 6, 3, true, true> with lo != 0,
    storing z while emitting the top-1 for the cross-rank merge) and pass 2
    reads them (asserted).  Every rank equals the single-GPU step on the
    concatenated batch (losses, rewards of its rows, its shard of every
    weight), and the single-GPU step equals OracleSMORL (the reference's
    helpers composed, smorl_gru.py:233-334)."""
    import random
    sys.path.insert(0, os.path.join(REPO, "ikea-recommender-system_amd"))
    Bk, L, steps = (32, 20, 2) if world == 8 else (64, 50, 3)
    c = dict(CFG, N=30001, L=L, H=128, B=Bk, STEPS=steps, WORLD=world, seed=41, q_weights=(1.0, 1.0, 1.0),
             lr=0.01)
    extra = dict(X6D3)
    ranks = _run_ranks("smorl", (1, 1), extra, c)
    from oracle.models import OracleSMORL
    torch.set_num_threads(8)
    orc = OracleSMORL(topk_div=1, topk_nov=1, **_smorl_extras(c), **_common(c))
    rs_o = random.getstate()
    ref = _make("smorl", (1, 1), c, device="cuda", **extra)
    rs_t = random.getstate()
    assert ref.SMORL_1.sup_head_output.flash_terms(world * c["B"]) == 636
    ref_losses, ref_rewards = [], []
    for i, b in enumerate(_batches(c)):
        random.setstate(rs_o)
        so, qo = orc.step(*b)
        rs_o = random.getstate()
        random.setstate(rs_t)
        sg, qg = ref.train_step(*b)
        rs_t = random.getstate()
        assert orc.last_main == ref.last_main
        rw = ref.last_rewards.cpu().numpy()
        np.testing.assert_allclose(rw, orc.last_rewards.numpy(), rtol=0, atol=1e-5)
        assert abs(so - sg) < 1e-4 and abs(qo - qg) < 1e-5, (i, so, sg, qo, qg)
        ref_losses.append((sg, qg))
        ref_rewards.append(rw)
    ref_losses, ref_rewards = np.array(ref_losses), np.stack(ref_rewards)
    for rank, g in enumerate(ranks):
        np.testing.assert_allclose(g["losses"], ref_losses, rtol=0, atol=1e-4)
        rows = slice(rank * c["B"], (rank + 1) * c["B"])
        np.testing.assert_allclose(g["rewards"], ref_rewards[:, rows], rtol=0, atol=1e-6)
        # 256 gathered rows: the stored-logit head on every rank's shard
        assert g["stored"].all() == (world * c["B"] % 256 == 0), (rank, g["stored"])
    _check_shards(ranks, ref, c)
