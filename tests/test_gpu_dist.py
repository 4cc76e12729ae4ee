"""Item-sharded multi-GPU GRU4Rec step (recommenders/hip/sharded.py), run as
2 ranks sharing the box's GPU with host-staged (gloo) collectives, equals the
single-GPU HIP step on the concatenated batch (= one reference step on it).
Tolerances as tests/test_gpu_supervised.py."""
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
CFG = dict(hidden_dim=64, embedding_dim=64, gru_layers=1, train_pad_embed=True, use_packed_seq=True,
           learning_rate=0.005, item_num=9001, state_size=12, action_dim=9001)
B, STEPS, WORLD = 128, 3, 2


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batches(world=WORLD, bad=False):
    """bad: step 1 carries an out-of-range target on rank 0's rows and a
    negative one on rank 1's (the reference's CrossEntropyLoss raises; here a
    NaN loss row with zero gradients, on one GPU and on every rank alike)."""
    from recommenders.data_utils.synthetic import SessionStream
    st = SessionStream(CFG["item_num"], CFG["state_size"], world * B * STEPS, seed=21)
    out = [list(st.batch(i, world * B)) for i in range(STEPS)]
    if bad:
        a = out[1][1] = torch.as_tensor(out[1][1]).clone()
        a[3] = CFG["action_dim"] + 7
        a[B + 5] = -2
    return [tuple(b) for b in out]


def _rank(rank, port, out, precision, world=WORLD, extra=None, bad=False, backend="gloo"):
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "ikea-recommender-system_amd"))
    import torch.distributed as dist
    if backend == "nccl":
        torch.cuda.set_device(0)
        os.environ["RG_COMM"] = "native"   # the library's own RCCL communicator (csrc/comm.hip)
    dist.init_process_group(backend, init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        from recommenders.models.GRU4Rec.model import GRU4Rec_trainer
        tr = GRU4Rec_trainer(device="cuda:0", shard_items=True, matmul_precision=precision, **CFG, **(extra or {}))
        assert world == 1 or tr.gru_model.trunk.n_local < CFG["item_num"] + 1   # the item table is row-sharded
        losses = []
        for s, a, r, sn, ln, nln, e in _batches(world, bad):
            sl = slice(rank * B, (rank + 1) * B)
            losses.append(tr.train_step(s[sl], a[sl], ln[sl]))
        sd = {k: v.cpu().numpy() for k, v in tr.gru_model.state_dict().items()}
        head = tr.gru_model.output
        stored = bool(head.stored_logits()) if hasattr(head, "stored_logits") else False
        np.savez(os.path.join(out, f"rank{rank}.npz"), losses=np.array(losses), stored=np.array(stored), **sd)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("precision", ["f32", "f32x6", "f32x6d3"])
def test_item_sharded_step_equals_single_gpu_global_batch(precision):
    """f32x6: every rank runs the fused split-bf16 head on its item shard
    (recommenders/hip/sharded.py); compared with the single-GPU fused head."""
    sys.path.insert(0, os.path.join(REPO, "ikea-recommender-system_amd"))
    out = tempfile.mkdtemp()
    ctx = mp.get_context("spawn")
    port = _port()
    procs = [ctx.Process(target=_rank, args=(r, port, out, precision)) for r in range(WORLD)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    from recommenders.models.GRU4Rec.model import GRU4Rec_trainer
    ref = GRU4Rec_trainer(device="cuda", matmul_precision=precision, **CFG)
    ref_losses = [ref.train_step(s, a, ln) for s, a, r, sn, ln, nln, e in _batches()]
    sd = {k: v.cpu().numpy() for k, v in ref.gru_model.state_dict().items()}
    from recommenders.hip.dist import item_shard
    lr = CFG["learning_rate"]
    for rank in range(WORLD):
        g = np.load(os.path.join(out, f"rank{rank}.npz"))
        np.testing.assert_allclose(g["losses"], ref_losses, rtol=0, atol=1e-4)
        # WORLD·B = 256 gathered rows: the fused precisions keep the shard's logits for pass 2
        assert bool(g["stored"]) == (precision != "f32"), (rank, precision)
        lo, hi = item_shard(CFG["action_dim"], WORLD, rank)
        elo, ehi = item_shard(CFG["item_num"] + 1, WORLD, rank)
        for k, v in sd.items():
            got = g[k]
            want = v[lo:hi] if k.startswith("output.") else (v[elo:ehi] if k == "embedding.weight" else v)
            d = np.abs(got - want)
            assert d.max() <= 2 * lr + 1e-5, (rank, k, float(d.max()))
            assert (d > 1e-4).mean() < 1e-3, (rank, k)


@pytest.mark.parametrize("world,precision,bad", [(2, "f32x6d3", False), (3, "f32x6", False), (2, "f32x6d3", True)])
def test_item_sharded_sampled_step_equals_single_gpu_global_batch(world, precision, bad):
    """The item-sharded sampled head (engine.ShardedSampledHead,
    csrc/sampled_shard.hip: the negatives' rows by one all-reduce, the targets'
    rows by all-to-all, gradients back to their owners) with the row-sharded
    item table, 2 and 3 ranks (9001 items: an uneven split over 3): every rank
    equals the single-GPU sampled step on the concatenated batch (same
    counter-based negatives) — losses, and its shard of every weight.  bad:
    invalid targets on both ranks give the NaN loss of the one-GPU step and
    leave every weight finite and equal to it."""
    sys.path.insert(0, os.path.join(REPO, "ikea-recommender-system_amd"))
    extra = dict(n_negatives=256, neg_seed=5)
    out = tempfile.mkdtemp()
    ctx = mp.get_context("spawn")
    port = _port()
    procs = [ctx.Process(target=_rank, args=(r, port, out, precision, world, extra, bad)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    from recommenders.models.GRU4Rec.model import GRU4Rec_trainer
    ref = GRU4Rec_trainer(device="cuda", matmul_precision=precision, **CFG, **extra)
    ref_losses = [ref.train_step(s, a, ln) for s, a, r, sn, ln, nln, e in _batches(world, bad)]
    assert np.isnan(ref_losses[1]) == bad and np.isfinite(ref_losses[0])
    sd = {k: v.cpu().numpy() for k, v in ref.gru_model.state_dict().items()}
    from recommenders.hip.dist import item_shard
    lr = CFG["learning_rate"]
    for rank in range(world):
        g = np.load(os.path.join(out, f"rank{rank}.npz"))
        np.testing.assert_allclose(g["losses"], ref_losses, rtol=0, atol=1e-5)
        lo, hi = item_shard(CFG["action_dim"], world, rank)
        elo, ehi = item_shard(CFG["item_num"] + 1, world, rank)
        for k, v in sd.items():
            got = g[k]
            want = v[lo:hi] if k.startswith("output.") else (v[elo:ehi] if k == "embedding.weight" else v)
            assert got.shape == want.shape, (rank, k)
            assert np.isfinite(got).all(), (rank, k)
            d = np.abs(got - want)
            assert d.max() <= 2 * lr + 1e-5, (rank, k, float(d.max()))
            assert (d > 1e-4).mean() < 1e-3, (rank, k)


def _comm_rank(port, out):
    """One rank over the nccl backend: dist.Comm's collectives through the
    library's own RCCL communicator (csrc/comm.hip) on the current stream."""
    sys.path.insert(0, os.path.join(REPO, "ikea-recommender-system_amd"))
    import torch.distributed as dist
    torch.cuda.set_device(0)
    os.environ["RG_COMM"] = "native"
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        from recommenders.hip.dist import Comm
        c = Comm()
        assert c.rc is not None and Comm().rc == c.rc   # one communicator per process group
        g = torch.Generator(device="cuda").manual_seed(3)
        res = {}
        side = torch.cuda.Stream()
        with torch.cuda.stream(side):   # (collectives follow the caller's stream)
            for name, dt in (("f32", torch.float32), ("i32", torch.int32), ("i64", torch.int64),
                             ("f16", torch.float16)):
                x = (torch.rand((37, 5), generator=g, device="cuda") * 1000).to(dt)
                y = torch.full_like(x, 7)
                c.all_to_all(y, x, [37], [37])
                res["a2a_" + name] = bool(torch.equal(y, x))
                e = torch.empty((0, 5), dtype=dt, device="cuda")
                c.all_to_all(e, e, [0], [0])
            v = torch.rand(1001, generator=g, device="cuda")
            w = v.clone()
            c.all_reduce(w)
            res["allreduce"] = bool(torch.equal(w, v))
            wk = c.all_reduce(w, async_op=True)
            wk.wait()
            ag = torch.empty(1001, device="cuda")
            c.all_gather(ag, v)
            res["allgather"] = bool(torch.equal(ag, v))
            rs = torch.empty(1001, device="cuda")
            c.reduce_scatter(rs, v)
            res["reduce_scatter"] = bool(torch.equal(rs, v))
        torch.cuda.synchronize()
        np.savez(os.path.join(out, "comm.npz"), **{k: np.array(v) for k, v in res.items()})
    finally:
        dist.destroy_process_group()


def test_native_rccl_comm_one_rank():
    """dist.Comm on the nccl backend runs its collectives through
    csrc/comm.hip (rg_comm_*): variable all-to-all of f32 / i32 / i64 / f16
    rows and empty ones, all-reduce (and its async handle), all-gather,
    reduce-scatter — one rank, so each returns its input exactly."""
    out = tempfile.mkdtemp()
    ctx = mp.get_context("spawn")
    p = ctx.Process(target=_comm_rank, args=(_port(), out))
    p.start()
    p.join(timeout=300)
    assert p.exitcode == 0
    g = np.load(os.path.join(out, "comm.npz"))
    assert all(bool(g[k]) for k in g.files), {k: bool(g[k]) for k in g.files}
    assert len(g.files) == 7


@pytest.mark.parametrize("extra", [None, dict(n_negatives=256, neg_seed=5)], ids=["full", "sampled"])
def test_item_sharded_step_over_native_rccl_one_rank(extra):
    """The item-sharded step (full-softmax and sampled heads) with its
    collectives on the library's RCCL communicator (one rank, nccl backend)
    equals the single-GPU step."""
    sys.path.insert(0, os.path.join(REPO, "ikea-recommender-system_amd"))
    out = tempfile.mkdtemp()
    ctx = mp.get_context("spawn")
    p = ctx.Process(target=_rank, args=(0, _port(), out, "f32x6d3", 1, extra, False, "nccl"))
    p.start()
    p.join(timeout=300)
    assert p.exitcode == 0
    from recommenders.models.GRU4Rec.model import GRU4Rec_trainer
    ref = GRU4Rec_trainer(device="cuda", matmul_precision="f32x6d3", **CFG, **(extra or {}))
    ref_losses = [ref.train_step(s, a, ln) for s, a, r, sn, ln, nln, e in _batches(1)]
    sd = {k: v.cpu().numpy() for k, v in ref.gru_model.state_dict().items()}
    g = np.load(os.path.join(out, "rank0.npz"))
    np.testing.assert_allclose(g["losses"], ref_losses, rtol=0, atol=1e-5)
    lr = CFG["learning_rate"]
    for k, v in sd.items():
        d = np.abs(g[k] - v)
        assert d.max() <= 2 * lr + 1e-5, (k, float(d.max()))
        assert (d > 1e-4).mean() < 1e-3, k


def _rank_lazy(rank, port, out, lazy):
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "ikea-recommender-system_amd"))
    import torch.distributed as dist
    from recommenders.hip import engine
    engine.LAZY_ADAM = lazy
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=WORLD)
    try:
        from recommenders.data_utils.synthetic import SessionStream
        from recommenders.models.GRU4Rec.model import GRU4Rec_trainer
        tr = GRU4Rec_trainer(device="cuda:0", shard_items=True, matmul_precision="f32x6d3", **CFG)
        assert (tr.gru_model.trunk.lazy is not None) == lazy
        st = SessionStream(CFG["item_num"], CFG["state_size"], WORLD * B * 6, seed=33)
        losses = []
        for i in range(6):
            s, a, r, sn, ln, nln, e = st.batch(i, WORLD * B)
            sl = slice(rank * B, (rank + 1) * B)
            losses.append(tr.train_step(s[sl], a[sl], ln[sl]))
            if i == 2:   # a mid-run read of the whole shard (state_dict materializes every row)
                mid = tr.gru_model.state_dict()["embedding.weight"].cpu().numpy()
        sd = {k: v.cpu().numpy() for k, v in tr.gru_model.state_dict().items()}
        np.savez(os.path.join(out, f"rank{rank}_{int(lazy)}.npz"), losses=np.array(losses), mid=mid, **sd)
    finally:
        dist.destroy_process_group()


def test_item_sharded_catch_up_adam_equals_eager_bitwise():
    """The row-sharded embedding table with catch-up Adam (each owner catches
    up the rows the ranks request, engine.Trunk._exchange_rows) against the
    eager sweep of the shard: 2 ranks (gloo), 6 steps, a mid-run state_dict —
    losses and every parameter bitwise equal."""
    out = tempfile.mkdtemp()
    ctx = mp.get_context("spawn")
    for lazy in (True, False):
        port = _port()
        procs = [ctx.Process(target=_rank_lazy, args=(r, port, out, lazy)) for r in range(WORLD)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(timeout=300)
            assert p.exitcode == 0
    for rank in range(WORLD):
        a = np.load(os.path.join(out, f"rank{rank}_1.npz"))
        b = np.load(os.path.join(out, f"rank{rank}_0.npz"))
        for k in a.files:
            assert np.array_equal(a[k], b[k]), (rank, k)
