"""Catch-up Adam (csrc/optim.hip rg_lazy_*, engine.LazyRows) against the eager
dense sweep (rg_adam_rows) it replaces: the reference's torch.optim.Adam moves
every row every step (GRU4Rec/model.py:124-127,153; BidirGRU4Rec/model.py:
150-176), and replaying a row's zero-gradient steps right before it is read
must give the same fp32 numbers bit for bit — after any pattern of reads,
gradients, evaluations and checkpoints."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

dev = "cuda"


def _call(*a):
    from recommenders import hip
    return hip.call(*a)


def _st():
    from recommenders import hip
    return hip.stream_ptr()


@pytest.mark.parametrize("rows,cols,bias,half", [(5000, 64, True, False), (3001, 128, False, True),
                                                 (1000, 256, True, False), (777, 32, False, False)])
def test_lazy_rows_equal_the_eager_sweep_bitwise(rows, cols, bias, half):
    """20 table steps, each with gradients on a random row subset and reads
    (catch-ups) of other random subsets in between; then every row caught up:
    P, M, V (and the bias companion, the fp16 copy) equal the eager sweep's."""
    from recommenders.hip.engine import AdamClock, LazyRows
    g = torch.Generator().manual_seed(rows + cols)
    P0 = torch.randn(rows, cols, generator=g) * 0.05
    b0 = torch.randn(rows, generator=g) * 0.05
    eP, eM, eV = P0.clone().to(dev), torch.zeros(rows, cols, device=dev), torch.zeros(rows, cols, device=dev)
    eb, ebm, ebv = b0.clone().to(dev), torch.zeros(rows, device=dev), torch.zeros(rows, device=dev)
    lP, lM, lV = P0.clone().to(dev), torch.zeros(rows, cols, device=dev), torch.zeros(rows, cols, device=dev)
    lb, lbm, lbv = b0.clone().to(dev), torch.zeros(rows, device=dev), torch.zeros(rows, device=dev)
    l16 = torch.zeros(rows, cols, dtype=torch.float16, device=dev) if half else None
    lz = LazyRows(rows, dev)
    tab = (lP.data_ptr(), lM.data_ptr(), lV.data_ptr(), cols, None if l16 is None else l16.data_ptr(),
           lb.data_ptr() if bias else None, lbm.data_ptr() if bias else None, lbv.data_ptr() if bias else None)
    eG, lG = torch.zeros(rows, cols, device=dev), torch.zeros(rows, cols, device=dev)
    eGb, lGb = torch.zeros(rows, device=dev), torch.zeros(rows, device=dev)
    etags = torch.zeros(rows, dtype=torch.int32, device=dev)
    ltags = torch.zeros(rows, dtype=torch.int32, device=dev)
    clock = AdamClock(0.01)
    for step in range(1, 21):
        # a read of a random subset (ids with repeats and out-of-range ones) before the step
        ids = torch.randint(-3, rows + 3, (rows // 7,), generator=g).to(dev)
        lz.catch_up(tab, ids.data_ptr(), ids.numel())
        if step == 9:
            lz.materialize(tab)   # an evaluation / checkpoint in the middle
            for a, e in ((lP, eP), (lM, eM), (lV, eV)):
                assert torch.equal(a, e)
        # gradients on a random subset (some rows every step, most never)
        hot = torch.randint(0, 20, (1,), generator=g).item()
        sub = torch.unique(torch.cat([torch.arange(hot), torch.randint(0, rows, (rows // 10,), generator=g)]))
        G = torch.randn(sub.numel(), cols, generator=g) * 1e-3
        Gb = torch.randn(sub.numel(), generator=g) * 1e-3
        sd = sub.to(dev)
        for T, GG in ((eG, G), (lG, G)):
            T[sd] = GG.to(dev)
        for T, GG in ((eGb, Gb), (lGb, Gb)):
            T[sd] = GG.to(dev)
        etags[sd] = step
        ltags[sd] = step
        a6 = clock.next_args()
        st = _st()
        _call("rg_adam_rows", eP.data_ptr(), eM.data_ptr(), eV.data_ptr(), eG.data_ptr(), etags.data_ptr(), step,
              rows, cols, a6, st)
        if bias:
            _call("rg_adam_rows", eb.data_ptr(), ebm.data_ptr(), ebv.data_ptr(), eGb.data_ptr(), etags.data_ptr(),
                  step, rows, 1, a6, st)
        lz.adam(tab, lG.data_ptr(), lGb.data_ptr() if bias else None, ltags.data_ptr(), step, a6)
        # rows read right after the step are current
        rd = torch.randint(0, rows, (50,), generator=g).to(dev)
        lz.catch_up(tab, rd.data_ptr(), rd.numel())
        rl = rd.long()
        assert torch.equal(lP[rl], eP[rl]) and torch.equal(lM[rl], eM[rl]) and torch.equal(lV[rl], eV[rl])
    lz.materialize(tab)
    torch.cuda.synchronize()
    for a, e in ((lP, eP), (lM, eM), (lV, eV)):   # bit patterns: ±0 told apart
        assert torch.equal(a.view(torch.int32), e.view(torch.int32))
    if bias:
        for a, e in ((lb, eb), (lbm, ebm), (lbv, ebv)):
            assert torch.equal(a.view(torch.int32), e.view(torch.int32))
    if half:
        assert torch.equal(l16, lP.half())
    assert torch.count_nonzero(lG) == 0 and int((lz.last != 20).sum()) == 0


@pytest.mark.parametrize("cols,bias", [(64, False), (256, True)])
def test_lazy_chains_longer_than_the_lds_window_bitwise(cols, bias):
    """1100 table steps (the kernel stages the newest 1024 steps' scalars in
    LDS and reads older ones from hist): rows 0–9 get gradients every step
    (magnitudes 1e-3 down to 1e-22, so v reaches the denormal range and √v
    the scaled path), rows 10–19 are read every step, rows 20–39 at step 500
    only, the rest never until the end (m = v = 0 rows included).  Every row
    equals the eager sweep bit for bit."""
    from recommenders.hip.engine import AdamClock, LazyRows
    rows, steps = 300, 1100
    g = torch.Generator().manual_seed(cols)
    P0 = torch.randn(rows, cols, generator=g) * 0.05
    b0 = torch.randn(rows, generator=g) * 0.05
    eP, eM, eV = P0.clone().to(dev), torch.zeros(rows, cols, device=dev), torch.zeros(rows, cols, device=dev)
    eb, ebm, ebv = b0.clone().to(dev), torch.zeros(rows, device=dev), torch.zeros(rows, device=dev)
    lP, lM, lV = P0.clone().to(dev), torch.zeros(rows, cols, device=dev), torch.zeros(rows, cols, device=dev)
    lb, lbm, lbv = b0.clone().to(dev), torch.zeros(rows, device=dev), torch.zeros(rows, device=dev)
    lz = LazyRows(rows, dev)
    tab = (lP.data_ptr(), lM.data_ptr(), lV.data_ptr(), cols, None,
           lb.data_ptr() if bias else None, lbm.data_ptr() if bias else None, lbv.data_ptr() if bias else None)
    eG, lG = torch.zeros(rows, cols, device=dev), torch.zeros(rows, cols, device=dev)
    eGb, lGb = torch.zeros(rows, device=dev), torch.zeros(rows, device=dev)
    etags = torch.zeros(rows, dtype=torch.int32, device=dev)
    ltags = torch.zeros(rows, dtype=torch.int32, device=dev)
    scale = (10.0 ** -torch.linspace(3, 22, 10)).view(10, 1)
    # the first 60 steps carry gradients on rows 0-39 (so the rows read late have non-zero moments)
    early = torch.arange(40, device=dev)
    hot = torch.arange(10, device=dev)
    reads = torch.arange(10, 20, device=dev).long()
    mid = torch.arange(20, 40, device=dev).long()
    clock = AdamClock(0.01)
    st = _st()
    for step in range(1, steps + 1):
        sd = early if step <= 60 else hot
        G = torch.randn(sd.numel(), cols, generator=g) * (scale.repeat(4, 1) if step <= 60 else scale)
        Gb = G[:, 0].clone()
        eG[sd] = G.to(dev)
        lG[sd] = G.to(dev)
        eGb[sd] = Gb.to(dev)
        lGb[sd] = Gb.to(dev)
        etags[sd] = step
        ltags[sd] = step
        a6 = clock.next_args()
        _call("rg_adam_rows", eP.data_ptr(), eM.data_ptr(), eV.data_ptr(), eG.data_ptr(), etags.data_ptr(), step,
              rows, cols, a6, st)
        if bias:
            _call("rg_adam_rows", eb.data_ptr(), ebm.data_ptr(), ebv.data_ptr(), eGb.data_ptr(), etags.data_ptr(),
                  step, rows, 1, a6, st)
        lz.adam(tab, lG.data_ptr(), lGb.data_ptr() if bias else None, ltags.data_ptr(), step, a6)
        lz.catch_up(tab, reads.data_ptr(), reads.numel())
        if step == 500:
            lz.catch_up(tab, mid.data_ptr(), mid.numel())
            assert torch.equal(lP[mid], eP[mid]) and torch.equal(lV[mid], eV[mid])
    assert torch.equal(lP[reads], eP[reads]) and torch.equal(lM[reads], eM[reads])
    assert float(eV[20:40].min()) < 1.2e-38   # denormal second moments are replayed
    lz.materialize(tab)
    torch.cuda.synchronize()
    for a, e in ((lP, eP), (lM, eM), (lV, eV)):   # bit patterns: ±0 told apart
        assert torch.equal(a.view(torch.int32), e.view(torch.int32))
    if bias:
        for a, e in ((lb, eb), (lbm, ebm), (lbv, ebv)):
            assert torch.equal(a.view(torch.int32), e.view(torch.int32))


def _pair(monkeypatch, make):
    """(eager trainer, catch-up trainer) built the same way."""
    from recommenders.hip import engine
    monkeypatch.setattr(engine, "LAZY_ADAM", False)
    eager = make()
    monkeypatch.setattr(engine, "LAZY_ADAM", True)
    lazy = make()
    return eager, lazy


def _nets(tr):
    return [getattr(tr, n) for n in ("gru_model", "SMORL_1", "SMORL_2", "DQN_1", "DQN_2") if hasattr(tr, n)]


@pytest.mark.parametrize("kind", ["gru4rec_sampled", "bidir_sampled", "gru4rec_full", "smorl",
                                  "gru4rec_sampled_targets_async"])
def test_trainers_with_catch_up_adam_equal_eager_bitwise(monkeypatch, kind):
    """20 steps of a trainer with catch-up Adam vs the eager dense sweeps:
    identical losses, and after a mid-run evaluation (model forward + the
    device eval path) and a state_dict / optimizer-state read, every parameter
    and Adam moment bitwise equal — also after the run.  *_targets_async: the
    targets' catch-up on the side stream (engine.TARGETS_ASYNC)."""
    import random
    if kind.endswith("_targets_async"):
        from recommenders.hip import engine
        monkeypatch.setattr(engine, "TARGETS_ASYNC", True)
        kind = kind[:-len("_targets_async")]
    from recommenders.data_utils.synthetic import SessionStream, unpopular_items
    from recommenders.hip.evalpath import eval_batch
    N, L, E, B = 3000, 12, 64, 256
    st = SessionStream(N, L, B * 21, seed=11)
    common = dict(hidden_dim=E, embedding_dim=E, gru_layers=1, train_pad_embed=True, use_packed_seq=True,
                  learning_rate=0.01, item_num=N, state_size=L, action_dim=N)

    def make():
        if kind == "smorl":
            from recommenders.models.SMORL.smorl_gru import SMORL_trainer
            g = torch.Generator().manual_seed(7)
            div = torch.randn(N + 1, 32, generator=g) * 0.01
            return SMORL_trainer(padding_pos="end", gamma=0.5, q_weights=[1.0, 1.0, 1.0], alpha=1.0, div_embedding=div,
                                 unpopular_actions_set=unpopular_items(st.item_counts()), topk_div=1, topk_nov=1,
                                 device=dev, **common)
        if kind == "bidir_sampled":
            from recommenders.models.BidirGRU4Rec.model import BidirGRU4Rec_trainer
            return BidirGRU4Rec_trainer(dropout=0.0, n_negatives=512, device=dev, **common)
        from recommenders.models.GRU4Rec.model import GRU4Rec_trainer
        return GRU4Rec_trainer(n_negatives=512 if kind == "gru4rec_sampled" else None, device=dev, **common)

    rs = random.getstate()
    eager, lazy = _pair(monkeypatch, make)
    assert all(n.trunk.lazy is None for n in _nets(eager)) and all(n.trunk.lazy is not None for n in _nets(lazy))
    outs = {}
    for name, tr in (("eager", eager), ("lazy", lazy)):
        random.setstate(rs)   # the double-Q main / boot draws
        losses = []
        for i in range(20):
            b = st.batch(i, B)
            out = tr.train_step(*b) if kind == "smorl" else tr.train_step(b[0], b[1], b[4])
            losses.append(out)
            if i == 9:
                net = _nets(tr)[0]
                net.eval()
                hb = st.batch(20, B)
                z = net(hb[0].to(dev), hb[4])
                z = (z[0] if isinstance(z, tuple) else z).float().cpu()
                r = eval_batch(net, hb[0], hb[4], hb[1], K=10, ks=[10], want_loss=True)
                net.train()
                outs.setdefault(name, {})["mid"] = (z, r.idx.cpu(), float(r.loss.item()),
                                                    {k: v.cpu().clone() for k, v in net.state_dict().items()})
                opt = tr.optimizer if hasattr(tr, "optimizer") else tr.optimizer_1
                osd = opt.state_dict()
                outs[name]["opt"] = {k: {kk: (vv.cpu().clone() if torch.is_tensor(vv) else vv)
                                         for kk, vv in v.items()} for k, v in osd["state"].items()}
        outs[name]["losses"] = losses
        outs[name]["final"] = [{k: v.cpu().clone() for k, v in n.state_dict().items()} for n in _nets(tr)]
    e, l = outs["eager"], outs["lazy"]
    assert e["losses"] == l["losses"]
    assert torch.equal(e["mid"][0], l["mid"][0]) and torch.equal(e["mid"][1], l["mid"][1])
    assert e["mid"][2] == l["mid"][2]
    for k in e["mid"][3]:
        assert torch.equal(e["mid"][3][k], l["mid"][3][k]), k
    for k in e["opt"]:
        for kk in e["opt"][k]:
            ve, vl = e["opt"][k][kk], l["opt"][k][kk]
            assert (torch.equal(ve, vl) if torch.is_tensor(ve) else ve == vl), (k, kk)
    for se, sl in zip(e["final"], l["final"]):
        for k in se:
            assert torch.equal(se[k], sl[k]), k
