"""GPU parity for the sampled-softmax head (config C3; csrc/sampled.hip).

The reference has no sampled softmax: parity is pinned
to the build's CPU restatement (oracle/models.py: sample_uniform, sampled_ce,
OracleSupervised(n_negatives=...)).  Tolerances as in test_gpu_supervised.py:
losses 1e-4 absolute; logits 1e-5; parameters 1e-4 for >= 99.9 % of elements,
never more than 2·lr (Adam's sign-like first steps).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def D(x, dt=None):
    t = torch.as_tensor(x).cuda()
    return t if dt is None else t.to(dt)


def run_head(B, S, A, HF, seed=0, collide=False, precision="f32"):
    """One sampled head step through the C ABI; returns device results and
    the inputs used."""
    from recommenders.hip import call, stream_ptr
    from oracle.models import sample_uniform
    g = torch.Generator().manual_seed(seed)
    h = torch.randn(B, HF, generator=g) * 0.5
    W = torch.randn(A, HF, generator=g) * 0.1
    bias = torch.randn(A, generator=g) * 0.1
    neg = torch.from_numpy(sample_uniform(seed, 0, S, A))
    tgt = torch.randint(0, A, (B,), generator=g)
    if collide:  # some targets equal negatives (and duplicated negatives)
        tgt[: min(B, S) // 2] = neg[: min(B, S) // 2]
    planes = precision.endswith("-fusedp")   # ... with h as bf16 K-planes (the GRU forward's output)
    fused = precision.endswith("-fused") or planes   # rg_sampled_logits: one launch, row-major Z
    precision = precision.replace("-fusedp", "").replace("-fused", "")
    ldz = (S + 3) // 4 * 4 if fused else (B + 3) // 4 * 4
    nT = call("rg_sampled_nparts", B, S, {"f32": 0, "f32x9": 9, "f32x6": 6}[precision])
    dh_, W_, b_, neg_, tgt_ = D(h), D(W), D(bias), D(neg, torch.int32), D(tgt)
    ZT = torch.full((B, ldz) if fused else (S, ldz), float("nan"), device="cuda")
    pm = torch.empty(nT, B, device="cuda")
    ps = torch.empty(nT, B, device="cuda")
    Wg = torch.empty(S, HF, device="cuda")
    bg = torch.empty(S, device="cuda")
    st = stream_ptr()
    if fused:
        hk = None
        if planes:
            hk = torch.empty(call("rg_head_plane_bytes", B, HF), dtype=torch.uint8, device="cuda")
            call("rg_head_planes", dh_.data_ptr(), B, HF, hk.data_ptr(), None, None, None, st)
        call("rg_sampled_logits", dh_.data_ptr(), W_.data_ptr(), b_.data_ptr(), neg_.data_ptr(), 0, 0, 0, A, B, S,
             HF, {"f32x9": 9, "f32x6": 6}[precision], ZT.data_ptr(), ldz, pm.data_ptr(), ps.data_ptr(), Wg.data_ptr(),
             bg.data_ptr(), None if hk is None else hk.data_ptr(), None, st)
    elif precision == "f32":
        call("rg_sampled_fwd", dh_.data_ptr(), W_.data_ptr(), b_.data_ptr(), neg_.data_ptr(), B, S, HF,
             ZT.data_ptr(), ldz, pm.data_ptr(), ps.data_ptr(), Wg.data_ptr(), bg.data_ptr(), st)
    else:
        terms = {"f32x9": 9, "f32x6": 6}[precision]
        work = torch.empty(call("rg_sampled_work_bytes", B, S, HF), dtype=torch.uint8, device="cuda")
        call("rg_sampled_fwd_x", dh_.data_ptr(), W_.data_ptr(), b_.data_ptr(), neg_.data_ptr(), 0, 0, 0, A, B, S,
             HF, terms, ZT.data_ptr(), ldz, pm.data_ptr(), ps.data_ptr(), Wg.data_ptr(), bg.data_ptr(),
             work.data_ptr(), st)
    lse = torch.empty(B, device="cuda")
    lrow = torch.empty(B, device="cuda")
    ids = torch.empty(B, dtype=torch.int32, device="cuda")
    dzp = torch.empty(B, device="cuda")
    gpos = torch.empty(B, HF, device="cuda")
    dhp = torch.empty(B, HF, device="cuda")
    gs = float(np.float32(1.0 / B))
    call("rg_sampled_lse", dh_.data_ptr(), W_.data_ptr(), b_.data_ptr(), tgt_.data_ptr(), B, A, HF, pm.data_ptr(),
         ps.data_ptr(), nT, gs, lse.data_ptr(), lrow.data_ptr(), ids.data_ptr(), dzp.data_ptr(), gpos.data_ptr(),
         dhp.data_ptr(), st)
    view = (lambda: ZT[:, :S].t()) if fused else (lambda: ZT[:, :B])   # (S, B) either way
    Z = view().clone()
    dbg = torch.empty(S, device="cuda")
    if fused:
        slabs = torch.empty((B + 127) // 128, S, device="cuda")
        call("rg_sampled_dz_rows", ZT.data_ptr(), ldz, lse.data_ptr(), B, S, gs, slabs.data_ptr(), dbg.data_ptr(), st)
    else:
        call("rg_sampled_dz", ZT.data_ptr(), ldz, lse.data_ptr(), B, S, gs, dbg.data_ptr(), st)
    torch.cuda.synchronize()
    out = dict(Z=Z.cpu(), Wg=Wg.cpu(), bg=bg.cpu(), lse=lse.cpu(), lrow=lrow.cpu(), ids=ids.cpu(), dzp=dzp.cpu(),
               gpos=gpos.cpu(), dhp=dhp.cpu(), dZ=view().cpu(), dbg=dbg.cpu())
    return out, dict(h=h, W=W, bias=bias, neg=neg, tgt=tgt)


def test_sample_uniform_matches_oracle_bit_exact():
    from recommenders.hip import call, stream_ptr
    from oracle.models import sample_uniform
    for seed, ctr, S, A in [(0, 0, 2048, 1_000_000), (123456789, 7, 1000, 37), (2**63 + 5, 2**40, 300, 2**31 - 1)]:
        out = torch.empty(S, dtype=torch.int32, device="cuda")
        call("rg_sample_uniform", seed, ctr, S, A, out.data_ptr(), stream_ptr())
        np.testing.assert_array_equal(out.cpu().numpy(), sample_uniform(seed, ctr, S, A))


@pytest.mark.parametrize("B,S,A,HF,collide", [(256, 256, 5000, 128, False), (37, 200, 300, 64, True),
                                              (300, 130, 100, 256, True), (128, 2048, 100000, 32, False),
                                              (2240, 2048, 50000, 256, True), (1120, 64, 700, 64, True),
                                              (416, 96, 3000, 256, False)])
@pytest.mark.parametrize("precision", ["f32", "f32x9", "f32x6", "f32x9-fused", "f32x6-fused", "f32x6-fusedp"])
def test_sampled_kernels_match_torch_fp32(B, S, A, HF, collide, precision):
    if precision != "f32" and (B % 32 or S % 32):
        pytest.skip("split-bf16 path needs B, S multiples of 32")
    o, x = run_head(B, S, A, HF, collide=collide, precision=precision)
    h, W, bias, neg, tgt = x["h"], x["W"], x["bias"], x["neg"], x["tgt"]
    zneg = h @ W[neg].t() + bias[neg]                       # (B, S)
    np.testing.assert_allclose(o["Z"].t().numpy(), zneg.numpy(), rtol=0, atol=1e-5)
    np.testing.assert_array_equal(o["Wg"].numpy(), W[neg].numpy())
    np.testing.assert_array_equal(o["bg"].numpy(), bias[neg].numpy())
    zpos = (h * W[tgt]).sum(1) + bias[tgt]
    lse = torch.logsumexp(torch.cat([zpos[:, None], zneg], 1), 1)
    np.testing.assert_allclose(o["lse"].numpy(), lse.numpy(), rtol=0, atol=1e-5)
    np.testing.assert_allclose(o["lrow"].numpy(), (lse - zpos).numpy(), rtol=0, atol=1e-5)
    np.testing.assert_array_equal(o["ids"].numpy(), tgt.numpy())
    g = 1.0 / B
    dzp = (torch.exp(zpos - lse) - 1) * g
    np.testing.assert_allclose(o["dzp"].numpy(), dzp.numpy(), rtol=0, atol=1e-6)
    np.testing.assert_allclose(o["gpos"].numpy(), (dzp[:, None] * h).numpy(), rtol=0, atol=1e-6)
    np.testing.assert_allclose(o["dhp"].numpy(), (dzp[:, None] * W[tgt]).numpy(), rtol=0, atol=1e-6)
    dZ = torch.exp(zneg - lse[:, None]) * g
    np.testing.assert_allclose(o["dZ"].t().numpy(), dZ.numpy(), rtol=1e-4, atol=1e-7)
    np.testing.assert_allclose(o["dbg"].numpy(), dZ.sum(0).numpy(), rtol=1e-4, atol=1e-6)


def test_invalid_target_gives_nan_row():
    from recommenders.hip import call, stream_ptr
    B, S, A, HF = 8, 128, 50, 32
    h = D(torch.randn(B, HF))
    W = D(torch.randn(A, HF) * 0.1)
    b = D(torch.zeros(A))
    neg = D(torch.arange(S) % A, torch.int32)
    tgt = D(torch.tensor([0, 1, 2, 3, 4, 5, 6, A]))
    ldz = 8
    ZT = torch.empty(S, ldz, device="cuda")
    pm, ps = torch.empty(1, B, device="cuda"), torch.empty(1, B, device="cuda")
    st = stream_ptr()
    call("rg_sampled_fwd", h.data_ptr(), W.data_ptr(), b.data_ptr(), neg.data_ptr(), B, S, HF, ZT.data_ptr(), ldz,
         pm.data_ptr(), ps.data_ptr(), None, None, st)
    outs = [torch.empty(B, device="cuda") for _ in range(2)]
    ids = torch.empty(B, dtype=torch.int32, device="cuda")
    dz = torch.empty(B, device="cuda")
    g2 = [torch.empty(B, HF, device="cuda") for _ in range(2)]
    call("rg_sampled_lse", h.data_ptr(), W.data_ptr(), b.data_ptr(), tgt.data_ptr(), B, A, HF, pm.data_ptr(),
         ps.data_ptr(), 1, 0.125, outs[0].data_ptr(), outs[1].data_ptr(), ids.data_ptr(), dz.data_ptr(),
         g2[0].data_ptr(), g2[1].data_ptr(), st)
    lrow = outs[1].cpu()
    assert torch.isfinite(lrow[:7]).all() and torch.isnan(lrow[7])
    assert int(ids.cpu()[7]) == -1 and float(dz.cpu()[7]) == 0.0


def test_split_precision_error_is_fp32_class():
    """f32x9 / f32x6 logits against an fp64 reference: the split-bf16 GEMM
    must be as accurate as the native fp32 MFMA path (max |error| within 2×
    (x9) / 3× (x6) of native fp32's, and both within 64 fp32 ulps of |z|max
    + Σ|h·w| scale)."""
    B, S, A, HF = 1024, 2048, 30000, 128
    errs = {}
    for prec in ("f32", "f32x9", "f32x6"):
        o, x = run_head(B, S, A, HF, precision=prec)
        h, W, bias, neg = x["h"].double(), x["W"].double(), x["bias"].double(), x["neg"]
        z64 = h @ W[neg].t() + bias[neg]
        scale = (h.abs() @ W[neg].abs().t()).max().item()
        errs[prec] = (o["Z"].t().double() - z64).abs().max().item()
        assert errs[prec] < 64 * 2.0 ** -24 * scale, (prec, errs[prec], scale)
    assert errs["f32x9"] <= 2.0 * errs["f32"] + 1e-9, errs
    assert errs["f32x6"] <= 3.0 * errs["f32"] + 1e-9, errs


@pytest.mark.parametrize("precision", ["f32x9", "f32x6", "f32x6d3"])
def test_split_precision_trainer_matches_oracle(precision):
    """GRU4Rec at C2 shapes (scaled down) with the sampled head on the split
    GEMM: same loss / weight tolerances as the native path."""
    from oracle.models import OracleSupervised
    from recommenders.data_utils.synthetic import SessionStream
    from recommenders.models.GRU4Rec.model import GRU4Rec_trainer
    E = H = 128
    N, L, B, S = 50000, 50, 1024, 2048
    cfg = dict(hidden_dim=H, embedding_dim=E, gru_layers=1, train_pad_embed=True, use_packed_seq=True,
               learning_rate=0.005, item_num=N, state_size=L, action_dim=N, n_negatives=S, neg_seed=11)
    torch.set_num_threads(8)
    orc = OracleSupervised(kind="gru4rec", **cfg)
    tr = GRU4Rec_trainer(device="cuda", matmul_precision=precision, **cfg)
    st = SessionStream(N, L, B * 3, seed=9)
    for i in range(3):
        s, a, r, sn, ln, nln, e = st.batch(i, B)
        lo = orc.step(s, a, ln)
        lg = tr.train_step(s, a, ln)
        assert abs(lo - lg) < 1e-4, (i, lo, lg)
    sd_o = orc.net.state_dict()
    for k, v in tr.gru_model.state_dict().items():
        d = (v.cpu() - sd_o[k]).abs()
        assert float(d.max()) <= 2 * cfg["learning_rate"] + 1e-5, k
        assert float((d > 1e-4).float().mean()) < 1e-3, (k, float((d > 1e-4).float().mean()))


@pytest.mark.parametrize("kind,E,H,N,L,B,S", [("gru4rec", 32, 32, 3000, 10, 256, 512),
                                              ("gru4rec", 64, 64, 20000, 20, 300, 1000),
                                              ("bidir", 32, 32, 5000, 12, 200, 256),
                                              ("gru4rec", 128, 128, 50000, 50, 1024, 2048),
                                              ("bidir", 128, 128, 50000, 50, 1024, 2048)])
def test_sampled_trainer_matches_oracle(kind, E, H, N, L, B, S):
    from oracle.models import OracleSupervised
    from recommenders.data_utils.synthetic import SessionStream
    from recommenders.models.BidirGRU4Rec.model import BidirGRU4Rec_trainer
    from recommenders.models.GRU4Rec.model import GRU4Rec_trainer
    cfg = dict(hidden_dim=H, embedding_dim=E, gru_layers=1, train_pad_embed=True, use_packed_seq=True,
               learning_rate=0.005, item_num=N, state_size=L, action_dim=N, n_negatives=S, neg_seed=11)
    torch.set_num_threads(8)
    orc = OracleSupervised(kind=kind, **cfg)
    if kind == "bidir":
        tr = BidirGRU4Rec_trainer(device="cuda", dropout=0.0, **cfg)
    else:
        tr = GRU4Rec_trainer(device="cuda", **cfg)
    st = SessionStream(N, L, B * 3, seed=9)
    for i in range(3):
        s, a, r, sn, ln, nln, e = st.batch(i, B)
        lo = orc.step(s, a, ln)
        lg = tr.train_step(s, a, ln)
        assert abs(lo - lg) < 1e-4, (i, lo, lg)
    sd_o = orc.net.state_dict()
    for k, v in tr.gru_model.state_dict().items():
        d = (v.cpu() - sd_o[k]).abs()
        assert float(d.max()) <= 2 * cfg["learning_rate"] + 1e-5, k
        assert float((d > 1e-4).float().mean()) < 1e-3, (k, float((d > 1e-4).float().mean()))
    # evaluation still scores every item with the trained head
    tr.set_eval()
    s, a, r, sn, ln, nln, e = st.batch(0, B)
    z = tr.gru_model(s.cuda(), ln).float().cpu()
    with torch.no_grad():
        orc.net.eval()
        zo = orc.net(s, ln)
    d = (z - zo).abs()
    assert float(d.mean()) < 1e-4, float(d.mean())


def _planes_ref(Wg):
    """(S, HF) fp32 rows -> the fragment-order bf16 planes of common.h
    plane_idx: [32-row block][16-deep slice j][plane p][lane (hh, n)] × 8."""
    S, HF = Wg.shape
    x = Wg.double().cpu().float()
    p0 = x.to(torch.bfloat16)
    r1 = x - p0.float()
    p1 = r1.to(torch.bfloat16)
    p2 = (r1 - p1.float()).to(torch.bfloat16)
    out = []
    for p in (p0, p1, p2):
        # (S/32, n, NS, hh, 8) -> (blk, j, hh, n, 8)
        out.append(p.view(S // 32, 32, HF // 16, 2, 8).permute(0, 2, 3, 1, 4))
    # (blk, j, p, hh, n, 8)
    return torch.stack(out, 2).contiguous().view(torch.int16).flatten()


@pytest.mark.parametrize("E,HF,emb16", [(128, 128, 0), (128, 256, 0), (64, 64, 1)])
def test_gather_neg_matches_gather_and_draw(E, HF, emb16):
    """rg_gather_neg (the sampled step's embedding gather with the negatives'
    row gather in the same launch): the embedding rows bit-equal to rg_gather,
    the negatives bit-equal to the draw / row lookup rg_sampled_logits makes
    itself, and the pre-gathered logits (draw = 2: bf16 planes, draw = 3: fp32
    fragments) bit-equal to the one-launch draw (draw = 1)."""
    from oracle.models import sample_uniform
    from recommenders.data_utils.synthetic import SessionStream
    from recommenders.hip import call, stream_ptr
    A, L, B, S = 50000, 50, 1024, 2048
    st = stream_ptr()
    g = torch.Generator().manual_seed(3)
    emb = D(torch.randn(A + 1, E, generator=g) * 0.1)
    table = emb.half() if emb16 else emb
    W = D(torch.randn(A, HF, generator=g) * 0.1)
    bias = D(torch.randn(A, generator=g) * 0.1)
    s, a, r, sn, ln, nln, e = SessionStream(A, L, B, seed=4).batch(0, B)
    s, ln = D(s), D(ln)
    perm, ls, offs = (torch.empty(B, dtype=torch.int32, device="cuda") for _ in range(3))
    offs = torch.empty(B + 1, dtype=torch.int32, device="cuda")
    call("rg_pack", ln.data_ptr(), B, L, 0, perm.data_ptr(), ls.data_ptr(), offs.data_ptr(), st)
    T = int(ln.clamp(1, L).sum())
    err = torch.zeros(1, dtype=torch.int32, device="cuda")
    X0, X1 = torch.full((T, E), float("nan"), device="cuda"), torch.full((T, E), float("nan"), device="cuda")
    t0, t1 = torch.empty(T, dtype=torch.int32, device="cuda"), torch.empty(T, dtype=torch.int32, device="cuda")
    call("rg_gather_h" if emb16 else "rg_gather", s.data_ptr(), B, L, perm.data_ptr(), ls.data_ptr(),
         offs.data_ptr(), table.data_ptr(), A + 1, E, 0, t0.data_ptr(), X0.data_ptr(), err.data_ptr(), st)
    ids = torch.full((S,), -7, dtype=torch.int32, device="cuda")
    Wg = torch.full((S, HF), float("nan"), device="cuda")
    bg = torch.full((S,), float("nan"), device="cuda")
    Wp = torch.zeros(S * HF * 6, dtype=torch.uint8, device="cuda")
    seed, counter = 11, 5
    call("rg_gather_neg", s.data_ptr(), B, L, perm.data_ptr(), ls.data_ptr(), offs.data_ptr(), table.data_ptr(),
         emb16, A + 1, E, 0, t1.data_ptr(), X1.data_ptr(), err.data_ptr(), W.data_ptr(), bias.data_ptr(), seed,
         counter, A, S, HF, ids.data_ptr(), Wg.data_ptr(), bg.data_ptr(), Wp.data_ptr(), 0, st)
    torch.cuda.synchronize()
    assert int(err) == 0
    assert torch.equal(X0, X1) and torch.equal(t0, t1)
    ref_ids = torch.from_numpy(sample_uniform(seed, counter, S, A)).cuda()
    assert torch.equal(ids.long(), ref_ids.long())
    assert torch.equal(Wg, W[ids.long()]) and torch.equal(bg, bias[ids.long()])
    assert torch.equal(Wp.view(torch.int16).cpu(), _planes_ref(Wg))
    # pre-gathered logits == the one-launch draw, bit for bit
    h = D(torch.randn(B, HF, generator=g) * 0.5)
    out = {}
    for draw in (1, 2):
        nT = call("rg_sampled_nparts", B, S, 6)
        Z = torch.full((B, S), float("nan"), device="cuda")
        pm, ps = torch.empty(nT, B, device="cuda"), torch.empty(nT, B, device="cuda")
        i2 = ids.clone() if draw == 2 else torch.full((S,), -7, dtype=torch.int32, device="cuda")
        Wg2 = Wg.clone() if draw == 2 else torch.full((S, HF), float("nan"), device="cuda")
        bg2 = bg.clone() if draw == 2 else torch.full((S,), float("nan"), device="cuda")
        call("rg_sampled_logits", h.data_ptr(), W.data_ptr(), bias.data_ptr(), i2.data_ptr(), draw, seed, counter, A,
             B, S, HF, 6, Z.data_ptr(), S, pm.data_ptr(), ps.data_ptr(), Wg2.data_ptr(), bg2.data_ptr(), None,
             Wp.data_ptr() if draw == 2 else None, st)
        torch.cuda.synchronize()
        out[draw] = (Z, pm, ps, i2, Wg2, bg2)
    for x1, x2 in zip(out[1], out[2]):
        assert torch.equal(x1, x2)
    with pytest.raises(RuntimeError):   # draw = 2 needs the planes
        call("rg_sampled_logits", h.data_ptr(), W.data_ptr(), bias.data_ptr(), ids.data_ptr(), 2, seed, counter, A,
             B, S, HF, 6, out[1][0].data_ptr(), S, out[1][1].data_ptr(), out[1][2].data_ptr(), Wg.data_ptr(),
             bg.data_ptr(), None, None, st)
    if HF > 128:
        with pytest.raises(RuntimeError):   # fp32 fragments: HF <= 128 only
            call("rg_gather_neg", s.data_ptr(), B, L, perm.data_ptr(), ls.data_ptr(), offs.data_ptr(),
                 table.data_ptr(), emb16, A + 1, E, 0, t1.data_ptr(), X1.data_ptr(), err.data_ptr(), W.data_ptr(),
                 bias.data_ptr(), seed, counter, A, S, HF, ids.data_ptr(), Wg.data_ptr(), bg.data_ptr(),
                 Wp.data_ptr(), 1, st)
        return
    # wfmt 1: the rows as fp32 fragments (common.h frag_idx), the rest unchanged;
    # draw = 3 reads them and splits in the kernel: bit-equal to draw = 1, with h
    # as fp32 rows and as its K-planes
    Wf = torch.full((S * HF,), float("nan"), device="cuda")
    ids3 = torch.full((S,), -7, dtype=torch.int32, device="cuda")
    Wg3, bg3 = torch.full((S, HF), float("nan"), device="cuda"), torch.full((S,), float("nan"), device="cuda")
    X3 = torch.full((T, E), float("nan"), device="cuda")
    call("rg_gather_neg", s.data_ptr(), B, L, perm.data_ptr(), ls.data_ptr(), offs.data_ptr(), table.data_ptr(),
         emb16, A + 1, E, 0, t1.data_ptr(), X3.data_ptr(), err.data_ptr(), W.data_ptr(), bias.data_ptr(), seed,
         counter, A, S, HF, ids3.data_ptr(), Wg3.data_ptr(), bg3.data_ptr(), Wf.data_ptr(), 1, st)
    torch.cuda.synchronize()
    assert torch.equal(X3, X0) and torch.equal(ids3, ids) and torch.equal(Wg3, Wg) and torch.equal(bg3, bg)
    # (blk, n, j, hh, q, 4) -> (blk, j, q, hh, n, 4)
    fr = Wg.view(S // 32, 32, HF // 16, 2, 2, 4).permute(0, 2, 4, 3, 1, 5).contiguous().flatten()
    assert torch.equal(Wf, fr)
    hk = torch.empty(call("rg_head_plane_bytes", B, HF), dtype=torch.uint8, device="cuda")
    call("rg_head_planes", h.data_ptr(), B, HF, hk.data_ptr(), None, None, None, st)
    for hp in (None, hk):
        Z = torch.full((B, S), float("nan"), device="cuda")
        nT = call("rg_sampled_nparts", B, S, 6)
        pm, ps = torch.empty(nT, B, device="cuda"), torch.empty(nT, B, device="cuda")
        i2, Wg2, bg2 = ids.clone(), Wg.clone(), bg.clone()
        call("rg_sampled_logits", h.data_ptr(), W.data_ptr(), bias.data_ptr(), i2.data_ptr(), 3, seed, counter, A,
             B, S, HF, 6, Z.data_ptr(), S, pm.data_ptr(), ps.data_ptr(), Wg2.data_ptr(), bg2.data_ptr(),
             None if hp is None else hp.data_ptr(), Wf.data_ptr(), st)
        torch.cuda.synchronize()
        for x1, x2 in zip(out[1], (Z, pm, ps, i2, Wg2, bg2)):
            assert torch.equal(x1, x2)
