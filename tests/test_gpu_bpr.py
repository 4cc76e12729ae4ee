"""GPU parity for the sampled BPR loss (csrc/sampled.hip: rg_bpr_rows,
rg_bpr_dz; SampledSoftmaxHead(loss="bpr")).

The reference trains with CrossEntropyLoss only (GRU4Rec/model.py:121); the
north star names "sampled-softmax/BPR logits", so BPR is build-defined like
the sampled softmax and pinned to the build's CPU restatement
(oracle/models.py: sampled_bpr, OracleSupervised(sampled_loss="bpr")).
Tolerances as in test_gpu_sampled.py: losses 1e-4 absolute, per-element
kernel outputs 1e-6 / 1e-5, parameters 1e-4 for >= 99.9 % of elements and
never more than 2·lr (Adam's sign-like first steps).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def D(x, dt=None):
    t = torch.as_tensor(x).cuda()
    return t if dt is None else t.to(dt)


def bpr_kernels(B, S, A, HF, layout, seed=0, bad_target=False):
    """Logits through the sampled forward of `layout` ("zt": rg_sampled_fwd,
    Zᵀ; "rows": rg_sampled_logits f32x9, row-major Z), then the BPR kernels."""
    from recommenders.hip import call, stream_ptr
    from oracle.models import sample_uniform
    g = torch.Generator().manual_seed(seed)
    h = torch.randn(B, HF, generator=g) * 0.5
    W = torch.randn(A, HF, generator=g) * 0.1
    bias = torch.randn(A, generator=g) * 0.1
    neg = torch.from_numpy(sample_uniform(seed, 0, S, A))
    tgt = torch.randint(0, A, (B,), generator=g)
    tgt[: min(B, S) // 4] = neg[: min(B, S) // 4]          # targets colliding with negatives
    if bad_target:
        tgt[-1] = A
    dh_, W_, b_, neg_, tgt_ = D(h), D(W), D(bias), D(neg, torch.int32), D(tgt)
    st = stream_ptr()
    Wg = torch.empty(S, HF, device="cuda")
    bg = torch.empty(S, device="cuda")
    if layout == "rows":
        ldz = (S + 3) // 4 * 4
        nT = call("rg_sampled_nparts", B, S, 9)
        Z = torch.full((B, ldz), float("nan"), device="cuda")
        zsb, zss = ldz, 1
        pm, ps = torch.empty(nT, B, device="cuda"), torch.empty(nT, B, device="cuda")
        call("rg_sampled_logits", dh_.data_ptr(), W_.data_ptr(), b_.data_ptr(), neg_.data_ptr(), 0, 0, 0, A, B, S,
             HF, 9, Z.data_ptr(), ldz, pm.data_ptr(), ps.data_ptr(), Wg.data_ptr(), bg.data_ptr(), None, None, st)
        view = lambda: Z[:, :S]  # noqa: E731
    else:
        ldz = (B + 3) // 4 * 4
        nT = call("rg_sampled_nparts", B, S, 0)
        Z = torch.full((S, ldz), float("nan"), device="cuda")
        zsb, zss = 1, ldz
        pm, ps = torch.empty(nT, B, device="cuda"), torch.empty(nT, B, device="cuda")
        call("rg_sampled_fwd", dh_.data_ptr(), W_.data_ptr(), b_.data_ptr(), neg_.data_ptr(), B, S, HF,
             Z.data_ptr(), ldz, pm.data_ptr(), ps.data_ptr(), Wg.data_ptr(), bg.data_ptr(), st)
        view = lambda: Z[:, :B].t()  # noqa: E731
    zfwd = view().clone()
    zpos = torch.empty(B, device="cuda")
    lrow = torch.empty(B, device="cuda")
    ids = torch.empty(B, dtype=torch.int32, device="cuda")
    dzp = torch.empty(B, device="cuda")
    gpos = torch.empty(B, HF, device="cuda")
    dhp = torch.empty(B, HF, device="cuda")
    gs = float(np.float32(1.0 / B))
    call("rg_bpr_rows", dh_.data_ptr(), W_.data_ptr(), b_.data_ptr(), tgt_.data_ptr(), B, A, HF, Z.data_ptr(), zsb,
         zss, S, gs, zpos.data_ptr(), lrow.data_ptr(), ids.data_ptr(), dzp.data_ptr(), gpos.data_ptr(),
         dhp.data_ptr(), st)
    slabs = torch.empty((B + 127) // 128, S, device="cuda")
    dbg = torch.empty(S, device="cuda")
    call("rg_bpr_dz", Z.data_ptr(), zsb, zss, zpos.data_ptr(), B, S, gs, slabs.data_ptr(), dbg.data_ptr(), st)
    torch.cuda.synchronize()
    out = dict(Z=zfwd.cpu(), zpos=zpos.cpu(), lrow=lrow.cpu(), ids=ids.cpu(), dzp=dzp.cpu(), gpos=gpos.cpu(),
               dhp=dhp.cpu(), dZ=view().cpu(), dbg=dbg.cpu())
    return out, dict(h=h, W=W, bias=bias, neg=neg, tgt=tgt)


@pytest.mark.parametrize("B,S,A,HF", [(256, 256, 5000, 128), (64, 96, 300, 32), (320, 2048, 50000, 64),
                                      (96, 128, 700, 256)])
@pytest.mark.parametrize("layout", ["zt", "rows"])
def test_bpr_kernels_match_autograd(B, S, A, HF, layout):
    if layout == "rows" and HF > 128:
        pytest.skip("the one-launch row-major forward covers HF <= 128")
    o, x = bpr_kernels(B, S, A, HF, layout)
    h, W, bias, neg, tgt = (x[k].double() if x[k].is_floating_point() else x[k] for k in
                            ("h", "W", "bias", "neg", "tgt"))
    zneg = (h @ W[neg].t() + bias[neg]).requires_grad_(True)
    zpos = ((h * W[tgt]).sum(1) + bias[tgt]).detach().requires_grad_(True)
    lrow = -torch.nn.functional.logsigmoid(zpos[:, None] - zneg).mean(1)
    lrow.mean().backward()
    np.testing.assert_allclose(o["Z"].double().numpy(), zneg.detach().numpy(), rtol=0, atol=1e-5)
    np.testing.assert_allclose(o["zpos"].double().numpy(), zpos.detach().numpy(), rtol=0, atol=1e-5)
    np.testing.assert_allclose(o["lrow"].double().numpy(), lrow.detach().numpy(), rtol=0, atol=1e-5)
    np.testing.assert_array_equal(o["ids"].numpy(), x["tgt"].numpy())
    np.testing.assert_allclose(o["dzp"].double().numpy(), zpos.grad.numpy(), rtol=0, atol=1e-7)
    np.testing.assert_allclose(o["gpos"].double().numpy(), (zpos.grad[:, None] * h).numpy(), rtol=0, atol=1e-7)
    np.testing.assert_allclose(o["dhp"].double().numpy(), (zpos.grad[:, None] * W[tgt]).numpy(), rtol=0, atol=1e-7)
    np.testing.assert_allclose(o["dZ"].double().numpy(), zneg.grad.numpy(), rtol=1e-4, atol=1e-9)
    np.testing.assert_allclose(o["dbg"].double().numpy(), zneg.grad.sum(0).numpy(), rtol=1e-4, atol=1e-8)


def test_bpr_invalid_target_gives_nan_row():
    o, _ = bpr_kernels(64, 64, 200, 32, "zt", bad_target=True)
    assert torch.isfinite(o["lrow"][:-1]).all() and torch.isnan(o["lrow"][-1])
    assert int(o["ids"][-1]) == -1 and float(o["dzp"][-1]) == 0.0


@pytest.mark.parametrize("kind,precision,E,N,L,B,S", [("gru4rec", "f32", 32, 3000, 10, 256, 512),
                                                      ("gru4rec", "f32x6", 128, 50000, 50, 1024, 2048),
                                                      ("bidir", "f32", 32, 5000, 12, 200, 256),
                                                      ("bidir", "f32x6", 64, 20000, 20, 512, 1024),
                                                      ("bidir", "f32x6d3", 64, 20000, 20, 512, 1024)])
def test_bpr_trainer_matches_oracle(kind, precision, E, N, L, B, S):
    from oracle.models import OracleSupervised
    from recommenders.data_utils.synthetic import SessionStream
    from recommenders.models.BidirGRU4Rec.model import BidirGRU4Rec_trainer
    from recommenders.models.GRU4Rec.model import GRU4Rec_trainer
    cfg = dict(hidden_dim=E, embedding_dim=E, gru_layers=1, train_pad_embed=True, use_packed_seq=True,
               learning_rate=0.005, item_num=N, state_size=L, action_dim=N, n_negatives=S, neg_seed=11,
               sampled_loss="bpr")
    torch.set_num_threads(8)
    orc = OracleSupervised(kind=kind, **cfg)
    if kind == "bidir":
        tr = BidirGRU4Rec_trainer(device="cuda", dropout=0.0, matmul_precision=precision, **cfg)
    else:
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
