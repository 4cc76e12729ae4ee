"""Model-level parity of the evaluation metric (BASELINE metric "HR@20/NDCG@20
parity"; north_star "bit-exact for top-k index lists").

1. The HIP GRU4Rec_trainer (native f32, fused split-bf16 f32x6 / f32x6d3 heads) and
   the CPU oracle (the reference's PyTorch-CPU math, pinned to the reference's
   golden vectors) are trained side by side on the same synthetic stream at
   C2 widths (H 128, L 50, N 50k, B 1024).  Both trained models are then
   evaluated on the same held-out batches (reference evaluate(),
   recommenders/evaluate/eval_protocol.py:123-263, get_hits_for_batch :62-100):
   * top-20 index lists under the canonical (value desc, index asc) order are
     identical, except where two items' oracle logits lie closer than the
     measured logit error bound (flips counted and bounded);
   * HR@20 / NDCG@20 differ by at most the rows whose target rank differs.
2. Full C2 size (A = 1,000,000, B = 4096): one training step per head
   precision; lse, per-row CE, the loss and dh are checked against a chunked
   fp64 restatement on the same h / W / b; device top-20 at A = 1M against the
   canonical top-20 of the same device logits.
"""
import numpy as np
import pytest
import torch

from oracle import metrics as om

pytestmark = pytest.mark.gpu

E = H = 128
N, L, B = 50000, 50, 1024
LR = 0.01
STEPS = 8   # enough for HR@20 > 0 on the held-out batches (popularity is learnt first)
K = 20


@pytest.fixture(scope="module")
def trained():
    from oracle.models import OracleSupervised
    from recommenders.data_utils.synthetic import SessionStream, unpopular_items
    from recommenders.models.GRU4Rec.model import GRU4Rec_trainer
    cfg = dict(hidden_dim=H, embedding_dim=E, gru_layers=1, train_pad_embed=True, use_packed_seq=True,
               learning_rate=LR, item_num=N, state_size=L, action_dim=N)
    torch.set_num_threads(8)
    orc = OracleSupervised(kind="gru4rec", **cfg)
    hips = {p: GRU4Rec_trainer(device="cuda", matmul_precision=p, **cfg) for p in ("f32", "f32x6", "f32x6d3")}
    # held-out batches come from the same stream (same item popularity), after the training ones
    st = SessionStream(N, L, B * (STEPS + 2), seed=9)
    for i in range(STEPS):
        s, a, r, sn, ln, nln, e = st.batch(i, B)
        lo = orc.step(s, a, ln)
        for p, tr in hips.items():
            lg = tr.train_step(s, a, ln)
            assert abs(lo - lg) < 1e-4, (p, i, lo, lg)
    loader = [(b[0], b[1], b[4]) for b in (st.batch(STEPS + i, B) for i in range(2))]
    return orc, hips, loader, unpopular_items(st.item_counts())


@pytest.mark.parametrize("precision", ["f32", "f32x6", "f32x6d3"])
def test_trained_model_top20_and_hr_ndcg_match_oracle(trained, precision):
    from recommenders.evaluate.eval_protocol import evaluate
    from recommenders.hip.evalpath import eval_batch
    orc, hips, loader, unpop = trained
    tr = hips[precision]
    tr.set_eval()
    orc.net.eval()
    ks = [10, 20]
    loss, hr, ndcg, *_ = evaluate(loader, tr.gru_model, "cuda", tr.cross_entropy_loss, "end", None, unpop,
                                  topk_hr_ndcg=ks, topk_to_consider_cov=[1])
    H_o, N_o = np.zeros(2), np.zeros(2)
    flips = rank_moves = n = 0
    worst_gap = delta_max = 0.0
    loss_o = 0.0
    for s, a, ln in loader:
        with torch.no_grad():
            z_o = orc.net(s, ln).double().numpy()
        z_h = tr.gru_model(s.cuda(), ln).double().cpu().numpy()
        delta = float(np.abs(z_h - z_o).max())          # measured logit error bound
        delta_max = max(delta_max, delta)
        idx_o = om.canonical_topk_fast(z_o, K)
        idx_h = eval_batch(tr.gru_model, s, ln, a, K=K, ks=ks, want_loss=False).idx.cpu().numpy()
        # the device list is the canonical order of the device logits
        np.testing.assert_array_equal(idx_h, om.canonical_topk_fast(z_h, K))
        f, g = om.topk_flip_report(z_o, idx_h, idx_o, 2 * delta)
        flips += f
        worst_gap = max(worst_gap, g)
        rank_moves += int((om.target_ranks(idx_h, a) != om.target_ranks(idx_o, a)).sum())
        h_, n_ = om.hits_from_lists(idx_o, a, ks)
        H_o += h_
        N_o += n_
        loss_o += float(torch.nn.functional.cross_entropy(torch.from_numpy(z_o), a))
        n += len(a)
    print(f"{precision}: logit bound {delta_max:.3g}, rows with a flipped top-20 {flips}/{n} "
          f"(largest flipped gap {worst_gap:.3g}), target-rank moves {rank_moves}; "
          f"HR@20 {hr[1]:.6f} vs {H_o[1] / n:.6f}, NDCG@20 {ndcg[1]:.6f} vs {N_o[1] / n:.6f}")
    assert delta_max < 1e-4
    assert H_o[1] > 0                                   # a non-trivial comparison
    assert flips <= max(2, n // 100)
    np.testing.assert_allclose(hr, H_o / n, rtol=0, atol=rank_moves / n + 1e-12)
    np.testing.assert_allclose(ndcg, N_o / n, rtol=0, atol=rank_moves / n + 1e-12)
    assert abs(float(loss) - loss_o / len(loader)) < 1e-4
    tr.set_train()


# ------------------------------------------------------------- full C2 size --
def _fp64_head(h, W, b, tgt, rows, chunk=131072):
    """lse, per-row CE and dh = ((softmax − onehot) W)/B in fp64, item-chunked."""
    h64, Bn = h[rows].double(), h.shape[0]
    A = W.shape[0]
    m = torch.full((len(rows),), -float("inf"), dtype=torch.float64, device=h.device)
    s = torch.zeros(len(rows), dtype=torch.float64, device=h.device)
    for j in range(0, A, chunk):
        z = h64 @ W[j:j + chunk].double().t() + b[j:j + chunk].double()
        mn = torch.maximum(m, z.max(1).values)
        s = s * torch.exp(m - mn) + torch.exp(z - mn[:, None]).sum(1)
        m = mn
    lse = m + torch.log(s)
    dh = torch.zeros(len(rows), h.shape[1], dtype=torch.float64, device=h.device)
    for j in range(0, A, chunk):
        z = h64 @ W[j:j + chunk].double().t() + b[j:j + chunk].double()
        dh += torch.exp(z - lse[:, None]) @ W[j:j + chunk].double()
    t = tgt[rows]
    zt = (h64 * W[t].double()).sum(1) + b[t].double()
    dh = (dh - W[t].double()) / Bn
    return lse, lse - zt, dh


def _cpu_fp32_dh(h, W, b, tgt, rows, B):
    """The reference's own CPU fp32 path on the same rows: nn.Linear logits,
    CrossEntropyLoss(mean over the B-row batch) and autograd
    (GRU4Rec/model.py:80, 121, 146-150) -> dh of those rows."""
    torch.set_num_threads(max(8, min(16, torch.get_num_threads())))
    hr = h[rows].cpu().float().requires_grad_(True)
    z = hr @ W.cpu().float().t() + b.cpu().float()
    loss = torch.nn.functional.cross_entropy(z, tgt[rows].cpu(), reduction="sum") / B
    loss.backward()
    return hr.grad.double().to(h.device)


@pytest.mark.parametrize("precision", ["f32x6", "f32", "f32x6d3"])
def test_full_c2_step_lse_ce_dh_against_fp64(precision):
    from recommenders.data_utils.synthetic import SessionStream
    from recommenders.models.GRU4Rec.model import GRU4Rec_trainer
    NF, BF = 1_000_000, 4096
    tr = GRU4Rec_trainer(hidden_dim=128, embedding_dim=128, gru_layers=1, train_pad_embed=True,
                         use_packed_seq=True, learning_rate=0.01, item_num=NF, state_size=50, action_dim=NF,
                         device="cuda", matmul_precision=precision)
    head = tr.gru_model.heads["output"]
    s, a, r, sn, ln, nln, e = SessionStream(NF, 50, BF, seed=2).batch(0, BF)
    W0, b0 = head.W.p.clone(), head.b.p.clone()
    loss = tr.train_step(s, a, ln)
    h = next(v for k, v in tr.gru_model.trunk._ws.items() if k[0] == "main").h
    w = head.fws("main", BF) if head.flash_terms(BF) else head.ws("main", BF, True)
    assert bool(head.flash_terms(BF)) == (precision != "f32")
    dh = tr.gru_model.dh_buffer(BF)
    rows = torch.arange(0, BF, 16, device="cuda")          # 256-row subset
    tgt = a.cuda()
    lse64, ce64, dh64 = _fp64_head(h, W0, b0, tgt, rows)
    e_lse = float((w.lse[rows].double() - lse64).abs().max())
    e_ce = float((w.loss_row[rows].double() - ce64).abs().max())
    e_dh = float((dh[rows].double() - dh64).abs().max())
    scale = float(dh64.abs().max())
    # the reference CPU fp32 path's own dh error on the same rows (the bar of
    # test_flash_error_is_fp32_class, here at the benched width A = 1M)
    e_cpu = float((_cpu_fp32_dh(h, W0, b0, tgt, rows, BF) - dh64).abs().max())
    floor = 8 * 2.0 ** -24 * scale
    print(f"{precision}: |lse err| {e_lse:.3g}, |CE err| {e_ce:.3g}, |dh err| {e_dh:.3g} "
          f"(reference CPU fp32 {e_cpu:.3g}, |dh| max {scale:.3g})")
    assert e_lse < 1e-4 and e_ce < 1e-4
    # split-bf16 precisions (the bench / trainer default f32x6d3 included):
    # within 2x of the reference CPU fp32 path; the native fp32-MFMA side path
    # ("f32": dh = dZ·W summed over 1M items in split-K slabs) within 4x
    assert e_dh <= max((4 if precision == "f32" else 2) * e_cpu, floor), (precision, e_dh, e_cpu)
    assert abs(loss - float(w.loss_row.double().mean())) < 1e-5
    assert np.isfinite(loss)


def test_topk_at_full_c2_width():
    """rg_topk over A = 1M items (the C2 head width): bit-exact canonical lists."""
    from recommenders.data_utils.synthetic import SessionStream
    from recommenders.hip.evalpath import head_for, topk_device
    from recommenders.models.GRU4Rec.model import GRU4Rec
    NF, BE = 1_000_000, 256
    m = GRU4Rec(hidden_size=128, embedding_dim=128, item_num=NF, state_size=50, action_dim=NF, device="cuda")
    m.eval()
    s, a, r, sn, ln, nln, e = SessionStream(NF, 50, BE, seed=8).batch(0, BE)
    h = m.hidden(s.cuda(), ln, slot="eval")
    head = head_for(m, 0)
    ws, z = head.logits_T(h, slot="eval")
    idx, vals, err = topk_device(head, ws, BE, K)
    assert int(err.item()) == 0
    zc = z.cpu().numpy()
    ref = om.canonical_topk_fast(zc, K)
    np.testing.assert_array_equal(idx.cpu().numpy(), ref)
    np.testing.assert_array_equal(vals.cpu().numpy(), np.take_along_axis(zc, ref, 1))
