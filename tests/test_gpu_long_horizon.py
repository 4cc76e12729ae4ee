"""Long-horizon training parity (round 3): the short trainer-vs-oracle tests
(tests/test_gpu_supervised.py) run 3-8 Adam steps, where a loose per-element
weight bound (2·lr on <= 0.1 % of elements) is sound but says nothing about
drift over a real run.  Here the HIP GRU4Rec_trainer is trained for several
epochs over a fixed set of batches — as the reference loop does
(recommenders/ikea/training/trainGRU.py:180-224; model step
recommenders/models/GRU4Rec/model.py:129-155) — at every head precision, next
to the CPU oracle (the reference's PyTorch-CPU math) on the same batches.

Two fp32 implementations that sum in different orders drift apart
chaotically over many Adam steps; the native fp32 head ("f32") against the
oracle is that control.  Bars (printed with the measured numbers):
  * every step's loss within max(1e-4, 3 × the control's worst deviation);
  * each parameter's relative Frobenius distance to the oracle's weights
    within 3 × the control's (+ 1e-6);
  * held-out HR@20 / NDCG@20 (reference evaluate math on each model's own
    logits) within 3 × the control's difference + 2 rows.
A fused precision whose dh / dW were not fp32-class would drift
systematically (bias accumulates through Adam's first moment), not
chaotically, and miss the 3× bar.
"""
import numpy as np
import pytest
import torch

from oracle import metrics as om

pytestmark = pytest.mark.gpu

PRECISIONS = ("f32", "f32x6", "f32x6d3")


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


def _heldout(z, a, ks=(20,)):
    idx = om.canonical_topk_fast(z, max(ks))
    h, n = om.hits_from_lists(idx, a, list(ks))
    return h / len(a), n / len(a)


@pytest.mark.parametrize("E,H,N,L,B,NB,EPOCHS", [(64, 64, 4000, 20, 256, 25, 8), (128, 128, 20000, 50, 512, 12, 6)])
def test_multi_epoch_drift_is_fp32_class(E, H, N, L, B, NB, EPOCHS):
    from oracle.models import OracleSupervised
    from recommenders.data_utils.synthetic import SessionStream
    from recommenders.models.GRU4Rec.model import GRU4Rec_trainer
    cfg = dict(hidden_dim=H, embedding_dim=E, gru_layers=1, train_pad_embed=True, use_packed_seq=True,
               learning_rate=0.005, item_num=N, state_size=L, action_dim=N)
    torch.set_num_threads(max(8, min(16, torch.get_num_threads())))
    orc = OracleSupervised(kind="gru4rec", **cfg)
    hips = {p: GRU4Rec_trainer(device="cuda", matmul_precision=p, **cfg) for p in PRECISIONS}
    st = SessionStream(N, L, B * (NB + 2), seed=21)
    batches = [st.batch(i, B) for i in range(NB)]
    held = [st.batch(NB + i, B) for i in range(2)]
    losses = {p: [] for p in ("oracle",) + PRECISIONS}
    for ep in range(EPOCHS):
        for b in batches:
            losses["oracle"].append(orc.step(b[0], b[1], b[4]))
            for p, tr in hips.items():
                losses[p].append(tr.train_step(b[0], b[1], b[4]))
    lo = np.asarray(losses["oracle"])
    dev = {p: float(np.abs(np.asarray(losses[p]) - lo).max()) for p in PRECISIONS}
    sd_o = orc.net.state_dict()
    drift = {p: {k: _rel(v, sd_o[k]) for k, v in hips[p].gru_model.state_dict().items()} for p in PRECISIONS}
    # held-out HR@20 / NDCG@20 of every model on its own logits
    orc.net.eval()
    hr, nd = {}, {}
    for name in ("oracle",) + PRECISIONS:
        H_, N_, n = 0.0, 0.0, 0
        for b in held:
            s, a, ln = b[0], b[1], b[4]
            if name == "oracle":
                with torch.no_grad():
                    z = orc.net(s, ln).double().numpy()
            else:
                hips[name].set_eval()
                z = hips[name].gru_model(s.cuda(), ln).double().cpu().numpy()
                hips[name].set_train()
            h_, n_ = _heldout(z, a.numpy())
            H_ += float(h_[0]) * len(a)
            N_ += float(n_[0]) * len(a)
            n += len(a)
        hr[name], nd[name] = H_ / n, N_ / n
    steps = EPOCHS * NB
    print(f"\n{steps} steps (B {B}, N {N}, H {H}); final loss oracle {lo[-1]:.6f} (first {lo[0]:.6f})")
    for p in PRECISIONS:
        worst = max(drift[p], key=drift[p].get)
        print(f"  {p:8s} max|dloss| {dev[p]:.3g}  worst param drift {worst} {drift[p][worst]:.3g}  "
              f"HR@20 {hr[p]:.5f} (oracle {hr['oracle']:.5f})  NDCG@20 {nd[p]:.5f} (oracle {nd['oracle']:.5f})")
    assert lo[-1] < lo[0] - 0.5            # the run actually learns
    assert hr["oracle"] > 0.02
    ctl = "f32"
    n_rows = 2 * B
    for p in ("f32x6", "f32x6d3"):
        assert dev[p] <= max(1e-4, 3 * dev[ctl]), (p, dev[p], dev[ctl])
        for k in drift[p]:
            assert drift[p][k] <= 3 * drift[ctl][k] + 1e-6, (p, k, drift[p][k], drift[ctl][k])
        assert abs(hr[p] - hr["oracle"]) <= 3 * abs(hr[ctl] - hr["oracle"]) + 2 / n_rows, (p, hr)
        assert abs(nd[p] - nd["oracle"]) <= 3 * abs(nd[ctl] - nd["oracle"]) + 2 / n_rows, (p, nd)
    # the control itself stays fp32-close to the oracle over the whole run
    assert dev[ctl] < 1e-3, dev
    assert max(drift[ctl].values()) < 1e-2, drift[ctl]
