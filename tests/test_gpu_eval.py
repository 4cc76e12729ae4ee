"""GPU parity of the evaluation path: device top-k vs the
canonical CPU top-k of the same logits (bit-exact index lists), HR/NDCG sums
vs the reference semantics (oracle.metrics.hits_for_batch), and the
evaluate() 7-tuple vs an oracle evaluation on host-copied logits."""
import numpy as np
import pytest
import torch

from oracle import metrics as om

pytestmark = pytest.mark.gpu


def _model(N=3000, H=32, L=8):
    from recommenders.models.GRU4Rec.model import GRU4Rec
    torch.manual_seed(3)
    return GRU4Rec(hidden_size=H, embedding_dim=H, item_num=N, state_size=L, action_dim=N, device="cuda")


@pytest.mark.parametrize("N,B,K", [(3000, 64, 20), (70000, 200, 20), (1000, 33, 64)])
def test_topk_matches_canonical_cpu_topk(N, B, K):
    from recommenders.data_utils.synthetic import SessionStream
    from recommenders.hip.evalpath import head_for, topk_device
    m = _model(N=N)
    m.eval()
    st = SessionStream(N, 8, B, seed=4)
    s, a, r, sn, ln, nln, e = st.batch(0, B)
    h = m.hidden(s.cuda(), ln, slot="eval")
    head = head_for(m, 0)
    ws, z = head.logits_T(h, slot="eval")
    idx, vals, err = topk_device(head, ws, B, K)
    zc = z.cpu().numpy()
    ref = om.canonical_topk(zc, K)
    assert int(err.item()) == 0
    np.testing.assert_array_equal(idx.cpu().numpy(), ref)
    np.testing.assert_array_equal(vals.cpu().numpy(), np.take_along_axis(zc, ref, 1))


def test_topk_with_planted_ties():
    """Exact ties (the reference's CPU topk order is implementation-defined):
    the device list is the (value desc, index asc) canonical order."""
    from recommenders.hip import call, stream_ptr
    B, A, K = 16, 5000, 20
    g = torch.Generator().manual_seed(1)
    Z = torch.randn(B, A, generator=g)
    Z[:, 100:140] = 7.0   # 40 exact ties at the top
    ZT = Z.t().contiguous().cuda()
    from recommenders.hip import load_library
    pb = load_library().rg_partial_block()
    nJ = (A + pb - 1) // pb
    pmax = torch.stack([Z[:, j * pb:(j + 1) * pb].max(1).values for j in range(nJ)]).contiguous().cuda()
    idx = torch.empty(B, K, dtype=torch.int32, device="cuda")
    call("rg_topk", ZT.data_ptr(), B, pmax.data_ptr(), B, A, K, idx.data_ptr(), None, None, stream_ptr())
    np.testing.assert_array_equal(idx.cpu().numpy(), np.tile(np.arange(100, 120), (B, 1)))


def test_evaluate_matches_oracle():
    from recommenders.data_utils.synthetic import SessionStream, unpopular_items
    from recommenders.evaluate.eval_protocol import evaluate
    N, L, B = 3000, 8, 100
    m = _model(N=N, L=L)
    st = SessionStream(N, L, 3 * B, seed=6)
    loader = [(b[0], b[1], b[4]) for b in (st.batch(i, B) for i in range(3))]
    g = torch.Generator().manual_seed(2)
    table = torch.randn(N + 1, 16, generator=g) * 0.01
    emb = torch.nn.Embedding.from_pretrained(table, freeze=True)
    unpop = unpopular_items(st.item_counts())
    ks = [1, 10, 20]
    loss, hr, ndcg, cov, div, nov, reps = evaluate(loader, m, "cuda", None, "end", emb, unpop, topk_hr_ndcg=ks,
                                                    topk_to_consider_div=3, topk_to_consider_nov=2,
                                                    topk_to_consider_cov=[1, 5])
    # oracle on host-copied logits of the same model
    H = np.zeros(3)
    Nd = np.zeros(3)
    L_, D_, N_, R_ = 0.0, 0.0, 0.0, np.zeros(3)
    covs = {1: set(), 5: set()}
    for s, a, ln in loader:
        z = m(s.cuda(), ln).float().cpu()
        h_, n_ = om.hits_for_batch(z, a, ks)
        H += h_
        Nd += n_
        L_ += float(torch.nn.functional.cross_entropy(z.double(), a))
        D_ += float(om.batch_diversity_rewards(s, z, ln, "end", 3, table).double().sum())
        N_ += om.batch_novelty_rewards(z, unpop, 1, 2).sum()
        top = torch.topk(z, 20).indices.numpy()
        for k in (1, 5):
            covs[k] |= set(top[:, :k].ravel().tolist())
        for i, k in enumerate(ks):
            R_[i] += (s.numpy()[:, :, None] == top[:, None, :k]).sum()
    n = 3 * B
    np.testing.assert_allclose(hr, H / n, atol=0)
    np.testing.assert_allclose(ndcg, Nd / n, atol=1e-12)
    assert abs(float(loss) - L_ / 3) < 1e-5
    assert abs(float(div) - D_ / n) < 1e-6
    assert abs(nov - N_ / n) < 1e-12
    np.testing.assert_allclose(reps, R_ / n, atol=0)
    for k in (1, 5):
        assert cov[k][1] == len(covs[k]) / N
