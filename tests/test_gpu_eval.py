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


@pytest.mark.parametrize("screen", [False, True])
@pytest.mark.parametrize("N,B,H,K", [(3000, 100, 32, 20), (70000, 256, 64, 10), (20011, 96, 128, 32),
                                     (5003, 65, 256, 1)])
def test_score_topk_equals_native_logits_topk(N, B, H, K, screen):
    """Evaluation scoring without a (B, A) buffer (SoftmaxHead.score_topk:
    rg_flash_score + rg_flash_lse + rg_flash_topk) against the native head's
    stored logits of the same h: the canonical top-K index lists AND values
    bitwise equal (the re-scoring repeats the native MFMA's fmaf chain), the
    per-row CE within fp32 rounding of rg_lse_combine's; ragged B.  screen
    (update_train_metrics, no targets): the chunk maxima from the 3-product
    screening pass, candidates within its error bound — the same lists."""
    from recommenders.data_utils.synthetic import SessionStream
    from recommenders.hip.evalpath import head_for
    from recommenders.models.GRU4Rec.model import GRU4Rec
    torch.manual_seed(5)
    m = GRU4Rec(hidden_size=H, embedding_dim=H, item_num=N, state_size=8, action_dim=N, device="cuda")
    m.eval()
    s, a, r, sn, ln, nln, e = SessionStream(N, 8, B, seed=11).batch(0, B)
    h = m.hidden(s.cuda(), ln, slot="eval")
    head = head_for(m, 0)
    idx, vals, loss_row = head.score_topk(h, K, None if screen else a.cuda(), screen=screen)
    ws, z = head.logits_T(h)
    zc = z.cpu().numpy()
    ref = om.canonical_topk(zc, K)
    assert int(head.top_scanned.item()) == 0
    np.testing.assert_array_equal(idx.cpu().numpy(), ref)
    np.testing.assert_array_equal(vals.cpu().numpy(), np.take_along_axis(zc, ref, 1))
    if not screen:
        ce = torch.nn.functional.cross_entropy(torch.from_numpy(zc).double(), a, reduction="none").numpy()
        np.testing.assert_allclose(loss_row.cpu().double().numpy(), ce, rtol=0, atol=2e-5)


def test_score_topk_row_chunks(monkeypatch):
    """Row-chunked scoring (chunk maxima capped, several chunks plus a ragged
    tail) gives the same lists and values as one chunk; the CE rows agree to
    fp32 rounding (the lse merges a different number of item splits)."""
    from recommenders.data_utils.synthetic import SessionStream
    from recommenders.hip import engine
    from recommenders.hip.evalpath import head_for
    N, B, K = 40000, 300, 20
    m = _model(N=N)
    m.eval()
    s, a, r, sn, ln, nln, e = SessionStream(N, 8, B, seed=12).batch(0, B)
    h = m.hidden(s.cuda(), ln, slot="eval")
    head = head_for(m, 0)
    i1, v1, l1 = (x.clone() for x in head.score_topk(h, K, a.cuda()))
    head.release_eval()
    monkeypatch.setattr(engine, "EVAL_CMAX_BYTES", 64 * 4 * ((N + 31) // 32))   # 64 rows per chunk
    i2, v2, l2 = head.score_topk(h, K, a.cuda(), slot="eval2")
    assert head._sws_eval["eval2"].R == 64
    np.testing.assert_array_equal(i1.cpu().numpy(), i2.cpu().numpy())
    np.testing.assert_array_equal(v1.cpu().numpy(), v2.cpu().numpy())
    np.testing.assert_allclose(l1.cpu().numpy(), l2.cpu().numpy(), rtol=4e-7, atol=0)


@pytest.mark.parametrize("screen", [False, True])
def test_score_topk_ragged_rows_at_catalogue_scale(screen):
    """A ragged final batch at A = 1M (B = 1000 rows in a 1024-row chunk): the
    chunk's zero padding rows (logits = the biases, a dense band of near-ties)
    are never selected or scanned — the top-k runs on the 1000 real rows only
    — and every row equals the native head's canonical top-K bitwise."""
    from recommenders.hip import engine
    N, B, HF, K = 1_000_000, 1000, 64, 20
    hd = engine.SoftmaxHead("x", N, HF, "cuda")
    g = torch.Generator().manual_seed(21)
    h = torch.tanh(torch.randn(B, HF, generator=g)).cuda()
    tgt = torch.randint(0, N, (B,), generator=g).cuda()
    idx, vals, _ = hd.score_topk(h, K, None if screen else tgt, screen=screen)
    assert hd._sws_eval["eval"].R == 1024
    torch.cuda.synchronize()
    assert int(hd.top_scanned.item()) == 0
    ws, z = hd.logits_T(h)
    rows = torch.arange(0, B, 7)
    zc = z[rows.cuda()].cpu().numpy()
    ref = om.canonical_topk_fast(zc, K)
    np.testing.assert_array_equal(idx[rows.cuda()].cpu().numpy(), ref)
    np.testing.assert_array_equal(vals[rows.cuda()].cpu().numpy(), np.take_along_axis(zc, ref, 1))


def test_eval_batch_tie_flood_is_exact():
    """eval_batch on a head whose logits hold a flood of exact ties (every
    item's weight row and bias equal): every row's candidate band overflows the
    cap, the rows are scanned whole, and the top-K ids are the lowest indices
    (canonical order) — never uninitialised ids; novelty reads valid ids."""
    from recommenders.hip.evalpath import eval_batch, head_for
    from recommenders.hip.qlearn import unpopular_bitmap
    from recommenders.data_utils.synthetic import SessionStream
    N, L, B, K = 5000, 8, 64, 20
    m = _model(N=N, L=L)
    head = head_for(m, 0)
    with torch.no_grad():
        head.W.p.copy_(head.W.p[0:1].expand_as(head.W.p))
        head.b.p.fill_(0.25)
    s, a, r, sn, ln, nln, e = SessionStream(N, L, B, seed=3).batch(0, B)
    for screen in (True, False):
        out = eval_batch(m, s, ln, a, K=K, ks=(20,), bitmap=unpopular_bitmap(set(range(0, N, 2)), N, "cuda"),
                         k_nov=K, want_loss=not screen, screen=screen)
        torch.cuda.synchronize()
        assert (out.idx.cpu() == torch.arange(K, dtype=torch.int32)).all()
        np.testing.assert_allclose(out.nov.cpu().numpy(), 0.5)
    assert int(head.top_scanned.item()) >= B


def test_eval_allocates_no_logits():
    """evaluate()'s per-batch scoring leaves no (B, A) buffer behind and
    allocates far less than one (C2-like width, A = 200k)."""
    from recommenders.data_utils.synthetic import SessionStream, unpopular_items
    from recommenders.evaluate.eval_protocol import evaluate
    from recommenders.models.GRU4Rec.model import GRU4Rec
    N, L, B = 200_000, 20, 1024
    m = GRU4Rec(hidden_size=128, embedding_dim=128, item_num=N, state_size=L, action_dim=N, device="cuda")
    st = SessionStream(N, L, 2 * B, seed=13)
    loader = [(b[0], b[1], b[4]) for b in (st.batch(i, B) for i in range(2))]
    torch.cuda.synchronize()
    base = torch.cuda.memory_allocated()
    torch.cuda.reset_peak_memory_stats()
    evaluate(loader, m, "cuda", None, "end", None, unpopular_items(st.item_counts()), topk_hr_ndcg=[20])
    torch.cuda.synchronize()
    zt_bytes = 4 * B * N
    assert torch.cuda.max_memory_allocated() - base < zt_bytes // 2
    assert not any(k[0] == "eval" for k in m.heads["output"]._ws)


def test_evaluate_unmapped_token_raises():
    """A predicted id with no input-vocabulary token: the reference's stoi
    raises KeyError inside evaluate(); here RemapError (a KeyError), and the
    diversity kernel never reads the table at row -1."""
    from recommenders.data_utils.synthetic import SessionStream, unpopular_items
    from recommenders.evaluate.eval_protocol import evaluate
    from recommenders.hip.remap import RemapError
    from recommenders.utils.tokenizer import Tokenizer
    N, L, B = 3000, 8, 64
    m = _model(N=N, L=L)
    st = SessionStream(N, L, B, seed=14)
    b = st.batch(0, B)
    loader = [(b[0], b[1], b[4])]
    names = [f"item{j}" for j in range(N)]
    tout = Tokenizer(names)
    tin = Tokenizer(names[: N // 2])        # no <unk>: half of the output ids cannot be mapped
    table = torch.randn(N // 2 + 2, 8)
    with pytest.raises(RemapError):
        evaluate(loader, m, "cuda", None, "end", torch.nn.Embedding.from_pretrained(table), unpopular_items(
            st.item_counts()), topk_hr_ndcg=[20], topk_to_consider_div=20, input_tokenizer=tin, output_tokenizer=tout)
    torch.cuda.synchronize()     # the device is healthy afterwards
