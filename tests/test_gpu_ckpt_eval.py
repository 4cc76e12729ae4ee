"""§8f rows on the GPU: checkpoint / resume compatibility (SaveBestModel dict,
torch.optim.Adam-format optimizer state, reference_save_best_model.py:18-41,
GRU4Rec/train.py:309-311), ``update_train_metrics`` against the reference's
per-batch metric math (eval_protocol.py:266-359) and the device tokenizer
remap (diversity.py:55-60, repetitiveness.py:42-47)."""
import numpy as np
import pytest
import torch

from oracle import metrics as om

pytestmark = pytest.mark.gpu

N, L, B, H = 600, 8, 64, 32


def _cfg(**kw):
    c = dict(hidden_dim=H, embedding_dim=H, gru_layers=1, train_pad_embed=True, use_packed_seq=True,
             learning_rate=0.01, item_num=N, state_size=L, action_dim=N)
    c.update(kw)
    return c


def _stream(n_batches):
    from recommenders.data_utils.synthetic import SessionStream
    return SessionStream(N, L, B * n_batches, seed=41)


def test_checkpoint_resume_is_bit_exact(tmp_path):
    """Save after 3 steps (SaveBestModel + optimizer.state_dict), load into a
    fresh trainer built with another seed, continue 2 steps: identical to an
    uninterrupted 5-step run, loss for loss and bit for bit."""
    from recommenders.models.GRU4Rec.model import GRU4Rec_trainer
    from recommenders.utils.save_best_model import SaveBestModel
    st = _stream(5)
    ref = GRU4Rec_trainer(device="cuda", **_cfg())
    run = GRU4Rec_trainer(device="cuda", **_cfg())
    l_ref = [ref.train_step(*(lambda b: (b[0], b[1], b[4]))(st.batch(i, B))) for i in range(5)]
    for i in range(3):
        b = st.batch(i, B)
        run.train_step(b[0], b[1], b[4])
    saver = SaveBestModel(str(tmp_path), max=True, metric_name="Val_NDCG@10")
    saver(0.5, 3, run.gru_model)
    saver(0.25, 4, run.gru_model)            # not better: the file keeps epoch 3
    torch.save(run.optimizer.state_dict(), tmp_path / "opt.pt")
    ck = torch.load(tmp_path / "best_model.pt", weights_only=True)
    assert set(ck) == {"epoch", "model_idx", "hidden_dim", "item_num", "action_dim", "state_size", "embedding_dim",
                       "model_state_dict"}
    assert ck["epoch"] == 3 and ck["model_idx"] == 1 and ck["item_num"] == N and ck["hidden_dim"] == H
    res = GRU4Rec_trainer(device="cuda", torch_rand_seed=5, **_cfg())
    res.gru_model.load_state_dict(ck["model_state_dict"])
    res.optimizer.load_state_dict(torch.load(tmp_path / "opt.pt", weights_only=True))
    assert res.clock.t == 3
    l_res = []
    for i in range(3, 5):
        b = st.batch(i, B)
        l_res.append(res.train_step(b[0], b[1], b[4]))
    assert l_res == l_ref[3:]
    for (k, v), (k2, v2) in zip(ref.gru_model.state_dict().items(), res.gru_model.state_dict().items()):
        assert k == k2 and torch.equal(v, v2), k


def test_reference_adam_resumes_from_hip_state():
    """The HIP trainer's model and optimizer state load into the reference's
    nn.Module + torch.optim.Adam (the oracle), and both continue the same 2
    steps within the training tolerances — the state is the reference's
    format, not a private one."""
    from oracle.models import OracleSupervised
    from recommenders.models.GRU4Rec.model import GRU4Rec_trainer
    st = _stream(5)
    tr = GRU4Rec_trainer(device="cuda", **_cfg())
    for i in range(3):
        b = st.batch(i, B)
        tr.train_step(b[0], b[1], b[4])
    orc = OracleSupervised(kind="gru4rec", **_cfg())
    orc.net.load_state_dict({k: v.cpu() for k, v in tr.gru_model.state_dict().items()})
    sd = tr.optimizer.state_dict()
    cpu_sd = {"state": {i: {k: (v.cpu() if torch.is_tensor(v) else v) for k, v in s.items()}
                        for i, s in sd["state"].items()}, "param_groups": sd["param_groups"]}
    orc.opt.load_state_dict(cpu_sd)
    for i in range(3, 5):
        b = st.batch(i, B)
        lo = orc.step(b[0], b[1], b[4])
        lg = tr.train_step(b[0], b[1], b[4])
        assert abs(lo - lg) < 1e-4, (i, lo, lg)
    sd_o = orc.net.state_dict()
    for k, v in tr.gru_model.state_dict().items():
        assert float((v.cpu() - sd_o[k]).abs().max()) < 1e-4, k
    # and back: the reference optimizer's state loads into a HIP trainer
    tr2 = GRU4Rec_trainer(device="cuda", **_cfg())
    tr2.optimizer.load_state_dict(orc.opt.state_dict())
    assert tr2.clock.t == 5


def test_sqn_optimizers_round_trip():
    from recommenders.models.SQN.sqn_gru import SQN_trainer
    st = _stream(3)
    cfg = _cfg(gamma=0.5)
    a = SQN_trainer(device="cuda", **cfg)
    for i in range(3):
        a.train_step(*st.batch(i, B))
    sd1, sd2 = a.optimizer_1.state_dict(), a.optimizer_2.state_dict()
    b = SQN_trainer(device="cuda", torch_rand_seed=3, **cfg)
    b.optimizer_1.load_state_dict(sd1)
    b.optimizer_2.load_state_dict(sd2)
    assert (b.clock_1.t, b.clock_2.t) == (a.clock_1.t, a.clock_2.t)
    for x, y in zip(b.optimizer_1.state_dict()["state"].values(), sd1["state"].values()):
        assert torch.equal(x["exp_avg"], y["exp_avg"]) and torch.equal(x["exp_avg_sq"], y["exp_avg_sq"])


class _Tok:
    """Minimal stoi / itos pair (the reference Tokenizer's interface)."""

    def __init__(self, vocab):
        self.itos_ = list(vocab)
        self.stoi_ = {t: i for i, t in enumerate(self.itos_)}

    def stoi(self, s):
        return self.stoi_[s]

    def itos(self, i):
        return self.itos_[i]

    def __len__(self):
        return len(self.itos_)


@pytest.mark.parametrize("tokenized", [False, True])
def test_update_train_metrics_matches_reference_math(tokenized):
    """Per-batch HR/NDCG, coverage sets, diversity / novelty sums and
    repetitions of update_train_metrics against the reference's formulas on
    the same logits (canonical top-k order); with tokenizers the predicted
    ids go through stoi(itos(.)) for diversity and repetitions only."""
    from recommenders.evaluate.eval_protocol import update_train_metrics
    from recommenders.models.GRU4Rec.model import GRU4Rec_trainer
    tr = GRU4Rec_trainer(device="cuda", **_cfg())
    st = _stream(3)
    for i in range(2):
        b = st.batch(i, B)
        tr.train_step(b[0], b[1], b[4])
    s, a, r, sn, ln, nln, e = st.batch(2, B)
    g = torch.Generator().manual_seed(3)
    table = torch.randn(N + 1, 16, generator=g)
    unpop = set(range(0, N, 4))
    ks, cov = [1, 5, 10], [1, 5]
    tin = tout = None
    if tokenized:   # output vocabulary = a permutation of the input one's item strings
        names = [f"item{j}" for j in range(N)]
        perm = np.random.default_rng(0).permutation(N)
        tin = _Tok(names + ["<pad>"])
        tout = _Tok([names[j] for j in perm])
    covd = {k: set() for k in cov}
    hits, ndcg, covd, div, nov, reps = update_train_metrics(
        s, a, ln, tr.gru_model, "cuda", "end", torch.nn.Embedding.from_pretrained(table), unpop, covd,
        topk_hr_ndcg=ks, topk_to_consider_div=3, topk_to_consider_nov=2, topk_to_consider_cov=cov,
        novelty_rew_signal=1.0, input_tokenizer=tin, output_tokenizer=tout)
    tr.set_eval()
    z = tr.gru_model(s.cuda(), ln).double().cpu()
    idx = torch.from_numpy(om.canonical_topk_fast(z.numpy(), 10))
    # reference formulas on the canonical lists
    h_ref, n_ref = om.hits_from_lists(idx.numpy(), a.numpy(), ks)
    np.testing.assert_allclose(hits, h_ref)
    np.testing.assert_allclose(ndcg, n_ref, rtol=1e-12)
    for k in cov:
        assert covd[k] == set(idx[:, :k].ravel().tolist())
    idx_in = idx
    if tokenized:
        idx_in = torch.tensor([[tin.stoi(tout.itos(int(x))) for x in row] for row in idx.tolist()])
    last = om.last_action(s, "end", ln)
    sim = torch.nn.functional.cosine_similarity(table[last].unsqueeze(1).double(), table[idx_in[:, :3]].double(),
                                                dim=2, eps=1e-6)
    assert abs(float(div) - float((1 - sim.mean(1)).sum())) < 1e-4
    flags = np.isin(idx[:, :2].numpy(), np.array(sorted(unpop)))
    assert abs(nov - float(flags.mean(1).sum())) < 1e-9
    rep_ref = [float((s.numpy()[:, :, None] == idx_in[:, None, :k].numpy()).sum()) for k in ks]
    np.testing.assert_allclose(reps, rep_ref)
