"""Pin the CPU oracle to the reference's own outputs (golden vectors made by
running the reference, tests/golden/make_golden.py) and to the reference's
known-answer tests.  CPU only."""
import json
import os
import random

import numpy as np
import pytest
import torch

from oracle import metrics as om
from oracle.models import OracleSMORL, OracleSQN, OracleSupervised

from conftest import GOLDEN

META = json.load(open(os.path.join(GOLDEN, "meta.json")))


def load(name):
    return dict(np.load(os.path.join(GOLDEN, f"{name}.npz")))


def batches(g):
    n = g["in_s"].shape[0]
    for i in range(n):
        yield (torch.from_numpy(g["in_s"][i]), torch.from_numpy(g["in_a"][i]),
               torch.from_numpy(g["in_r"][i]), torch.from_numpy(g["in_s_next"][i]),
               torch.from_numpy(g["in_len"][i]), torch.from_numpy(g["in_next_len"][i]),
               torch.from_numpy(g["in_is_end"][i]))


def assert_sd(net, g, prefix, atol=0.0):
    sd = net.state_dict()
    for k, v in sd.items():
        ref = g[prefix + k]
        np.testing.assert_allclose(v.numpy(), ref, rtol=0, atol=atol, err_msg=prefix + k)


SUP_CASES = ["gru4rec_packed", "gru4rec_unpacked_fixedpad", "gru4rec_layers2", "bidir_packed",
             "bidir_dropout"]


@pytest.mark.parametrize("name", SUP_CASES)
def test_supervised_oracle_matches_reference(name):
    g = load(name)
    cfg = dict(META["cases"][name]["config"])
    kind = META["cases"][name]["kind"]
    dropout = cfg.pop("dropout", 0.0)
    tr = OracleSupervised(kind=kind, dropout=dropout, **cfg)
    # initial weights: bit-identical (same RNG consumption order)
    assert_sd(tr.net, g, "init.")
    tr.net.eval()
    bs = list(batches(g))
    with torch.no_grad():
        np.testing.assert_allclose(tr.net(bs[0][0], bs[0][4]).numpy(), g["logits0"], rtol=0, atol=1e-6)
    tr.net.train()
    losses = [tr.step(b[0], b[1], b[4]) for b in bs]
    np.testing.assert_allclose(losses, g["losses"], rtol=0, atol=1e-6)
    assert_sd(tr.net, g, "final.", atol=1e-6)
    if name == "gru4rec_layers2":
        # quirk: only layer 0 feeds h[0]; layer-1 weights never move
        for k in ("weight_ih_l1", "weight_hh_l1", "bias_ih_l1", "bias_hh_l1"):
            np.testing.assert_array_equal(g["init.gru." + k], g["final.gru." + k])


def test_sqn_oracle_matches_reference():
    g = load("sqn_packed")
    cfg = META["cases"]["sqn_packed"]["config"]
    tr = OracleSQN(**cfg)
    assert_sd(tr.nets[0], g, "init1.")
    assert_sd(tr.nets[1], g, "init2.")
    sup, q, mains = [], [], []
    for b in batches(g):
        x, y = tr.step(*b)
        sup.append(x)
        q.append(y)
        mains.append(tr.last_main)
    np.testing.assert_array_equal(mains, g["main_idx"])
    assert set(mains) == {0, 1}, "golden case should exercise both double-Q branches"
    np.testing.assert_allclose(sup, g["sup_losses"], rtol=0, atol=1e-6)
    np.testing.assert_allclose(q, g["q_losses"], rtol=0, atol=1e-7)
    assert_sd(tr.nets[0], g, "final1.", atol=1e-6)
    assert_sd(tr.nets[1], g, "final2.", atol=1e-6)


def test_smorl_oracle_matches_composed_reference():
    g = load("smorl_composed")
    cfg = dict(META["cases"]["smorl_composed"]["config"])
    table = torch.from_numpy(g["div_table"])
    unpop = set(int(x) for x in g["unpopular"])
    tr = OracleSMORL(div_embedding=table, unpopular_actions_set=unpop, **cfg)
    assert_sd(tr.nets[0], g, "init1.")
    assert_sd(tr.nets[1], g, "init2.")
    sup, q, rw = [], [], []
    for b in batches(g):
        x, y = tr.step(*b)
        sup.append(x)
        q.append(y)
        rw.append(tr.last_rewards.numpy())
    np.testing.assert_allclose(np.stack(rw), g["rewards"], rtol=0, atol=1e-6)
    np.testing.assert_allclose(sup, g["sup_losses"], rtol=0, atol=1e-6)
    np.testing.assert_allclose(q, g["q_losses"], rtol=0, atol=1e-6)
    assert_sd(tr.nets[0], g, "final1.", atol=1e-6)
    assert_sd(tr.nets[1], g, "final2.", atol=1e-6)


def test_metrics_oracle_matches_reference():
    g = load("metrics")
    preds = torch.from_numpy(g["preds"])
    hits, ndcg = om.hits_for_batch(preds, torch.from_numpy(g["true_idx"]), list(g["ks"]))
    np.testing.assert_array_equal(hits, g["hits"])
    np.testing.assert_allclose(ndcg, g["ndcg"], rtol=0, atol=1e-12)
    unpop = set(int(x) for x in g["unpop"])
    np.testing.assert_array_equal(om.batch_novelty_rewards(preds, unpop, 1, 1), g["nov1"])
    np.testing.assert_array_equal(om.batch_novelty_rewards(preds, unpop, 2, 5), g["nov5"])
    table = torch.from_numpy(g["div_table"])
    s, lens = torch.from_numpy(g["s"]), torch.from_numpy(g["lens"])
    np.testing.assert_allclose(om.batch_diversity_rewards(s, preds, lens, "end", 1, table).numpy(),
                               g["div1"], rtol=0, atol=1e-6)
    np.testing.assert_allclose(om.batch_diversity_rewards(s, preds, lens, "end", 3, table).numpy(),
                               g["div3"], rtol=0, atol=1e-6)


# --- the reference's own known-answer tests, restated -----------------------

def _q3():
    q_acc = torch.tensor([[1., 2, 3, 4, 5], [-1, -2, -3, -4, -5]])
    q_div = torch.tensor([[10., 20, 30, 40, 50], [0.1, 0.2, 0.3, 0.4, 0.5]])
    q_nov = torch.tensor([[100., 200, 300, 400, 500], [11, 21, 31, 41, 51]])
    return torch.stack([q_acc, q_div, q_nov], dim=1)


def test_known_answer_q_helpers():
    # test/test_tensor_operations.py:10-78
    res = om.gather_heads(_q3(), torch.tensor([3, 1]))
    assert torch.equal(res, torch.tensor([[4, 40, 400], [-2, 0.2, 21]]))
    w = torch.tensor([0.1, 0.5, 0.4])
    wl = om.weighted_q_loss(torch.tensor([[4, 40, 400], [-2, 0.2, 21]]), w)
    # reference compares with torch.equal (fails on float rounding); closeness is the real pin
    assert torch.allclose(wl, torch.tensor([180.4, 8.3]))
    q = _q3()[:, :, :3]
    tgt = om.weighted_heads(q, w)
    exp = torch.tensor([[0.1 * 1 + 0.5 * 10 + 100 * 0.4, 2 * 0.1 + 20 * 0.5 + 200 * 0.4,
                         3 * 0.1 + 30 * 0.5 + 300 * 0.4],
                        [0.1 * -1 + 0.5 * 0.10 + 11 * 0.4, -2 * 0.1 + 0.20 * 0.5 + 21 * 0.4,
                         -3 * 0.1 + 0.30 * 0.5 + 31 * 0.4]])
    assert torch.allclose(tgt, exp)
    assert torch.equal(om.max_action(tgt), torch.tensor([2, 2]))


def test_known_answer_novelty():
    # test/test_novelty.py:6-23
    preds = torch.tensor([[100, 50, 0, 0, 0], [100, -10, 10, 0, 0]])
    unpop = {0, 1, 10, 11, 12, 13}
    assert np.array_equal(om.batch_novelty_rewards(preds, unpop, 2), [2, 2])
    assert np.array_equal(om.batch_novelty_rewards(preds, unpop, 2, 2), [2, 1])


def test_known_answer_hr_ndcg():
    # test/test_evaluation.py:155-267 (hand-made logits, k in {1, 2, 10})
    a = torch.tensor([9, 0, 2, 1, 1, 1, 9, 0, 1])
    a_type = torch.tensor([0, 0, 0, 0, 0, 0, 1, 1, 1])
    up = [1., 2, 3, 4, 5, 6, 7, 8, 9, 10]
    preds = torch.tensor([up, up[::-1], [1, 2, 100, 2, 2, 2, 2, 2, 2, 2], up, up[::-1],
                          [1, 1.5, 100, 2, 2, 2, 2, 2, 2, 2], up, up[::-1],
                          [1, 3, 100, 2, 2, 2, 2, 2, 2, 2]])
    ks = [1, 2, 10]
    expect = {0: ([3 / 6, 4 / 6, 1], [3 / 6, (3 + 1 / np.log2(3)) / 6,
                                       (3 + 1 / np.log2(3) + 2 / np.log2(10)) / 6]),
              1: ([2 / 3, 1, 1], [2 / 3, (2 + 1 / np.log2(3)) / 3, (2 + 1 / np.log2(3)) / 3])}
    for t in (0, 1):
        m = a_type == t
        h, n = om.hits_for_batch(preds[m], a[m], ks)
        assert np.allclose(h / m.sum().item(), expect[t][0])
        assert np.allclose(n / m.sum().item(), expect[t][1])


def test_known_answer_last_action():
    # test/test_diversity.py:5-19
    back = torch.tensor([[1, 2, 3, 3, 0, 0], [12, 13, 2, 0, 0, 0]])
    front = torch.tensor([[0, 0, 1, 2, 3, 3], [0, 0, 0, 12, 13, 2]])
    assert torch.equal(om.last_action(back, "end", torch.tensor([4, 3])), torch.tensor([3, 2]))
    assert torch.equal(om.last_action(front, "beg"), torch.tensor([3, 2]))
