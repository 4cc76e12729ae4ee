"""Golden-vector generator — runs THE REFERENCE ITSELF (build container only).

Usage (from the repo root, where /root/reference exists):

    PYTHONPATH=/root/reference PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

It imports the reference trainers / helpers read-only, feeds them small
deterministic synthetic batches and records inputs, initial weights, per-step
losses and post-step weights as ``tests/golden/*.npz`` (+ ``meta.json``).
The fixtures are data (inputs and expected outputs) only; nothing of the
reference's source travels.  The GPU box never runs this script.

SMORL: the shipped ``SMORL_trainer.train_step`` raises (2 rewards vs 3 heads,
``smorl_gru.py:311``), so the SMORL case drives the reference's own
``SMORL_GRU_Net`` + helper functions in the sequence of
``smorl_gru.py:247-332`` with the novelty reward stacked third
(SURVEY.md §8c "SMORL oracle").
"""
from __future__ import annotations

import importlib.util
import json
import os
import random
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))

# Load the build's synthetic stream by file path (the name ``recommenders``
# resolves to the reference package in this process).
_spec = importlib.util.spec_from_file_location(
    "ikea_synth", os.path.join(REPO, "ikea-recommender-system_amd", "recommenders",
                               "data_utils", "synthetic.py"))
synth = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(synth)

from recommenders.models.GRU4Rec.model import GRU4Rec_trainer  # noqa: E402
from recommenders.models.BidirGRU4Rec.model import BidirGRU4Rec_trainer  # noqa: E402
from recommenders.models.SQN.sqn_gru import SQN_trainer  # noqa: E402
from recommenders.models.SMORL.smorl_gru import SMORL_trainer  # noqa: E402
from recommenders.utils.tensor_operations import (  # noqa: E402
    gather_from_3d, weighted_q_loss, get_weighted_q_target, get_max_action)
from recommenders.evaluate.diversity import get_batch_diversity_rewards  # noqa: E402
from recommenders.evaluate.novelty import get_batch_novelty_rewards  # noqa: E402
from recommenders.evaluate.eval_protocol import get_hits_for_batch  # noqa: E402

N_ITEMS, EMB, HID, L, B, STEPS, LR = 300, 16, 16, 6, 24, 3, 0.01


def sd_np(prefix, module):
    return {f"{prefix}{k}": v.detach().cpu().numpy().copy() for k, v in module.state_dict().items()}


def batches(seed, n_batches, item_num=N_ITEMS, state_size=L, batch=B, mu=None):
    st = synth.SessionStream(item_num, state_size, batch * n_batches, seed=seed,
                             mean_session_len=mu)
    return st, [st.batch(i, batch) for i in range(n_batches)]


def pack_batches(bs):
    out = {}
    for name, j in (("s", 0), ("a", 1), ("r", 2), ("s_next", 3), ("len", 4),
                    ("next_len", 5), ("is_end", 6)):
        out[f"in_{name}"] = np.stack([b[j].numpy() for b in bs])
    return out


def case_supervised(name, kind, seed, **kw):
    st, bs = batches(seed, STEPS)
    common = dict(hidden_dim=HID, embedding_dim=EMB, gru_layers=kw.get("gru_layers", 1),
                  train_pad_embed=kw.get("train_pad_embed", True),
                  use_packed_seq=kw.get("use_packed_seq", True), learning_rate=LR,
                  item_num=N_ITEMS, state_size=L, action_dim=N_ITEMS, device="cpu")
    if kind == "bidir":
        tr = BidirGRU4Rec_trainer(dropout=kw.get("dropout", 0.0), **common)
    else:
        tr = GRU4Rec_trainer(**common)
    rec = {}
    rec.update(sd_np("init.", tr.gru_model))
    tr.set_eval()
    with torch.no_grad():
        rec["logits0"] = tr.gru_model(bs[0][0], bs[0][4]).numpy()
    tr.set_train()
    losses = []
    for (s, a, r, sn, ln, nln, e) in bs:
        losses.append(tr.train_step(s, a, ln))
    rec["losses"] = np.array(losses, dtype=np.float64)
    rec.update(sd_np("final.", tr.gru_model))
    grads = {p: (t.grad is not None) for p, t in tr.gru_model.named_parameters()}
    rec.update(pack_batches(bs))
    meta = dict(kind=kind, seed=seed, config=dict(common, **kw, device="cpu"),
                params_with_grad=grads)
    meta["config"].pop("device")
    return name, rec, meta


def case_sqn(name, seed, steps=4, **kw):
    st, bs = batches(seed, steps)
    common = dict(hidden_dim=HID, embedding_dim=EMB, train_pad_embed=kw.get("train_pad_embed", True),
                  use_packed_seq=kw.get("use_packed_seq", True), learning_rate=LR,
                  item_num=N_ITEMS, state_size=L, action_dim=N_ITEMS, gamma=0.5,
                  gru_layers=1, device="cpu")
    tr = SQN_trainer(**common)
    rec = {}
    rec.update(sd_np("init1.", tr.DQN_1))
    rec.update(sd_np("init2.", tr.DQN_2))
    py_state = random.getstate()
    draws = [random.uniform(0, 1) for _ in range(steps)]
    random.setstate(py_state)
    sup_l, q_l = [], []
    for (s, a, r, sn, ln, nln, e) in bs:
        x, y = tr.train_step(s, a, r, sn, ln, nln, e)
        sup_l.append(x)
        q_l.append(y)
    rec["sup_losses"] = np.array(sup_l)
    rec["q_losses"] = np.array(q_l)
    rec["main_idx"] = np.array([0 if d <= 0.5 else 1 for d in draws])
    rec.update(sd_np("final1.", tr.DQN_1))
    rec.update(sd_np("final2.", tr.DQN_2))
    rec.update(pack_batches(bs))
    cfg = dict(common)
    cfg.pop("device")
    return name, rec, dict(kind="sqn", seed=seed, config=cfg)


def case_smorl(name, seed, steps=4):
    st, bs = batches(seed, steps)
    g = torch.Generator().manual_seed(7)
    div_table = torch.randn(N_ITEMS + 1, 8, generator=g) * 0.01
    div_emb = torch.nn.Embedding.from_pretrained(div_table, freeze=True)
    unpop = synth.unpopular_items(st.item_counts())
    w = torch.tensor([1.0, 1.0, 1.0])
    gamma, alpha, topk_div, topk_nov, nov_sig = 0.5, 1.0, 1, 1, 1.0
    tr = SMORL_trainer(hidden_dim=HID, embedding_dim=EMB, padding_pos="end", train_pad_embed=True,
                       use_packed_seq=True, learning_rate=LR, item_num=N_ITEMS, state_size=L,
                       action_dim=N_ITEMS, gamma=gamma, gru_layers=1, q_weights=w, alpha=alpha,
                       div_embedding=div_emb, unpopular_actions_set=unpop, topk_div=topk_div,
                       device="cpu")
    rec = {}
    rec.update(sd_np("init1.", tr.SMORL_1))
    rec.update(sd_np("init2.", tr.SMORL_2))
    sup_l, q_l, mains, rewards = [], [], [], []
    for (s, a, r_acc, sn, ln, nln, e) in bs:
        # smorl_gru.py:247-332 with the third reward stacked (composition).
        r_acc = r_acc.unsqueeze(1)
        if random.uniform(0, 1) <= 0.5:
            main, boot, opt, k = tr.SMORL_1, tr.SMORL_2, tr.optimizer_1, 0
        else:
            main, boot, opt, k = tr.SMORL_2, tr.SMORL_1, tr.optimizer_2, 1
        sup, q_all = main(s, ln)
        sup_loss = tr.cross_entropy_loss(sup, a)
        q = gather_from_3d(q_all, a, num_heads=q_all.size(1))
        with torch.no_grad():
            _, q_out_next = main(sn, nln)
            a_star = get_max_action(get_weighted_q_target(q_vals=q_out_next, w=w))
            _, q_boot = boot(sn, ln)
            q_next = gather_from_3d(q_boot, a_star, num_heads=q_boot.size(1))
            q_next[e, :] = 0.0
            r_div = get_batch_diversity_rewards(s=s, predictions=sup, len_states=nln,
                                                padding_pos="end", topk_to_consider=topk_div,
                                                embedding_layer=div_emb, device="cpu")
            r_nov = torch.from_numpy(get_batch_novelty_rewards(sup, unpop, nov_sig, topk_nov))
            rr = torch.stack([r_acc.squeeze(), r_div.to(torch.float64), r_nov], dim=1)
            rr = rr.to(torch.float32)
        q_loss = torch.mean(weighted_q_loss((rr + gamma * q_next - q) ** 2, w))
        loss = sup_loss + alpha * q_loss
        opt.zero_grad()
        loss.backward()
        opt.step()
        sup_l.append(sup_loss.item())
        q_l.append(q_loss.item())
        mains.append(k)
        rewards.append(rr.numpy())
    rec["sup_losses"] = np.array(sup_l)
    rec["q_losses"] = np.array(q_l)
    rec["main_idx"] = np.array(mains)
    rec["rewards"] = np.stack(rewards)
    rec["div_table"] = div_table.numpy()
    rec["unpopular"] = np.array(sorted(unpop), dtype=np.int64)
    rec.update(sd_np("final1.", tr.SMORL_1))
    rec.update(sd_np("final2.", tr.SMORL_2))
    rec.update(pack_batches(bs))
    cfg = dict(hidden_dim=HID, embedding_dim=EMB, train_pad_embed=True, use_packed_seq=True,
               learning_rate=LR, item_num=N_ITEMS, state_size=L, action_dim=N_ITEMS,
               gamma=gamma, gru_layers=1, q_weights=[1.0, 1.0, 1.0], alpha=alpha,
               topk_div=topk_div, topk_nov=topk_nov, nov_rew_sig=nov_sig, padding_pos="end")
    return name, rec, dict(kind="smorl", seed=seed, config=cfg, composed=True)


def case_metrics(name, seed):
    g = torch.Generator().manual_seed(seed)
    Bm, Am = 64, 500
    preds = torch.randn(Bm, Am, generator=g)
    true_idx = torch.randint(0, Am, (Bm,), generator=g)
    # plant some hits at known ranks
    top = torch.topk(preds, 25).indices
    true_idx[:20] = top[torch.arange(20), torch.arange(20)]
    ks = [1, 5, 10, 20]
    hits, ndcg = get_hits_for_batch(preds, true_idx, top_k=ks)
    unpop = set(range(0, Am, 3))
    nov1 = get_batch_novelty_rewards(preds, unpop, 1, 1)
    nov5 = get_batch_novelty_rewards(preds, unpop, 2, 5)
    table = torch.randn(Am + 1, 8, generator=g)
    emb = torch.nn.Embedding.from_pretrained(table, freeze=True)
    s = torch.randint(0, Am, (Bm, 5), generator=g)
    lens = torch.randint(1, 6, (Bm,), generator=g)
    s[torch.arange(5).view(1, -1) >= lens.view(-1, 1)] = Am
    div1 = get_batch_diversity_rewards(s, preds, lens, "end", 1, emb, device="cpu")
    div3 = get_batch_diversity_rewards(s, preds, lens, "end", 3, emb, device="cpu")
    rec = dict(preds=preds.numpy(), true_idx=true_idx.numpy(), ks=np.array(ks), hits=hits,
               ndcg=ndcg, unpop=np.array(sorted(unpop)), nov1=nov1, nov5=nov5,
               div_table=table.numpy(), s=s.numpy(), lens=lens.numpy(), div1=div1.numpy(),
               div3=div3.numpy())
    return name, rec, dict(kind="metrics", seed=seed)


def main():
    torch.set_num_threads(1)
    cases = [
        case_supervised("gru4rec_packed", "gru4rec", 11),
        case_supervised("gru4rec_unpacked_fixedpad", "gru4rec", 12, use_packed_seq=False,
                        train_pad_embed=False),
        case_supervised("gru4rec_layers2", "gru4rec", 13, gru_layers=2),
        case_supervised("bidir_packed", "bidir", 14, dropout=0.0),
        case_supervised("bidir_dropout", "bidir", 15, dropout=0.3),
        case_sqn("sqn_packed", 16),
        case_smorl("smorl_composed", 17),
        case_metrics("metrics", 18),
    ]
    meta = {"torch": torch.__version__, "numpy": np.__version__, "cases": {}}
    for name, rec, m in cases:
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **rec)
        meta["cases"][name] = m
    with open(os.path.join(HERE, "meta.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True, default=str)
    print("wrote", [c[0] for c in cases])


if __name__ == "__main__":
    sys.exit(main())
