"""GPU parity: SQN double-Q and SMORL 3-reward steps vs the reference's golden
vectors (tests/golden/sqn_packed.npz — the reference SQN_trainer itself;
smorl_composed.npz — the reference helpers composed, since the shipped SMORL
step raises).  Tolerances as tests/test_gpu_supervised.py; Q losses 1e-5."""
import json
import os
import random

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from test_gpu_supervised import bt, compare_params, load

pytestmark = pytest.mark.gpu

META = json.load(open(os.path.join(GOLDEN, "meta.json")))


def test_sqn_matches_reference_golden():
    from recommenders.models.SQN.sqn_gru import SQN_trainer
    g = load("sqn_packed")
    cfg = META["cases"]["sqn_packed"]["config"]
    tr = SQN_trainer(device="cuda", **cfg)
    for net, pre in ((tr.DQN_1, "init1."), (tr.DQN_2, "init2.")):
        for k, v in net.state_dict().items():
            np.testing.assert_array_equal(v.cpu().numpy(), g[pre + k], err_msg=k)
    sup, q, mains = [], [], []
    for i in range(g["in_s"].shape[0]):
        x, y = tr.train_step(*bt(g, i))
        sup.append(x)
        q.append(y)
        mains.append(tr.last_main)
    np.testing.assert_array_equal(mains, g["main_idx"])
    np.testing.assert_allclose(sup, g["sup_losses"], rtol=0, atol=1e-4)
    np.testing.assert_allclose(q, g["q_losses"], rtol=0, atol=1e-5)
    compare_params(tr.DQN_1.state_dict(), g, "final1.", cfg["learning_rate"])
    compare_params(tr.DQN_2.state_dict(), g, "final2.", cfg["learning_rate"])


def test_smorl_matches_composed_reference_golden():
    from recommenders.models.SMORL.smorl_gru import SMORL_trainer
    g = load("smorl_composed")
    cfg = dict(META["cases"]["smorl_composed"]["config"])
    table = torch.nn.Embedding.from_pretrained(torch.from_numpy(g["div_table"]), freeze=True)
    unpop = set(int(x) for x in g["unpopular"])
    q_weights = torch.tensor(cfg.pop("q_weights"))
    tr = SMORL_trainer(device="cuda", div_embedding=table, unpopular_actions_set=unpop, q_weights=q_weights,
                       **cfg)
    for net, pre in ((tr.SMORL_1, "init1."), (tr.SMORL_2, "init2.")):
        for k, v in net.state_dict().items():
            np.testing.assert_array_equal(v.cpu().numpy(), g[pre + k], err_msg=k)
    sup, q, rw = [], [], []
    for i in range(g["in_s"].shape[0]):
        x, y = tr.train_step(*bt(g, i))
        sup.append(x)
        q.append(y)
        rw.append(tr.last_rewards.cpu().numpy().copy())
    np.testing.assert_allclose(np.stack(rw), g["rewards"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(sup, g["sup_losses"], rtol=0, atol=1e-4)
    np.testing.assert_allclose(q, g["q_losses"], rtol=0, atol=1e-5)
    compare_params(tr.SMORL_1.state_dict(), g, "final1.", cfg["learning_rate"])
    compare_params(tr.SMORL_2.state_dict(), g, "final2.", cfg["learning_rate"])


@pytest.mark.parametrize("N,L,B,H", [(20000, 20, 512, 64), (6000, 10, 160, 256)])
def test_sqn_matches_oracle_medium(N, L, B, H):
    """H = 256 runs the time-stepped GRU (config C5's hidden size)."""
    from oracle.models import OracleSQN
    from recommenders.data_utils.synthetic import SessionStream
    from recommenders.models.SQN.sqn_gru import SQN_trainer
    cfg = dict(hidden_dim=H, embedding_dim=H, train_pad_embed=True, use_packed_seq=True, learning_rate=0.005,
               item_num=N, state_size=L, action_dim=N, gamma=0.5, gru_layers=1)
    torch.set_num_threads(8)
    orc = OracleSQN(**cfg)
    rs_o = random.getstate()
    tr = SQN_trainer(device="cuda", **cfg)
    rs_t = random.getstate()
    st = SessionStream(N, L, B * 4, seed=9)
    for i in range(4):
        b = st.batch(i, B)
        random.setstate(rs_o)   # both draw main/boot from Python's global RNG
        so, qo = orc.step(*b)
        rs_o = random.getstate()
        random.setstate(rs_t)
        sg, qg = tr.train_step(*b)
        rs_t = random.getstate()
        assert orc.last_main == tr.last_main
        assert abs(so - sg) < 1e-4 and abs(qo - qg) < 1e-5, (i, so, sg, qo, qg)


@pytest.mark.parametrize("precision", ["f32", "f32x6", "f32x6d3"])
def test_smorl_c5_shape_matches_oracle(precision):
    """Config C5's model shape on one GPU, scaled down in items and batch:
    SMORL 3-reward at d256 (E = H = 256: the time-stepped GRU), fp16 item
    table (fp32 master + Adam), seq_len 100, top-k rewards with k > 1, against
    the oracle's restatement of the same storage.  f32x6: the supervised head
    on the fused split-bf16 path with its top-k recomputed for the rewards."""
    from oracle.models import OracleSMORL
    from recommenders.data_utils.synthetic import SessionStream, unpopular_items
    from recommenders.models.SMORL.smorl_gru import SMORL_trainer
    N, L, B, E = 4000, 100, 128, 256
    st = SessionStream(N, L, B * 4, seed=17)
    g = torch.Generator().manual_seed(7)
    table = torch.randn(N + 1, 32, generator=g) * 0.01
    unpop = unpopular_items(st.item_counts())
    cfg = dict(hidden_dim=E, embedding_dim=E, padding_pos="end", train_pad_embed=True, use_packed_seq=True,
               learning_rate=0.005, item_num=N, state_size=L, action_dim=N, gamma=0.5, gru_layers=1,
               q_weights=[1.0, 0.5, 2.0], alpha=1.0, div_embedding=table, unpopular_actions_set=unpop, topk_div=3,
               topk_nov=2, nov_rew_sig=1.0, fp16_embeddings=True)
    torch.set_num_threads(8)
    orc = OracleSMORL(**cfg)
    rs_o = random.getstate()
    tr = SMORL_trainer(device="cuda", matmul_precision=precision, **cfg)
    rs_t = random.getstate()
    for i in range(4):
        b = st.batch(i, B)
        random.setstate(rs_o)
        so, qo = orc.step(*b)
        rs_o = random.getstate()
        random.setstate(rs_t)
        sg, qg = tr.train_step(*b)
        rs_t = random.getstate()
        assert orc.last_main == tr.last_main
        np.testing.assert_allclose(tr.last_rewards.cpu().numpy(), orc.last_rewards.numpy(), rtol=0, atol=1e-5)
        assert abs(so - sg) < 1e-4 and abs(qo - qg) < 1e-5, (i, so, sg, qo, qg)
    lr = cfg["learning_rate"]
    for mine, ref in ((tr.SMORL_1, orc.nets[0]), (tr.SMORL_2, orc.nets[1])):
        sd_o = ref.state_dict()
        for k, v in mine.state_dict().items():
            d = (v.cpu() - sd_o[k]).abs()
            assert float(d.max()) <= 2 * lr + 1e-5, k
            assert float((d > 1e-4).float().mean()) < 1e-3, k
        assert torch.equal(mine.trunk.emb16.cpu(), mine.trunk.emb.p.cpu().half())


def test_smorl_c4_bench_path_matches_oracle():
    """The benched C4 instantiation (bench.py --config c4) at an oracle-sized
    item count: SMORL 3-reward, H = E = 128, B % 32 == 0, L 50, precision
    f32x6d3 (fused supervised head k_flash_fwd<128, 6, 3, true>: pass 1's
    top-1 for the rewards re-scored in fp32, rg_flash_topk K = 1), screening
    argmax for the double-Q target, q_weights [1, 1, 1], topk_div = topk_nov
    = 1 — against OracleSMORL (the reference's helpers composed,
    smorl_gru.py:233-334)."""
    from oracle.models import OracleSMORL
    from recommenders.data_utils.synthetic import SessionStream, unpopular_items
    from recommenders.models.SMORL.smorl_gru import SMORL_trainer
    N, L, B, E = 30000, 50, 256, 128
    st = SessionStream(N, L, B * 4, seed=21)
    g = torch.Generator().manual_seed(7)
    table = torch.randn(N + 1, 64, generator=g) * 0.01
    unpop = unpopular_items(st.item_counts())
    cfg = dict(hidden_dim=E, embedding_dim=E, padding_pos="end", train_pad_embed=True, use_packed_seq=True,
               learning_rate=0.01, item_num=N, state_size=L, action_dim=N, gamma=0.5, gru_layers=1,
               q_weights=[1.0, 1.0, 1.0], alpha=1.0, div_embedding=table, unpopular_actions_set=unpop, topk_div=1,
               topk_nov=1, nov_rew_sig=1.0)
    torch.set_num_threads(8)
    orc = OracleSMORL(**cfg)
    rs_o = random.getstate()
    tr = SMORL_trainer(device="cuda", matmul_precision="f32x6d3", **cfg)
    rs_t = random.getstate()
    assert tr.SMORL_1.sup_head_output.flash_terms(B) == 636
    for i in range(4):
        b = st.batch(i, B)
        random.setstate(rs_o)
        so, qo = orc.step(*b)
        rs_o = random.getstate()
        random.setstate(rs_t)
        sg, qg = tr.train_step(*b)
        rs_t = random.getstate()
        assert orc.last_main == tr.last_main
        np.testing.assert_allclose(tr.last_rewards.cpu().numpy(), orc.last_rewards.numpy(), rtol=0, atol=1e-5)
        assert abs(so - sg) < 1e-4 and abs(qo - qg) < 1e-5, (i, so, sg, qo, qg)
    lr = cfg["learning_rate"]
    for mine, ref in ((tr.SMORL_1, orc.nets[0]), (tr.SMORL_2, orc.nets[1])):
        sd_o = ref.state_dict()
        for k, v in mine.state_dict().items():
            d = (v.cpu() - sd_o[k]).abs()
            assert float(d.max()) <= 2 * lr + 1e-5, k
            assert float((d > 1e-4).float().mean()) < 1e-3, k


def test_smorl_unmapped_token_raises_before_update():
    """Tokenizer pair where a predicted output id has no input token: the
    reference's stoi raises KeyError inside the diversity reward, before its
    backward; here RemapError is raised before any parameter update (weights,
    Adam moments and clocks unchanged), on train_step and train_step_async."""
    from recommenders.data_utils.synthetic import SessionStream, unpopular_items
    from recommenders.hip.remap import RemapError
    from recommenders.models.SMORL.smorl_gru import SMORL_trainer
    from recommenders.utils.tokenizer import Tokenizer
    N, L, B, E = 2000, 10, 64, 32
    st = SessionStream(N, L, B, seed=5)
    names = [f"item{j}" for j in range(N)]
    tout = Tokenizer(names)
    tin = Tokenizer(names[: N // 4])     # no <unk>: three quarters of the ids cannot be mapped
    table = torch.randn(N // 4 + 2, 16)
    tr = SMORL_trainer(hidden_dim=E, embedding_dim=E, padding_pos="end", train_pad_embed=True, use_packed_seq=True,
                       learning_rate=0.01, item_num=N, state_size=L, action_dim=N, gamma=0.5, gru_layers=1,
                       q_weights=[1.0, 1.0, 1.0], alpha=1.0, div_embedding=table,
                       unpopular_actions_set=unpopular_items(st.item_counts()), topk_div=8, topk_nov=1,
                       device="cuda", input_tokenizer=tin, output_tokenizer=tout)
    before = [{k: v.clone() for k, v in net.state_dict().items()} for net in (tr.SMORL_1, tr.SMORL_2)]
    clocks = (tr.clock_1.t, tr.clock_2.t)
    for fn in (tr.train_step, tr.train_step_async):
        with pytest.raises(RemapError):
            fn(*st.batch(0, B))
    torch.cuda.synchronize()
    assert (tr.clock_1.t, tr.clock_2.t) == clocks
    for net, sd in zip((tr.SMORL_1, tr.SMORL_2), before):
        for k, v in net.state_dict().items():
            assert torch.equal(v, sd[k]), k


@pytest.mark.parametrize("kind", ["sqn", "smorl"])
def test_double_q_steps_are_bitwise_repeatable(kind):
    """Two runs of the same SQN / SMORL steps are bit for bit identical: the
    Q heads' row gradients are summed per action through the sorted scatter
    (recommenders/hip/qlearn.q_heads_backward), not float atomics — 300
    actions for 512 rows, so most actions collect several contributions."""
    from recommenders.data_utils.synthetic import SessionStream
    N, L, B, E = 300, 8, 512, 32
    st = SessionStream(N, L, B * 3, seed=23)
    cfg = dict(hidden_dim=E, embedding_dim=E, train_pad_embed=True, use_packed_seq=True, learning_rate=0.01,
               item_num=N, state_size=L, action_dim=N, gamma=0.5, gru_layers=1)
    runs = []
    for _ in range(2):
        random.seed(4)
        if kind == "sqn":
            from recommenders.models.SQN.sqn_gru import SQN_trainer
            tr = SQN_trainer(device="cuda", **cfg)
            nets = (tr.DQN_1, tr.DQN_2)
        else:
            from recommenders.models.SMORL.smorl_gru import SMORL_trainer
            g = torch.Generator().manual_seed(7)
            tr = SMORL_trainer(device="cuda", padding_pos="end", q_weights=[1.0, 0.5, 2.0], alpha=1.0,
                               div_embedding=torch.randn(N + 1, 16, generator=g) * 0.01,
                               unpopular_actions_set=set(range(0, N, 3)), nov_rew_sig=1.0, topk_div=1, topk_nov=1,
                               **cfg)
            nets = (tr.SMORL_1, tr.SMORL_2)
        losses = [tr.train_step(*st.batch(i, B)) for i in range(3)]
        runs.append((losses, [{k: v.cpu() for k, v in n.state_dict().items()} for n in nets]))
    assert runs[0][0] == runs[1][0]
    for sd0, sd1 in zip(runs[0][1], runs[1][1]):
        for k in sd0:
            assert torch.equal(sd0[k], sd1[k]), k
