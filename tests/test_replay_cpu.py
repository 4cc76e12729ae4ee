"""Host logic of the replay-buffer ingest and the tokenizer (SURVEY §8f ranks
2 and 4): the session store's transitions follow the reference's
preprocessing rules (pinned by its known-answer test through
transitions_from_sessions), the columnar formats round-trip, the reference's
pickled-DataFrame input reads back with the reference dtypes, and the
Tokenizer / remap table follow the reference's stoi / itos semantics."""
import numpy as np
import pandas as pd
import pytest
import torch

from recommenders.data_utils.replay_buffer import ReplayBuffer, SessionStore
from recommenders.data_utils.synthetic import transitions_from_sessions
from recommenders.utils.tokenizer import Tokenizer

SESS = [[1, 2, 3, 4], [6, 7, 8, 9, 10, 11], [100, 101]]
P = 999


@pytest.mark.parametrize("pad_pos", ["end", "beg"])
def test_session_store_matches_reference_rules(pad_pos):
    rew = [[0.2, 1.0, 0.2, 0.2], [0.2] * 6, [1.0, 0.2]]
    st = SessionStore.from_sessions(SESS, rew)
    ev = np.arange(len(st))
    s, a, r, sn, tl, tnl, e = st.host_batch(ev, 3, P, pad_pos)
    s2, a2, sn2, tl2, tnl2, e2 = transitions_from_sessions(SESS, 3, P, pad_pos)
    assert np.array_equal(s.numpy(), s2) and np.array_equal(sn.numpy(), sn2)
    assert np.array_equal(a.numpy(), a2) and np.array_equal(tl.numpy(), tl2) and np.array_equal(tnl.numpy(), tnl2)
    assert np.array_equal(e.numpy(), e2)
    assert np.array_equal(r.numpy(), np.concatenate(rew))
    # any subset / order of events gives the same rows
    pick = np.array([11, 0, 5, 3])
    s3 = st.host_batch(pick, 3, P, pad_pos)[0]
    assert np.array_equal(s3.numpy(), s2[pick])


def test_session_store_npz_round_trip(tmp_path):
    st = SessionStore.from_sessions(SESS)
    st.save(tmp_path / "sess.npz")
    st2 = SessionStore.load(tmp_path / "sess.npz")
    for k in ("items", "rewards", "offsets"):
        assert np.array_equal(getattr(st, k), getattr(st2, k))
    with pytest.raises(ValueError):
        SessionStore([1, 2], [0.0, 0.0], [0, 2, 2])   # empty session


def _frame():
    s, a, sn, tl, tnl, e = transitions_from_sessions(SESS, 3, P, "end")
    return pd.DataFrame({"state": list(map(list, s)), "next_state": list(map(list, sn)), "action": a,
                         "r_act": np.where(np.arange(len(a)) % 3 == 0, 1.0, 0.2), "true_state_len": tl,
                         "true_next_state_len": tnl, "is_end": e})


def test_replay_buffer_reads_reference_pickle_and_npz(tmp_path):
    df = _frame()
    df.to_pickle(tmp_path / "replay.df")           # this test's own file, in the reference's input format
    rb = ReplayBuffer(str(tmp_path / "replay.df"), num_items=P)
    assert len(rb) == len(df)
    for i in (0, 3, 11):
        s, a, r, sn, tl, tnl, e = rb[i]
        assert list(s) == df.state[i] and list(sn) == df.next_state[i]
        assert (a, r, tl, tnl, e) == (df.action[i], df.r_act[i], df.true_state_len[i], df.true_next_state_len[i],
                                      df.is_end[i])
    batch = next(iter(torch.utils.data.DataLoader(rb, batch_size=5)))
    assert [t.dtype for t in batch] == [torch.int64, torch.int64, torch.float64, torch.int64, torch.int64,
                                        torch.int64, torch.bool]
    rb.save_npz(tmp_path / "replay.npz")
    rb2 = ReplayBuffer(str(tmp_path / "replay.npz"), num_items=P)
    for i in range(len(rb)):
        for x, y in zip(rb[i], rb2[i]):
            assert np.array_equal(x, y)


def test_tokenizer_semantics(tmp_path):
    t = Tokenizer(["a", "b", "c"], unknown=True)
    assert (t.stoi("a"), t.stoi("c"), t.unk_idx, t.pad_idx, len(t)) == (0, 2, 3, 4, 5)
    assert t.stoi("zzz") == t.unk_idx and t.itos(4) == "<pad>"
    t2 = Tokenizer(["x", "y"])
    with pytest.raises(KeyError):
        t2.stoi("a")
    t.save_to_file(tmp_path / "tok.json")
    t3 = Tokenizer.from_file(tmp_path / "tok.json")
    assert t3.stoi_ == t.stoi_ and t3.itos_ == t.itos_ and t3.unknown and t3.pad_idx == 4
    t4 = Tokenizer(["p", "q"])
    t4.extend(["r"])                                # reference numbering: len - 1 + i
    assert t4.stoi("r") == 2 and t4.itos(3) == "r"


def test_remap_table_follows_stoi_itos():
    from recommenders.hip.remap import remap_table
    out = Tokenizer(["b", "a", "d"], padding=False)
    inp = Tokenizer(["a", "b", "c"])                # "d" is not in the input vocabulary
    lut = remap_table(inp, out, "cpu")
    assert lut.tolist() == [1, 0, -1]
    inp_unk = Tokenizer(["a", "b", "c"], unknown=True)
    assert remap_table(inp_unk, out, "cpu").tolist() == [1, 0, inp_unk.unk_idx]
