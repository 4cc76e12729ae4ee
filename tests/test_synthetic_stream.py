"""Batch contract: the synthetic transition builder follows
the reference preprocessing rules, pinned by the reference's own known-answer
test (test/test_preprocessing.py:5-140: 3 sessions, state_len 3, pad 999)."""
import numpy as np
import torch

from recommenders.data_utils.synthetic import SessionStream, transitions_from_sessions, unpopular_items

SESS = [[1, 2, 3, 4], [6, 7, 8, 9, 10, 11], [100, 101]]
P = 999


def test_known_answer_end_padding():
    s, a, sn, tl, tnl, e = transitions_from_sessions(SESS, 3, P, "end")
    truth = [[P, P, P], [1, P, P], [1, 2, P], [1, 2, 3], [P, P, P], [6, P, P], [6, 7, P],
             [6, 7, 8], [7, 8, 9], [8, 9, 10], [P, P, P], [100, P, P]]
    nxt = [[1, P, P], [1, 2, P], [1, 2, 3], [2, 3, 4], [6, P, P], [6, 7, P], [6, 7, 8],
           [7, 8, 9], [8, 9, 10], [9, 10, 11], [100, P, P], [100, 101, P]]
    assert np.array_equal(s, truth)
    assert np.array_equal(sn, nxt)
    assert list(a) == [1, 2, 3, 4, 6, 7, 8, 9, 10, 11, 100, 101]
    assert list(tl) == [1, 1, 2, 3, 1, 1, 2, 3, 3, 3, 1, 1]
    assert list(tnl) == [1, 2, 3, 3, 1, 2, 3, 3, 3, 3, 1, 2]
    assert list(e) == [False, False, False, True] + [False] * 5 + [True, False, True]


def test_known_answer_beg_padding():
    s, a, sn, *_ = transitions_from_sessions(SESS, 3, P, "beg")
    truth = [[P, P, P], [P, P, 1], [P, 1, 2], [1, 2, 3], [P, P, P], [P, P, 6], [P, 6, 7],
             [6, 7, 8], [7, 8, 9], [8, 9, 10], [P, P, P], [P, P, 100]]
    nxt = [[P, P, 1], [P, 1, 2], [1, 2, 3], [2, 3, 4], [P, P, 6], [P, 6, 7], [6, 7, 8],
           [7, 8, 9], [8, 9, 10], [9, 10, 11], [P, P, 100], [P, 100, 101]]
    assert np.array_equal(s, truth)
    assert np.array_equal(sn, nxt)


def test_stream_tuple_layout_and_determinism():
    st = SessionStream(1000, 8, 512, seed=3)
    b = st.batch(1, 128)
    dt = [torch.int64, torch.int64, torch.float64, torch.int64, torch.int64, torch.int64, torch.bool]
    assert [x.dtype for x in b] == dt
    s, a, r, sn, ln, nln, e = b
    assert s.shape == (128, 8) and sn.shape == (128, 8)
    assert int(ln.min()) >= 1 and int(ln.max()) <= 8
    assert set(np.unique(r.numpy())) <= {0.2, 1.0}
    # end padding: position >= len is pad unless the state is the all-pad first state
    pos = torch.arange(8).view(1, -1)
    first = (s == 1000).all(1)
    assert ((s[~first] == 1000) == (pos >= ln[~first].view(-1, 1))).all()
    b2 = SessionStream(1000, 8, 512, seed=3).batch(1, 128)
    assert all(torch.equal(x, y) for x, y in zip(b, b2))
    u = unpopular_items(st.item_counts())
    assert len(u) > 0 and max(u) < 1000
