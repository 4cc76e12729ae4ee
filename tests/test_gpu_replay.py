"""Device replay ingest: transitions built on the MI355X
from the session store equal the host builder (itself pinned to the
reference's preprocessing known-answer test) bit for bit; the loader covers
every event once per epoch; the pinned double-buffered H2D prefetcher hands
the trainer the same batches as direct host tensors."""
import numpy as np
import pytest
import torch

from recommenders.data_utils.replay_buffer import DeviceLoader, DeviceSessions, PinnedPrefetcher, SessionStore

pytestmark = pytest.mark.gpu


def _store(n_sess, max_len, seed):
    rng = np.random.default_rng(seed)
    lens = rng.integers(1, max_len + 1, n_sess)
    items = rng.integers(0, 5000, int(lens.sum()))
    rew = np.where(rng.random(int(lens.sum())) < 0.1, 1.0, 0.2)
    return SessionStore(items, rew, np.concatenate([[0], np.cumsum(lens)]))


@pytest.mark.parametrize("pad_pos,L", [("end", 10), ("beg", 10), ("end", 1), ("end", 70)])
def test_device_transitions_equal_host(pad_pos, L):
    st = _store(300, 40, L)
    ds = DeviceSessions(st, L, 5000, pad_pos)
    ev = np.random.default_rng(1).permutation(len(st))[:1000]
    dev = ds.batch(torch.from_numpy(ev))
    host = st.host_batch(ev, L, 5000, pad_pos)
    for d, h in zip(dev, host):
        assert torch.equal(d.cpu(), h), (pad_pos, L)


def test_device_loader_epoch():
    st = _store(200, 30, 3)
    ds = DeviceSessions(st, 8, 5000)
    seen = torch.cat([b[1].cpu() for b in DeviceLoader(ds, 64, shuffle=False, drop_last=False)])
    assert torch.equal(seen, torch.from_numpy(st.items.astype(np.int64)))
    n = 0
    for b in DeviceLoader(ds, 64, shuffle=True, seed=5):
        assert b[0].shape == (64, 8) and b[0].device.type == "cuda"
        n += 1
    assert n == len(st) // 64


def test_pinned_prefetcher_feeds_trainer():
    from recommenders.data_utils.synthetic import SessionStream
    from recommenders.models.GRU4Rec.model import GRU4Rec_trainer
    cfg = dict(hidden_dim=32, embedding_dim=32, gru_layers=1, train_pad_embed=True, use_packed_seq=True,
               learning_rate=0.01, item_num=800, state_size=8, action_dim=800, device="cuda")
    st = SessionStream(800, 8, 64 * 6, seed=4)
    host = [st.batch(i, 64) for i in range(6)]
    a, b = GRU4Rec_trainer(**cfg), GRU4Rec_trainer(**cfg)
    la = [a.train_step(x[0], x[1], x[4]) for x in host]
    lb = []
    for x in PinnedPrefetcher(host):
        assert x[0].device.type == "cuda"
        lb.append(b.train_step(x[0], x[1], x[4]))
    assert la == lb
