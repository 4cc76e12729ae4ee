"""Deterministic synthetic session stream.

Produces replay-buffer transitions with exactly the tuple layout and dtypes the
reference's ``ReplayBuffer.__getitem__`` + torch default collate hand to
``train_step`` (``recommenders/data_utils/replay_buffer.py:65-74``):

    s        int64 (B, L)   end-padded with pad id = item_num
    a        int64 (B,)
    r        float64 (B,)   click 0.2 / buy 1.0
    s_next   int64 (B, L)
    s_len    int64 (B,)     in [1, L]
    s_next_len int64 (B,)   in [1, L]
    is_end   bool (B,)

Transition rules follow the reference preprocessing
(``recommenders/data_utils/preprocessing.py:5-29`` get_state,
``:143-170`` get_next_state, ``:426-464`` is_end / length clamps):

* state = the last <= L items *before* the current event, padded with pad id;
* true_len = clamp(n_items_before, 1, L)  (first state is all-pad with len 1);
* next_state = the last <= L items up to and including the current event;
* true_next_len = min(n_items_before + 1, L);
* is_end = the event is the last of its session.

Item popularity is Zipf(alpha) over ranks mapped through a seeded
permutation of [0, N); session length is Geometric(1/mu) on {1, 2, ...}
(mean mu) truncated at 4L.  Everything is driven by one ``numpy.random.PCG64(seed)`` so the HIP path
and the CPU oracle consume byte-identical batches.
"""
from __future__ import annotations

import numpy as np
import torch


class SessionStream:
    """A finite stream of transitions, sliced into consecutive batches."""

    def __init__(
        self,
        item_num: int,
        state_size: int,
        n_transitions: int,
        seed: int = 1,
        zipf_alpha: float = 1.1,
        mean_session_len: float | None = None,
        p_buy: float = 0.046,
        pad_pos: str = "end",
    ):
        if pad_pos not in ("end", "beg"):
            raise ValueError("pad_pos must be 'end' or 'beg'")
        self.item_num = int(item_num)
        self.state_size = L = int(state_size)
        self.pad_id = self.item_num
        self.pad_pos = pad_pos
        rng = np.random.Generator(np.random.PCG64(seed))
        mu = float(mean_session_len) if mean_session_len else max(L / 2.0, 1.0)

        # Zipf popularity over ranks 1..N, mapped through a seeded permutation.
        ranks = np.arange(1, self.item_num + 1, dtype=np.float64)
        w = ranks ** (-zipf_alpha)
        cdf = np.cumsum(w)
        cdf /= cdf[-1]
        perm = rng.permutation(self.item_num).astype(np.int64)

        # Sessions until we have enough events (each event = one transition).
        lens = []
        total = 0
        p_geo = 1.0 / mu
        while total < n_transitions:
            # numpy's geometric has support {1, 2, ...} and mean mu.
            chunk = np.minimum(rng.geometric(p_geo, size=4096), 4 * L)
            lens.append(chunk)
            total += int(chunk.sum())
        sess_len = np.concatenate(lens)
        csum = np.cumsum(sess_len)
        n_sess = int(np.searchsorted(csum, n_transitions) + 1)
        sess_len = sess_len[:n_sess]
        n_events = int(sess_len.sum())

        u = rng.random(n_events)
        items = perm[np.minimum(np.searchsorted(cdf, u, side="right"), self.item_num - 1)]
        rewards = np.where(rng.random(n_events) < p_buy, 1.0, 0.2).astype(np.float64)

        starts = np.concatenate([[0], np.cumsum(sess_len)[:-1]]).astype(np.int64)
        sess_of_event = np.repeat(np.arange(n_sess), sess_len)
        n_bef = np.arange(n_events, dtype=np.int64) - starts[sess_of_event]
        is_end = n_bef == (sess_len[sess_of_event] - 1)

        self.items = items
        self.s, self.s_len = self._window(items, starts[sess_of_event], n_bef, n_bef, L)
        self.s_next, _ = self._window(items, starts[sess_of_event], n_bef + 1, n_bef, L)
        self.a = items.astype(np.int64)
        self.r = rewards
        self.true_len = np.clip(n_bef, 1, L).astype(np.int64)
        self.true_next_len = np.minimum(n_bef + 1, L).astype(np.int64)
        self.is_end = is_end
        self.n = n_transitions
        for name in ("s", "s_next", "a", "r", "true_len", "true_next_len", "is_end"):
            setattr(self, name, getattr(self, name)[:n_transitions])

    def _window(self, items, start, n_hist, n_bef, L):
        """State made of the last min(n_hist, L) items of the session history."""
        n = items.shape[0]
        take = np.minimum(n_hist, L)
        first = start + n_hist - take
        out = np.full((n, L), self.pad_id, dtype=np.int64)
        pos = np.arange(L)[None, :]
        valid = pos < take[:, None]
        src = first[:, None] + pos
        src = np.where(valid, src, 0)
        vals = items[src]
        if self.pad_pos == "end":
            out = np.where(valid, vals, self.pad_id)
        else:
            shift = (L - take)[:, None]
            pos_b = pos - shift
            valid_b = pos_b >= 0
            src_b = np.where(valid_b, first[:, None] + pos_b, 0)
            out = np.where(valid_b, items[src_b], self.pad_id)
        return out.astype(np.int64), take

    def __len__(self):
        return self.n

    def batch(self, i: int, batch_size: int):
        """Batch ``i`` (consecutive slice, no shuffle) as the 7-tuple of torch tensors."""
        lo = i * batch_size
        hi = lo + batch_size
        if hi > self.n:
            raise IndexError("stream exhausted")
        t = torch.from_numpy
        return (
            t(self.s[lo:hi].copy()),
            t(self.a[lo:hi].copy()),
            t(self.r[lo:hi].copy()),
            t(self.s_next[lo:hi].copy()),
            t(self.true_len[lo:hi].copy()),
            t(self.true_next_len[lo:hi].copy()),
            t(self.is_end[lo:hi].copy()),
        )

    def item_counts(self) -> np.ndarray:
        return np.bincount(self.a, minlength=self.item_num)


def unpopular_items(counts: np.ndarray, quantile: float = 0.9) -> set:
    """Unpopular set rule of ``recommenders/data_utils/item_frequency.py:8-24``:
    items (that occur) whose frequency is below the ``quantile`` of the
    frequency distribution of occurring items."""
    occ = np.nonzero(counts)[0]
    freq = counts[occ]
    thresh = np.quantile(freq, q=quantile)
    return set(int(i) for i in occ[freq < thresh])


def transitions_from_sessions(sessions, state_len, pad_id, pad_pos="end"):
    """Transition builder over explicit sessions (list of item lists); used to
    check the rules against the reference's known-answer preprocessing test."""
    items = np.concatenate([np.asarray(x, dtype=np.int64) for x in sessions])
    lens = np.array([len(x) for x in sessions], dtype=np.int64)
    starts = np.concatenate([[0], np.cumsum(lens)[:-1]])
    sess = np.repeat(np.arange(len(sessions)), lens)
    n_bef = np.arange(items.shape[0]) - starts[sess]
    st = SessionStream.__new__(SessionStream)
    st.pad_id = pad_id
    st.pad_pos = pad_pos
    s, _ = st._window(items, starts[sess], n_bef, n_bef, state_len)
    s_next, _ = st._window(items, starts[sess], n_bef + 1, n_bef, state_len)
    true_len = np.clip(n_bef, 1, state_len)
    true_next_len = np.minimum(n_bef + 1, state_len)
    is_end = n_bef == lens[sess] - 1
    return s, items, s_next, true_len, true_next_len, is_end
