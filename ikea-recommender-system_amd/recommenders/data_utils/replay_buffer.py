"""Replay-buffer ingest (reference
``recommenders/data_utils/replay_buffer.py:24-74``).

* ``ReplayBuffer`` — the reference Dataset (same constructor, ``__len__``,
  ``__getitem__`` tuple) over a columnar store: int32 states / next states
  (N × L), int32 actions and lengths, float64 rewards, bool ends.  It reads
  the reference's pickled DataFrame (the user's own file, ``pd.read_pickle``
  as the reference does) or this build's ``.npz`` (``save_npz``; plain arrays,
  loaded with ``allow_pickle=False``).
* ``SessionStore`` — the sessions once, as CSR (items int32, rewards f64,
  offsets int64; ``.npz``), from which every transition is derived by the
  reference rules (preprocessing.py:5-29, 143-170, 426-464): on the host
  (``host_batch``, the checker) or on the MI355X (``DeviceSessions``:
  csrc/replay.hip, no per-batch host copies).
* ``DeviceLoader`` — shuffled (``torch.randperm``, seeded) or sequential
  batches of device transitions, epoch by epoch.
* ``PinnedPrefetcher`` — for host batches (e.g. a DataLoader over
  ``ReplayBuffer``): pinned staging, H2D on a side stream one batch ahead,
  the compute stream waits only for the batch it takes (double buffer).
"""
from __future__ import annotations

import numpy as np
import torch

_COLS = ("states", "actions", "reward", "next_states", "true_state_len", "true_next_state_len", "is_end")


class ReplayBuffer(torch.utils.data.Dataset):
    """Returns s, a, r, s', s_len, s_next_len, is_end (reference order)."""

    def __init__(self, dir, num_items, state_name="state", next_state_name="next_state",  # noqa: A002
                 action_name="action", end_name="is_end", state_len_name="true_state_len",
                 true_next_state_len_name="true_next_state_len", reward_name="r_act"):
        super().__init__()
        self.dir = dir
        self.num_items = num_items
        if str(dir).endswith(".npz"):
            with np.load(dir, allow_pickle=False) as z:
                cols = {k: z[k] for k in _COLS}
        else:
            import pandas as pd
            df = pd.read_pickle(dir)
            cols = {"states": np.array(df[state_name].values.tolist()),
                    "next_states": np.array(df[next_state_name].values.tolist()),
                    "actions": df[action_name].to_numpy(), "reward": df[reward_name].to_numpy(),
                    "true_state_len": df[state_len_name].to_numpy(),
                    "true_next_state_len": df[true_next_state_len_name].to_numpy(),
                    "is_end": df[end_name].to_numpy()}
        self._set(cols)

    def _set(self, cols):
        i32 = lambda x: np.ascontiguousarray(x, dtype=np.int32)  # noqa: E731
        self.states, self.next_states = i32(cols["states"]), i32(cols["next_states"])
        self.actions = i32(cols["actions"])
        self.reward = np.ascontiguousarray(cols["reward"], dtype=np.float64)
        self.true_state_len = i32(cols["true_state_len"])
        self.true_next_state_len = i32(cols["true_next_state_len"])
        self.is_end = np.ascontiguousarray(cols["is_end"], dtype=bool)

    @classmethod
    def from_arrays(cls, num_items, **cols):
        rb = cls.__new__(cls)
        rb.dir, rb.num_items = None, num_items
        rb._set(cols)
        return rb

    def save_npz(self, path):
        np.savez(path, **{k: getattr(self, k) for k in _COLS})

    def __len__(self):
        return len(self.actions)

    def __getitem__(self, idx):
        # int64 like the reference's np.array of Python ints, so default collate gives the same dtypes
        return (self.states[idx].astype(np.int64), np.int64(self.actions[idx]), self.reward[idx],
                self.next_states[idx].astype(np.int64), np.int64(self.true_state_len[idx]),
                np.int64(self.true_next_state_len[idx]), self.is_end[idx])


class SessionStore:
    """Sessions as CSR: event e of session k is items[off[k] + i]."""

    def __init__(self, items, rewards, offsets):
        self.items = np.ascontiguousarray(items, dtype=np.int32)
        self.rewards = np.ascontiguousarray(rewards, dtype=np.float64)
        self.offsets = np.ascontiguousarray(offsets, dtype=np.int64)
        if self.offsets[0] != 0 or self.offsets[-1] != len(self.items) or np.any(np.diff(self.offsets) <= 0):
            raise ValueError("offsets must start at 0, end at len(items) and strictly increase (no empty session)")
        if len(self.rewards) != len(self.items):
            raise ValueError("one reward per event")

    @classmethod
    def from_sessions(cls, sessions, rewards=None):
        lens = [len(x) for x in sessions]
        items = np.concatenate([np.asarray(x, dtype=np.int64) for x in sessions])
        rew = (np.concatenate([np.asarray(x, dtype=np.float64) for x in rewards]) if rewards is not None
               else np.zeros(len(items)))
        return cls(items, rew, np.concatenate([[0], np.cumsum(lens)]))

    @classmethod
    def load(cls, path):
        with np.load(path, allow_pickle=False) as z:
            return cls(z["items"], z["rewards"], z["offsets"])

    def save(self, path):
        np.savez(path, items=self.items, rewards=self.rewards, offsets=self.offsets)

    def __len__(self):
        return len(self.items)   # one transition per event

    def event_session(self):
        return np.repeat(np.arange(len(self.offsets) - 1, dtype=np.int32), np.diff(self.offsets))

    def host_batch(self, ev, state_size, pad_id, pad_pos="end"):
        """The 7-tuple for event indices ``ev`` on the host (numpy rules of
        data_utils.synthetic, pinned by the reference's preprocessing test)."""
        from .synthetic import SessionStream
        ev = np.asarray(ev, dtype=np.int64)
        sess = self.event_session()[ev]
        start = self.offsets[sess]
        n_bef = ev - start
        w = SessionStream.__new__(SessionStream)
        w.pad_id, w.pad_pos = pad_id, pad_pos
        items = self.items.astype(np.int64)
        s, _ = w._window(items, start, n_bef, n_bef, state_size)
        s_next, _ = w._window(items, start, n_bef + 1, n_bef, state_size)
        t = torch.from_numpy
        return (t(s), t(items[ev].copy()), t(self.rewards[ev].copy()), t(s_next),
                t(np.clip(n_bef, 1, state_size)), t(np.minimum(n_bef + 1, state_size)),
                t(ev == self.offsets[sess + 1] - 1))


class DeviceSessions:
    """A SessionStore resident in HBM; ``batch(ev)`` builds transitions there."""

    def __init__(self, store, state_size, pad_id, pad_pos="end", device="cuda"):
        self.device = torch.device(device)
        self.L, self.pad_id, self.pad_end = int(state_size), int(pad_id), pad_pos == "end"
        if pad_pos not in ("end", "beg"):
            raise ValueError("pad_pos must be 'end' or 'beg'")
        self.n = len(store)
        self.items = torch.from_numpy(store.items).to(self.device)
        self.rewards = torch.from_numpy(store.rewards).to(self.device)
        self.ev_sess = torch.from_numpy(store.event_session()).to(self.device)
        self.offsets = torch.from_numpy(store.offsets).to(self.device)

    def batch(self, ev):
        from recommenders.hip import call, stream_ptr
        ev = ev.to(self.device, torch.int64).contiguous()
        B, L = ev.numel(), self.L
        z = lambda *sh, dt=torch.int64: torch.empty(*sh, dtype=dt, device=self.device)  # noqa: E731
        s, s_next, a, ln, nln = z(B, L), z(B, L), z(B), z(B), z(B)
        r = z(B, dt=torch.float64)
        e = z(B, dt=torch.bool)
        call("rg_build_transitions", self.items.data_ptr(), self.rewards.data_ptr(), self.ev_sess.data_ptr(),
             self.offsets.data_ptr(), ev.data_ptr(), B, L, self.pad_id, 1 if self.pad_end else 0, s.data_ptr(),
             a.data_ptr(), r.data_ptr(), s_next.data_ptr(), ln.data_ptr(), nln.data_ptr(), e.data_ptr(),
             stream_ptr())
        return s, a, r, s_next, ln, nln, e


class DeviceLoader:
    """Batches of device transitions: a seeded permutation per epoch
    (DataLoader(shuffle=True) equivalent, one upload per epoch) or the
    events in order; drop_last like the reference's training loaders."""

    def __init__(self, sessions, batch_size, shuffle=True, drop_last=True, seed=0):
        self.sessions, self.B = sessions, int(batch_size)
        self.shuffle, self.drop_last = shuffle, drop_last
        self.gen = torch.Generator().manual_seed(seed)

    def __len__(self):
        n = self.sessions.n
        return n // self.B if self.drop_last else -(-n // self.B)

    def __iter__(self):
        n = self.sessions.n
        order = torch.randperm(n, generator=self.gen) if self.shuffle else torch.arange(n)
        order = order.to(self.sessions.device)
        for i in range(len(self)):
            yield self.sessions.batch(order[i * self.B:(i + 1) * self.B])


class PinnedPrefetcher:
    """Host batches -> device batches, one ahead: each batch is copied into
    pinned memory and sent H2D on a side stream; the consumer's stream waits
    on that copy's event only when it takes the batch."""

    def __init__(self, batches, device="cuda"):
        self.src = batches
        self.device = torch.device(device)
        self.stream = torch.cuda.Stream(device=self.device)

    def _stage(self, b):
        if b is None:
            return None
        with torch.cuda.stream(self.stream):
            out = tuple(torch.as_tensor(x).pin_memory().to(self.device, non_blocking=True) for x in b)
            ev = torch.cuda.Event()
            ev.record(self.stream)
        return out, ev

    def __iter__(self):
        it = iter(self.src)
        nxt = self._stage(next(it, None))
        while nxt is not None:
            cur, ev = nxt
            nxt = self._stage(next(it, None))          # the next copy overlaps this batch's step
            torch.cuda.current_stream(self.device).wait_event(ev)
            for t in cur:
                t.record_stream(torch.cuda.current_stream(self.device))
            yield cur
