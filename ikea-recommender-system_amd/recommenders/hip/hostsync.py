"""The step's scalar results read back without waiting for the rest of the step.

The reference's ``train_step`` returns its losses as Python floats
(GRU4Rec/model.py:155 ``.item()``), which synchronises the whole step.  Here
the losses (and the step's error flags) are copied to pinned host memory by
one non-blocking D2H on the launch stream right where they are final — before
the backward, the head's pass 2 and the Adam sweeps are queued behind them —
and ``train_step`` waits only for that copy.  The host then queues the next
step while the GPU still runs this one's backward, so the step boundary costs
no GPU idle time; anything that reads parameters afterwards is ordered behind
the update on the same streams (and the head's side stream is joined by its
parameter properties), exactly as before."""
from __future__ import annotations

import torch


class HostScalars:
    def __init__(self):
        self._buf = None
        self._ev = None
        self._keep = None
        self._n = 0

    def capture(self, *tensors):
        """Enqueue the D2H of the first element of every tensor (float64 on the
        host: exact for fp32 / fp64 losses and int32 flags)."""
        dev = tensors[0].device
        vals = torch.cat([t.reshape(-1)[:1].to(torch.float64) for t in tensors])
        n = vals.numel()
        if self._buf is None or self._buf.numel() < n:
            self._buf = torch.empty(n, dtype=torch.float64, pin_memory=True)
            self._ev = torch.cuda.Event()
        self._buf[:n].copy_(vals, non_blocking=True)
        self._ev.record(torch.cuda.current_stream(dev))
        self._keep = vals   # the device source stays alive until the copy ran
        self._n = n

    def get(self):
        """The captured values as Python floats (waits for the copy only)."""
        self._ev.synchronize()
        self._keep = None
        return [float(x) for x in self._buf[:self._n].tolist()]
