"""Optional per-kernel HIP-event timing for bench.py (off by default).

Events are recorded on torch's current stream, which is the stream every
kernel of the step is launched on (recommenders.hip.stream_ptr)."""
from __future__ import annotations

import contextlib

import torch

_active = None


class KernelTimer:
    def __init__(self):
        self.pairs = {}

    def elapsed_ms(self):
        torch.cuda.synchronize()
        return {k: [a.elapsed_time(b) for a, b in v] for k, v in self.pairs.items()}


@contextlib.contextmanager
def timing(timer):
    global _active
    prev, _active = _active, timer
    try:
        yield timer
    finally:
        _active = prev


@contextlib.contextmanager
def region(name):
    if _active is None:
        yield
        return
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    a.record()
    try:
        yield
    finally:
        b.record()
        _active.pairs.setdefault(name, []).append((a, b))
