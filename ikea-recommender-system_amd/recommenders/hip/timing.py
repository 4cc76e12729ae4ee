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
def region(name, exact=False):
    """Time the enclosed launches with a pair of events on the current
    stream.  exact=True (a region of ONE library kernel launched through
    RG_TLAUNCH, csrc/common.h): the library stamps the events at that
    kernel's own start / end (hipExtLaunchKernelGGL), so the duration excludes
    the event-record commands around it (which add microseconds to a
    microseconds-long kernel); if no such launch happened, the region falls
    back to the stream events."""
    if _active is None:
        yield
        return
    from . import call
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    a.record()
    if exact:
        b.record()   # (creates the event; the launch re-records both)
        call("rg_timing_events", a.cuda_event, b.cuda_event)
    try:
        yield
    finally:
        if exact:
            if call("rg_timing_events", None, None):   # not consumed: plain stream events
                b.record()
        else:
            b.record()
        _active.pairs.setdefault(name, []).append((a, b))
