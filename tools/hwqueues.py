"""Which torch streams share a hardware queue (GPU_MAX_HW_QUEUES, HIP's
default 4 per process)?  Streams on one queue run in order even when they
are independent.  Keeps stream 0 of the list (or the default stream) busy
with GEMMs and times a tiny kernel on every other one.

    python tools/hwqueues.py [--n 8]
"""
import argparse
import time

import torch

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=8)
a = ap.parse_args()
dev = torch.device("cuda", 0)
streams = [torch.cuda.default_stream(dev)] + [torch.cuda.Stream() for _ in range(a.n)]
big = torch.rand(8192, 8192, device=dev)
y = torch.zeros(16, device=dev)
for bi, busy in enumerate(streams[:3]):
    for k, s in enumerate(streams):
        if s is busy:
            continue
        torch.cuda.synchronize()
        with torch.cuda.stream(busy):
            for _ in range(10):
                big = big @ big * 1e-4
        t0 = time.perf_counter()
        with torch.cuda.stream(s):
            y.add_(1.0)
            e = torch.cuda.Event()
            e.record()
        e.synchronize()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"busy stream {bi} ({'default' if bi == 0 else 'created'}), probe stream {k}: done after "
              f"{(t1 - t0) * 1e3:7.2f} ms of {(t2 - t0) * 1e3:7.2f}{'  SHARED' if t1 - t0 > 0.5 * (t2 - t0) else ''}",
              flush=True)
