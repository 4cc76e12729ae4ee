"""Does a stream created with a CU mask (hipExtStreamCreateWithCUMask, every
CU enabled) get a hardware queue of its own?  The process's other streams
share GPU_MAX_HW_QUEUES (4) queues in an order that depends on how many
streams exist (tools/hwqueues.py); a CU mask is a property of the
queue, so a masked stream cannot share one.  Keeps one stream busy with
GEMMs and times a tiny kernel on another, as tools/hwqueues.py.

    python tools/hwqueues_cumask.py [--n 8]
"""
import argparse
import ctypes
import time

import torch

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=8)
a = ap.parse_args()
dev = torch.device("cuda", 0)
torch.zeros(1, device=dev)
hip = ctypes.CDLL("libamdhip64.so")
ncu = torch.cuda.get_device_properties(dev).multi_processor_count
words = (ncu + 31) // 32
mask = (ctypes.c_uint32 * words)(*([0xFFFFFFFF] * words))


def masked_stream():
    h = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(h), ctypes.c_uint32(words), mask)
    assert rc == 0, rc
    return torch.cuda.ExternalStream(h.value, device=dev)


named = [("default", torch.cuda.default_stream(dev))]
named += [(f"pool{i}", torch.cuda.Stream()) for i in range(a.n)]
named += [(f"masked{i}", masked_stream()) for i in range(3)]
big = torch.rand(8192, 8192, device=dev)
y = torch.zeros(16, device=dev)
print(f"{ncu} CUs, mask of {words} words", flush=True)
for bname, busy in [named[0], named[1], named[-3], named[-2]]:
    for name, s in named:
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
        print(f"busy {bname}, probe {name}: done after {(t1 - t0) * 1e3:7.2f} ms of {(t2 - t0) * 1e3:7.2f}"
              f"{'  SHARED' if t1 - t0 > 0.5 * (t2 - t0) else ''}", flush=True)
