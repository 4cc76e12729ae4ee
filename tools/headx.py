"""Time the full-softmax head forward at C2 shapes (B 4096, A 1M, H 128):
native fp32 (rg_head_fwd) vs split-bf16 (rg_head_fwd_x, 9 / 6 terms)."""
import argparse
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "ikea-recommender-system_amd"))
import torch  # noqa: E402

from recommenders.hip import call, load_library, stream_ptr  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--B", type=int, default=4096)
ap.add_argument("--A", type=int, default=1_000_000)
ap.add_argument("--H", type=int, default=128)
ap.add_argument("--iters", type=int, default=5)
a = ap.parse_args()
B, A, H = a.B, a.A, a.H
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)
h = torch.randn(B, H, device=dev, generator=g) * 0.3
W = torch.randn(A, H, device=dev, generator=g) * 0.05
bias = torch.randn(A, device=dev, generator=g) * 0.05
ldz = (B + 3) // 4 * 4
pb = load_library().rg_partial_block()
nJ = (A + pb - 1) // pb
ZT = torch.empty(A, ldz, device=dev)
pm = torch.empty(nJ, B, device=dev)
ps = torch.empty(nJ, B, device=dev)
pa = torch.empty(nJ, B, dtype=torch.int32, device=dev)
work = torch.empty(call("rg_head_work_bytes", B, H), dtype=torch.uint8, device=dev)
st = stream_ptr()
fl = 2.0 * B * A * H
for name, terms in (("f32", 0), ("f32x9", 9), ("f32x6", 6)):
    def run():
        if terms == 0:
            call("rg_head_fwd", h.data_ptr(), W.data_ptr(), bias.data_ptr(), B, A, H, ZT.data_ptr(), ldz,
                 pm.data_ptr(), ps.data_ptr(), pa.data_ptr(), 1, st)
        else:
            call("rg_head_fwd_x", h.data_ptr(), W.data_ptr(), bias.data_ptr(), B, A, H, terms, ZT.data_ptr(), ldz,
                 pm.data_ptr(), ps.data_ptr(), pa.data_ptr(), 1, work.data_ptr(), st)
    run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        run()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.iters
    print(f"head fwd {name:6s} {ms:8.3f} ms  {fl / ms / 1e9:7.1f} TFLOP/s (fp32-equivalent)", flush=True)
