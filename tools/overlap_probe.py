"""Would the fused head's passes gain from running side by side?  Pass 2 of
one workspace (stored logits, dW + Adam: VALU-bound) and pass 1 of another
(split-bf16 logits: MFMA-bound) at C2 shapes, first one after the other on one
stream, then concurrently on two streams; prints both wall times (ms per
pair).  A feasibility probe for pipelining step t's pass 2 with step t+1's
pass 1 over item halves.

    python tools/overlap_probe.py [--iters 5]
"""
import argparse
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "ikea-recommender-system_amd"))
import torch  # noqa: E402

from recommenders.hip import call, host_floats, stream_ptr  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--B", type=int, default=4096)
ap.add_argument("--A", type=int, default=1_000_000)
ap.add_argument("--H", type=int, default=128)
ap.add_argument("--iters", type=int, default=5)
a = ap.parse_args()
B, A, H, terms = a.B, a.A, a.H, 6
dev = "cuda"
u8 = lambda n: torch.empty(int(n), dtype=torch.uint8, device=dev)  # noqa: E731
hb, wb = call("rg_head_plane_bytes", B, H), call("rg_head_plane_bytes", A, H)
nrb = -(-B // call("rg_flash_rows_per_block", H))
ns = -(-min(max(1, 256 // nrb), -(-A // 32)) // 8) * 8
adam6 = host_floats([0.1, 0.999, 0.001, 0.0316, 1e-8, -1e-9])


def make(seed):
    g = torch.Generator(device=dev).manual_seed(seed)
    s = dict(h=torch.randn(B, H, device=dev, generator=g) * 0.3, W=torch.randn(A, H, device=dev, generator=g) * 0.05,
             b=torch.randn(A, device=dev, generator=g) * 0.05, tgt=torch.randint(0, A, (B,), device=dev, generator=g))
    s.update(mW=torch.zeros_like(s["W"]), vW=torch.zeros_like(s["W"]), mb=torch.zeros_like(s["b"]),
             vb=torch.zeros_like(s["b"]), Hk=u8(hb), Hr=u8(hb), Wk=u8(wb), Wr=u8(wb),
             bp=torch.empty((A + 31) // 32 * 32, device=dev), pm=torch.empty(ns, B, device=dev),
             pl=torch.empty(ns, B, device=dev), pO=torch.empty(ns, H, B, device=dev), lse=torch.empty(B, device=dev),
             zt=torch.empty(B, device=dev), rows=torch.empty(B, 2, device=dev),
             dww=u8(max(call("rg_flash_dw_work_bytes", B, A, H), 16)),
             zs=torch.empty(call("rg_flash_zs_bytes", B, A) // 4, device=dev))
    st = stream_ptr()
    call("rg_head_planes", s["h"].data_ptr(), B, H, s["Hk"].data_ptr(), s["Hr"].data_ptr(), None, None, st)
    call("rg_head_planes", s["W"].data_ptr(), A, H, s["Wk"].data_ptr(), s["Wr"].data_ptr(), s["b"].data_ptr(),
         s["bp"].data_ptr(), st)
    return s


def pass1(s):
    call("rg_flash_fwd_top", s["Hk"].data_ptr(), s["Wk"].data_ptr(), s["Wr"].data_ptr(), s["bp"].data_ptr(), B, A, H,
         terms, ns, s["pm"].data_ptr(), s["pl"].data_ptr(), s["pO"].data_ptr(), None, None, None, s["zs"].data_ptr(),
         stream_ptr())


def prep2(s):
    st = stream_ptr()
    call("rg_flash_lse", s["pm"].data_ptr(), s["pl"].data_ptr(), ns, s["h"].data_ptr(), s["W"].data_ptr(),
         s["b"].data_ptr(), s["tgt"].data_ptr(), 0, A, A, B, H, s["lse"].data_ptr(), s["zt"].data_ptr(), st)
    call("rg_flash_rows", s["lse"].data_ptr(), s["tgt"].data_ptr(), 0, A, B, s["rows"].data_ptr(), st)


def pass2(s):
    call("rg_flash_dw_adam_planes", s["Hk"].data_ptr(), s["Hr"].data_ptr(), s["Wk"].data_ptr(), s["bp"].data_ptr(),
         s["rows"].data_ptr(), 1.0 / B, B, A, H, terms, s["W"].data_ptr(), s["mW"].data_ptr(), s["vW"].data_ptr(),
         s["b"].data_ptr(), s["mb"].data_ptr(), s["vb"].data_ptr(), adam6, None, None, s["Wk"].data_ptr(),
         s["Wr"].data_ptr(), s["bp"].data_ptr(), s["dww"].data_ptr(), s["dww"].numel(), s["zs"].data_ptr(),
         stream_ptr())


X, Y = make(1), make(2)
for s in (X, Y):   # logits stored and row records made once; pass 2 re-reads the same stored logits
    pass1(s)
    prep2(s)
torch.cuda.synchronize()
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
for it in range(a.iters):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    pass2(X)
    pass1(Y)
    torch.cuda.synchronize()
    seq = (time.perf_counter() - t0) * 1e3
    t0 = time.perf_counter()
    with torch.cuda.stream(s1):
        pass2(X)
    with torch.cuda.stream(s2):
        pass1(Y)
    torch.cuda.synchronize()
    con = (time.perf_counter() - t0) * 1e3
    print(f"iter {it}: pass 2 then pass 1 {seq:.3f} ms, side by side {con:.3f} ms ({con / seq:.3f}x)", flush=True)
