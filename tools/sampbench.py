"""Time the sampled-softmax forward standalone (north-star shapes: B 4096,
S 2048, HF 128 / 256) with HIP events over back-to-back launches; prints µs,
TFLOP/s and the Zᵀ write rate per precision."""
import argparse
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "ikea-recommender-system_amd"))
import torch  # noqa: E402

from recommenders.hip import call, stream_ptr  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--B", type=int, default=4096)
ap.add_argument("--S", type=int, default=2048)
ap.add_argument("--A", type=int, default=1_000_000)
ap.add_argument("--HF", type=int, nargs="+", default=[128, 256])
ap.add_argument("--iters", type=int, default=50)
ap.add_argument("--prec", nargs="+", default=["f32", "f32x9", "f32x6"])
ap.add_argument("--fused", action="store_true", help="also time the one-launch rg_sampled_logits (HF <= 128)")
ap.add_argument("--hot", action="store_true", help="fused: the same draw every launch (W rows cache-resident)")
ap.add_argument("--planes", action="store_true", help="fused: h as bf16 K-planes (as the GRU forward leaves them)")
a = ap.parse_args()
dev = "cuda"
for HF in a.HF:
    B, S, A = a.B, a.S, a.A
    g = torch.Generator(device=dev).manual_seed(0)
    h = torch.randn(B, HF, device=dev, generator=g) * 0.3
    W = torch.randn(A, HF, device=dev, generator=g) * 0.05
    bias = torch.randn(A, device=dev, generator=g) * 0.05
    neg = torch.randint(0, A, (S,), device=dev, generator=g, dtype=torch.int32)
    ldz = (B + 3) // 4 * 4
    nT = call("rg_sampled_nparts", B, S, 9)  # the larger count
    ZT = torch.empty(S, ldz, device=dev)
    pm = torch.empty(nT, B, device=dev)
    ps = torch.empty(nT, B, device=dev)
    Wg = torch.empty(S, HF, device=dev)
    bg = torch.empty(S, device=dev)
    work = torch.empty(call("rg_sampled_work_bytes", B, S, HF), dtype=torch.uint8, device=dev)
    st = stream_ptr()
    fl = 2.0 * B * S * HF
    for prec in a.prec:
        it = [0]

        def run():
            it[0] += 1  # a fresh draw every launch: the negatives' rows come from HBM as in a step
            if prec == "f32":
                call("rg_sampled_fwd", h.data_ptr(), W.data_ptr(), bias.data_ptr(), neg.data_ptr(), B, S, HF,
                     ZT.data_ptr(), ldz, pm.data_ptr(), ps.data_ptr(), Wg.data_ptr(), bg.data_ptr(), st)
            else:
                call("rg_sampled_fwd_x", h.data_ptr(), W.data_ptr(), bias.data_ptr(), neg.data_ptr(), 1, 7, it[0], A, B,
                     S, HF, 9 if prec == "f32x9" else 6, ZT.data_ptr(), ldz, pm.data_ptr(), ps.data_ptr(),
                     Wg.data_ptr(), bg.data_ptr(), work.data_ptr(), st)
        for _ in range(3):
            run()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(a.iters):
            run()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / a.iters * 1e3
        print(f"HF {HF} {prec:6s} {us:8.2f} us  {fl / us / 1e6:7.1f} TFLOP/s  Z write {B * S * 4 / us / 1e3:6.0f} GB/s",
              flush=True)
        if a.fused and prec != "f32" and HF <= 256:
            ldzr = (S + 3) // 4 * 4
            Zr = torch.empty(B, ldzr, device=dev)
            terms = 9 if prec == "f32x9" else 6
            hk = None
            if a.planes and HF <= 128:
                hk = torch.empty(call("rg_head_plane_bytes", B, HF), dtype=torch.uint8, device=dev)
                call("rg_head_planes", h.data_ptr(), B, HF, hk.data_ptr(), None, None, None, st)

            def fz():
                it[0] += 0 if a.hot else 1
                call("rg_sampled_logits", h.data_ptr(), W.data_ptr(), bias.data_ptr(), neg.data_ptr(), 1, 7, it[0], A,
                     B, S, HF, terms, Zr.data_ptr(), ldzr, pm.data_ptr(), ps.data_ptr(), Wg.data_ptr(), bg.data_ptr(),
                     None if hk is None else hk.data_ptr(), None, st)
            for _ in range(3):
                fz()
            torch.cuda.synchronize()
            e0.record()
            for _ in range(a.iters):
                fz()
            e1.record()
            torch.cuda.synchronize()
            uf = e0.elapsed_time(e1) / a.iters * 1e3
            print(f"   fused one-launch {uf:8.2f} us  {fl / uf / 1e6:7.1f} TFLOP/s  "
                  f"({terms * fl / uf / 1e6 / 2500:.3f} of bf16 peak), Z write {B * S * 4 / uf / 1e3:6.0f} GB/s",
                  flush=True)
