"""Time the fused split-bf16 head stages at C2 shapes (B 4096, A 1M, H 128):
W planes, pass 1 (rg_flash_fwd), the dh combine and pass 2 with Adam
(rg_flash_dw_adam).  --zs: pass 1 also stores the logits and pass 2 reads
them (the stored-logit head).  IKEA_REC_HIP_LIB selects a diagnostic variant
build."""
import argparse
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "ikea-recommender-system_amd"))
import torch  # noqa: E402

from recommenders.hip import call, host_floats, stream_ptr  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--B", type=int, default=4096)
ap.add_argument("--A", type=int, default=1_000_000)
ap.add_argument("--H", type=int, default=128)
ap.add_argument("--iters", type=int, default=4)
ap.add_argument("--terms", type=int, nargs="+", default=[6, 9])
ap.add_argument("--zs", action="store_true")
a = ap.parse_args()
B, A, H = a.B, a.A, a.H
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)
h = torch.randn(B, H, device=dev, generator=g) * 0.3
W = torch.randn(A, H, device=dev, generator=g) * 0.05
bias = torch.randn(A, device=dev, generator=g) * 0.05
mW, vW = torch.zeros_like(W), torch.zeros_like(W)
mb, vb = torch.zeros_like(bias), torch.zeros_like(bias)
tgt = torch.randint(0, A, (B,), device=dev, generator=g)
u8 = lambda n: torch.empty(int(n), dtype=torch.uint8, device=dev)  # noqa: E731
hb, wb = call("rg_head_plane_bytes", B, H), call("rg_head_plane_bytes", A, H)
Hk, Hr, Wk, Wr = u8(hb), u8(hb), u8(wb), u8(wb)
bp = torch.empty((A + 31) // 32 * 32, device=dev)
nrb = -(-B // call("rg_flash_rows_per_block", H))
ns = -(-min(max(1, 256 // nrb), -(-A // 32)) // 8) * 8
pm, pl = torch.empty(ns, B, device=dev), torch.empty(ns, B, device=dev)
pO = torch.empty(ns, H, B, device=dev)
lse, zt = torch.empty(B, device=dev), torch.empty(B, device=dev)
rows = torch.empty(B, 2, device=dev)
dh = torch.empty(B, H, device=dev)
adam6 = host_floats([0.1, 0.999, 0.001, 0.0316, 1e-8, -1e-9])  # tiny step: W stays put
st = stream_ptr()
gs = 1.0 / B
dwb = call("rg_flash_dw_work_bytes", B, A, H)
dww = u8(max(dwb, 16))
zs = torch.empty(call("rg_flash_zs_bytes", B, A) // 4, device=dev) if a.zs else None
zp = None if zs is None else zs.data_ptr()
call("rg_head_planes", h.data_ptr(), B, H, Hk.data_ptr(), Hr.data_ptr(), None, None, st)
fl = 2.0 * B * A * H
for terms in a.terms:
    stages = {
        "planes_W": lambda: call("rg_head_planes", W.data_ptr(), A, H, Wk.data_ptr(), Wr.data_ptr(), bias.data_ptr(),
                                 bp.data_ptr(), st),
        "pass1": lambda: call("rg_flash_fwd_top", Hk.data_ptr(), Wk.data_ptr(), Wr.data_ptr(), bp.data_ptr(), B, A,
                              H, terms, ns, pm.data_ptr(), pl.data_ptr(), pO.data_ptr(), None, None, None, zp, st),
        "combine": lambda: (call("rg_flash_lse", pm.data_ptr(), pl.data_ptr(), ns, h.data_ptr(), W.data_ptr(),
                                 bias.data_ptr(), tgt.data_ptr(), 0, A, A, B, H, lse.data_ptr(), zt.data_ptr(), st),
                            call("rg_flash_rows", lse.data_ptr(), tgt.data_ptr(), 0, A, B, rows.data_ptr(), st),
                            call("rg_flash_dh", pm.data_ptr(), pO.data_ptr(), rows.data_ptr(), ns, W.data_ptr(),
                                 gs, B, H, dh.data_ptr(), st)),
        # as the trainers run it: the updated W also leaves as the next pass 1's planes
        "pass2": lambda: call("rg_flash_dw_adam_planes", Hk.data_ptr(), Hr.data_ptr(), Wk.data_ptr(), bp.data_ptr(),
                              rows.data_ptr(), gs, B, A, H, terms, W.data_ptr(), mW.data_ptr(), vW.data_ptr(),
                              bias.data_ptr(), mb.data_ptr(), vb.data_ptr(), adam6, None, None, Wk.data_ptr(),
                              Wr.data_ptr(), bp.data_ptr(), dww.data_ptr(), dwb, zp, st),
    }
    for name, fn in stages.items():
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.iters
        extra = ""
        if name in ("pass1", "pass2"):
            nprod = {6: 12, 9: 18, 636: 9 if name == "pass1" else 12}[terms]   # plane products per pass
            if a.zs and name == "pass2":
                nprod //= 2   # (the S contraction is read, not recomputed)
            extra = f"  {nprod * fl / ms / 1e9:7.1f} TFLOP/s bf16 MFMA ({nprod * fl / ms / 1e9 / 2500:.3f} of peak)"
        print(f"terms {terms} {name:8s} {ms:8.3f} ms{extra}", flush=True)
