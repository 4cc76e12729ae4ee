"""Max |error| against fp64 of the fused head's outputs (lse, CE, dh, dW, db)
per precision next to the native fp32 head, at two operand scales (the
test's, and a trained-like one with logits of several units).  Prints one
table per scale: python tools/prec_err.py"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "ikea-recommender-system_amd"))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
import torch  # noqa: E402

from test_gpu_flash_head import fp64_reference, run_flash, run_native  # noqa: E402

TERMS = {"f32x9": 9, "f32x6": 6, "f32x6d3": 636}
dev = "cuda"
for (B, A, HF, hs, ws, seed) in [(512, 30000, 128, 0.5, 0.1, 5), (512, 30000, 128, 0.9, 0.6, 6),
                                 (1024, 100000, 128, 0.9, 0.3, 7)]:
    g = torch.Generator().manual_seed(seed)
    h = torch.tanh(torch.randn(B, HF, generator=g) * 2) * hs
    W = torch.randn(A, HF, generator=g) * ws
    b = torch.randn(A, generator=g) * ws
    tgt = torch.randint(0, A, (B,), generator=g)
    r = fp64_reference(h, W, b, tgt)
    r["ce"] = r["lse"] - r["zt"]
    hd, Wd, bd, td = h.to(dev), W.to(dev), b.to(dev), tgt.to(dev)
    errs = {"f32": run_native(hd, Wd, bd, td)}
    for p, t in TERMS.items():
        o = run_flash(hd, Wd, bd, td, t, 16)
        o["ce"] = o["lse"] - o["zt"]
        errs[p] = o
    keys = ("lse", "ce", "dh", "dW", "db")
    print(f"B {B} A {A} HF {HF} |h|<{hs} W~{ws}  max|Z| {float(r['Z'].abs().max()):.2f}")
    for p, o in errs.items():
        print(f"  {p:8s} " + "  ".join(f"{k} {float((o[k] - r[k]).abs().max()):.3e}" for k in keys))
    # relative-to-native ratios
    for p in TERMS:
        print(f"  {p:8s} /native " + "  ".join(
            f"{k} {float((errs[p][k] - r[k]).abs().max()) / max(float((errs['f32'][k] - r[k]).abs().max()), 1e-30):.2f}"
            for k in keys))
