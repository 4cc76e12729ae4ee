"""Phase stamps of the one-launch sampled logits (k_sampled_logits, HKP path)
at the north-star shapes.  Needs the diagnostic library:
    tools/build_variant.sh sfstamp sampled.hip -DSF_STAMP
    IKEA_REC_HIP_LIB=variants/lib_sfstamp.so python tools/sfstamp.py
Per wave: 0 start, 1 after the ingest barrier, 2/3/4/5 after the epilogue of
chunk 0/1/2/3 (s_memrealtime, 100 MHz); 6/7 s_memtime at start / end (clock)."""
import argparse
import ctypes as C
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "ikea-recommender-system_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from recommenders.hip import call, load_library, stream_ptr  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--B", type=int, default=4096)
ap.add_argument("--S", type=int, default=2048)
ap.add_argument("--A", type=int, default=1_000_000)
ap.add_argument("--HF", type=int, default=128)
ap.add_argument("--iters", type=int, default=200)
ap.add_argument("--wp", choices=["none", "cold", "warm"], default="none",
                help="draw = 2: W planes / biases pre-gathered; cold = written before the 256 MB of other traffic")
a = ap.parse_args()
dev = "cuda"
B, S, A, HF = a.B, a.S, a.A, a.HF
g = torch.Generator(device=dev).manual_seed(0)
h = torch.randn(B, HF, device=dev, generator=g) * 0.3
W = torch.randn(A, HF, device=dev, generator=g) * 0.05
bias = torch.randn(A, device=dev, generator=g) * 0.05
neg = torch.zeros(S, dtype=torch.int32, device=dev)
nT = call("rg_sampled_nparts", B, S, 6)
pm = torch.empty(nT, B, device=dev)
ps = torch.empty(nT, B, device=dev)
Wg = torch.empty(S, HF, device=dev)
bg = torch.empty(S, device=dev)
Z = torch.empty(B, S, device=dev)
hk = torch.empty(call("rg_head_plane_bytes", B, HF), dtype=torch.uint8, device=dev)
st = stream_ptr()
call("rg_head_planes", h.data_ptr(), B, HF, hk.data_ptr(), None, None, None, st)
junk = torch.empty(64 << 20, device=dev)
lib = load_library()
nwg = (S // 256) * (B // 128)
n = nwg * 8 * 8
buf = np.zeros(n, dtype=np.uint64)
rows = []
wp_src = torch.randint(0, 1 << 14, (S * HF * 3,), dtype=torch.int16, device=dev)
wp = torch.empty_like(wp_src)
bg_src = torch.randn(S, device=dev)
for it in range(a.iters):
    if a.wp == "cold":
        wp.copy_(wp_src)
        bg.copy_(bg_src)
    junk.add_(1.0)   # 256 MB of other traffic between launches, as in a step
    if a.wp == "warm":
        wp.copy_(wp_src)
        bg.copy_(bg_src)
    pre = a.wp != "none"
    call("rg_sampled_logits", h.data_ptr(), W.data_ptr(), bias.data_ptr(), neg.data_ptr(), 2 if pre else 1, 7, it + 1,
         A, B, S, HF, 6, Z.data_ptr(), S, pm.data_ptr(), ps.data_ptr(), Wg.data_ptr(), bg.data_ptr(), hk.data_ptr(),
         wp.data_ptr() if pre else None, st)
    if it >= a.iters - 20:
        torch.cuda.synchronize()
        assert lib.rg_sf_stamp_read(buf.ctypes.data_as(C.c_void_p), C.c_int64(n)) == 0
        rows.append(buf.reshape(nwg * 8, 8).astype(np.int64).copy())
ph = []
for r in rows:
    t = r[:, :6]
    t0 = t[:, 0].min()
    clk = (r[:, 7] - r[:, 6]) / ((t[:, 5] - t[:, 0]) * 10e-9) / 1e9   # GHz
    ph.append([np.median(t[:, 0] - t0), (t[:, 0] - t0).max(), np.median(t[:, 1] - t[:, 0]),
               np.median(t[:, 2] - t[:, 1]), np.median(t[:, 3] - t[:, 2]), np.median(t[:, 4] - t[:, 3]),
               np.median(t[:, 5] - t[:, 4]), (t[:, 5].max() - t0), np.median(clk)])
ph = np.median(np.asarray(ph, dtype=np.float64), axis=0)
names = ["start skew (median)", "start skew (max)", "ingest (start -> barrier)", "chunk 0 + MFMA 1 + epi 0",
         "MFMA 2 + epi 1", "MFMA 3 + epi 2", "epi 3", "total (first start -> last end)"]
for nm, v in zip(names, ph[:8]):
    print(f"{nm:34s} {v * 10e-3:7.2f} us")
print(f"{'in-kernel clock':34s} {ph[8]:7.2f} GHz")
