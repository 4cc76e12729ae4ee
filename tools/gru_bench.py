"""Time the persistent GRU recurrences (csrc/gru.hip) at config C5's trunk
shape: H 256, L 100, B 8192, session lengths 1 + Geometric(2/L) clipped at L
(SURVEY §8d stream), and at C2's H 128 for reference.  Prints per-launch ms
and the fp32-MFMA fraction (2·tokens·3H·H flops per direction)."""
import sys, os, json
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "ikea-recommender-system_amd"))
import numpy as np
import torch
import recommenders.hip as C

dev = "cuda"
PEAK_F32_MFMA = 157.3e12


def run(H, B, L, reps=10):
    rng = np.random.default_rng(0)
    lens = np.minimum(1 + rng.geometric(2.0 / L, B) - 1, L).clip(1, L)
    lens_t = torch.from_numpy(lens.astype(np.int64)).to(dev)
    T = int(lens.sum())
    perm = torch.empty(B, dtype=torch.int32, device=dev)
    ls = torch.empty(B, dtype=torch.int32, device=dev)
    offs = torch.empty(B + 1, dtype=torch.int32, device=dev)
    st = C.stream_ptr()
    C.call("rg_pack", lens_t.data_ptr(), B, L, 0, perm.data_ptr(), ls.data_ptr(), offs.data_ptr(), st)
    k = 1 / H ** 0.5
    Whh = (torch.rand(3 * H, H, device=dev) * 2 - 1) * k
    bhh = (torch.rand(3 * H, device=dev) * 2 - 1) * k
    Gi = torch.randn(T, 3 * H, device=dev) * 0.5
    hout = torch.zeros(B, H, device=dev)
    saved = torch.zeros(5, T, H, device=dev)
    dGi = torch.zeros(T, 3 * H, device=dev)
    dGh = torch.zeros(T, 3 * H, device=dev)
    dh = torch.randn(B, H, device=dev)
    wide = H > 128
    work = torch.zeros(C.call("rg_gru_wide_work_bytes", H) // 4 if wide else 1, device=dev)

    def fwd():
        if wide:
            C.call("rg_gru_fwd_wide", Gi.data_ptr(), Whh.data_ptr(), bhh.data_ptr(), perm.data_ptr(), ls.data_ptr(),
                   offs.data_ptr(), B, H, hout.data_ptr(), H, 0, saved.data_ptr(), T * H, work.data_ptr(), st)
        else:
            C.call("rg_gru_fwd", Gi.data_ptr(), Whh.data_ptr(), bhh.data_ptr(), perm.data_ptr(), ls.data_ptr(),
                   offs.data_ptr(), B, H, hout.data_ptr(), H, 0, saved.data_ptr(), T * H, st)

    def bwd():
        if wide:
            C.call("rg_gru_bwd_wide", saved.data_ptr(), T * H, Whh.data_ptr(), perm.data_ptr(), ls.data_ptr(),
                   offs.data_ptr(), B, H, dh.data_ptr(), H, 0, dGi.data_ptr(), dGh.data_ptr(), work.data_ptr(), st)
        else:
            C.call("rg_gru_bwd", saved.data_ptr(), T * H, Whh.data_ptr(), perm.data_ptr(), ls.data_ptr(),
                   offs.data_ptr(), B, H, dh.data_ptr(), H, 0, dGi.data_ptr(), dGh.data_ptr(), st)

    out = {"H": H, "B": B, "L": L, "tokens": T}
    for name, f in (("fwd", fwd), ("bwd", bwd)):
        f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            f()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        fl = 2.0 * T * 3 * H * H
        out[name + "_ms"] = round(ms, 3)
        out[name + "_mfma_frac"] = round(fl / (ms * 1e-3) / PEAK_F32_MFMA, 3)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    run(256, 8192, 100)
    run(256, 4096, 50)
    run(128, 4096, 50)
