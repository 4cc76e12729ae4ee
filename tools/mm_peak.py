"""Practical bf16 MFMA ceiling on this box: torch.matmul (hipBLASLt) bf16 GEMMs."""
import torch
for n in (8192, 16384):
    a = torch.randn(n, n, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(n, n, device="cuda", dtype=torch.bfloat16)
    for _ in range(3):
        c = a @ b
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    it = 20 if n == 8192 else 5
    e0.record()
    for _ in range(it):
        c = a @ b
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / it
    tf = 2 * n ** 3 / ms / 1e9
    print(f"bf16 GEMM {n}^3: {ms:.3f} ms, {tf:.0f} TFLOP/s ({tf / 2500:.3f} of 2.5 PF)", flush=True)
