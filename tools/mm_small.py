"""Calibration for the sampled logits shape (B 4096 x S 2048, HF 128): hipBLASLt/rocBLAS
GEMMs through torch — fp32 (4096x128)@(128x2048) and the bf16 GEMM with the split-bf16
work (K = 6 x 128 = 768) — times with HIP events over back-to-back launches."""
import torch
B, S, HF = 4096, 2048, 128
for name, dt, K in (("fp32 K=128", torch.float32, HF), ("bf16 K=768", torch.bfloat16, 6 * HF),
                    ("bf16 K=128", torch.bfloat16, HF)):
    a = torch.randn(B, K, device="cuda", dtype=dt)
    b = torch.randn(K, S, device="cuda", dtype=dt)
    for _ in range(5):
        c = a @ b
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        c = a @ b
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 50 * 1e3
    print(f"{name}: {us:.2f} us, {2 * B * S * K / us / 1e6:.1f} TFLOP/s", flush=True)
