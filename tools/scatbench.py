"""Time rg_scatter_rows (deterministic sort-based scatter) at the step's shapes."""
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "ikea-recommender-system_amd"))
import torch
from recommenders.hip import call, stream_ptr

dev = "cuda"
for n_max, n, E, rows in ((204800, 90000, 128, 1000001), (6144, 6144, 128, 1000000), (6144, 6144, 1, 1000000),
                          (204800, 90000, 256, 1000001)):
    g = torch.Generator(device=dev).manual_seed(0)
    # Zipf-like ids: many repeats of a few popular items
    u = torch.rand(n_max, device=dev, generator=g)
    ids = (u ** 6 * rows).to(torch.int32)
    src = torch.randn(n_max, E, device=dev)
    G = torch.zeros(rows, E, device=dev)
    tags = torch.zeros(rows, dtype=torch.int32, device=dev)
    nt = torch.tensor([n], dtype=torch.int32, device=dev)
    nb = call("rg_scatter_rows_work_bytes", n_max, E, rows)
    work = torch.empty(nb, dtype=torch.uint8, device=dev)
    f = lambda: call("rg_scatter_rows", ids.data_ptr(), src.data_ptr(), E, E, nt.data_ptr(), n_max, -1, G.data_ptr(),
                     rows, tags.data_ptr(), 1, 0, work.data_ptr(), nb, stream_ptr())
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        f()
    e1.record()
    torch.cuda.synchronize()
    print(f"n_max {n_max} n {n} E {E}: {e0.elapsed_time(e1) / 20 * 1e3:.1f} us", flush=True)
