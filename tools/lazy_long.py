"""Catch-up Adam at steady state: a config's trainer with catch-up Adam and
its eager twin (engine.LAZY_ADAM False) trained side by side for many steps
on the same batches (cycled), ms/step per window.  A sampled head's negative
row is re-read about every A/S steps, so its replay chain grows for the first
~A/S steps before the cost settles; a short bench run sees the early cost.

    python tools/lazy_long.py [--config c3] [--steps 800] [--window 100]
"""
import argparse
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "ikea-recommender-system_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
from recommenders.data_utils.synthetic import SessionStream  # noqa: E402
from recommenders.hip import engine  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c3")
ap.add_argument("--steps", type=int, default=800)
ap.add_argument("--window", type=int, default=100)
ap.add_argument("--nbatch", type=int, default=100)
ap.add_argument("--lazy-only", action="store_true", help="no eager twin (A/B of catch-up variants)")
ap.add_argument("--prefetch", type=int, default=1, help="engine.PREFETCH_NEGATIVES")
a = ap.parse_args()
sys.argv = [sys.argv[0]]
args = bench.parse()
dev = torch.device("cuda", 0)
B, N, L = args.batch, args.items, args.seq
st = SessionStream(N, L, B * a.nbatch, seed=2)
args.item_counts = st.item_counts()
batches = [bench.pinned(st.batch(i, B)) for i in range(a.nbatch)]
trs = {}
engine.PREFETCH_NEGATIVES = bool(a.prefetch)
modes = (True,) if a.lazy_only else (True, False)
for lazy in modes:
    engine.LAZY_ADAM = lazy
    trs[lazy] = bench.make_trainer(a.config, args, dev, False)
    trs[lazy].set_train()
engine.LAZY_ADAM = True
for w0 in range(0, a.steps, a.window):
    out = []
    for lazy in modes:
        tr = trs[lazy]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(w0, w0 + a.window):
            tr.train_step(*bench.step_args(a.config, batches[i % a.nbatch]))
        torch.cuda.synchronize()
        out.append(f"{'lazy' if lazy else 'eager'} {(time.perf_counter() - t0) / a.window * 1e3:.3f} ms/step")
    print(f"{a.config} steps {w0}-{w0 + a.window}: " + ", ".join(out), flush=True)
