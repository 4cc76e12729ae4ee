"""North-star side run alone (bench.py's: GRU4Rec at C2 shapes with 2048
sampled negatives, kernel-exact events on the gather and the sampled logits),
for same-box A/B of variant libraries (IKEA_REC_HIP_LIB):

    python tools/nstime.py [--steps 30] [--warmup 5] [--reps 2]

Prints one line per repetition: gather / sampled_fwd ms and the HBM-roofline
fraction as bench.py's north_star_target computes it."""
import argparse
import importlib.util
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
bench = importlib.util.module_from_spec(spec)
spec.loader.exec_module(bench)
import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=30)
ap.add_argument("--warmup", type=int, default=5)
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--config", default="c2s")
a = ap.parse_args()
sys.argv = [sys.argv[0]]
args = bench.parse()
from recommenders.data_utils.synthetic import SessionStream  # noqa: E402
dev = torch.device("cuda", 0)
B, L, N, E = args.batch, args.seq, args.items, args.dim
n = a.warmup + a.steps
st = SessionStream(N, L, B * n, seed=2)
batches, tok = [], []
for i in range(n):
    b = st.batch(i, B)
    batches.append(bench.pinned(b))
    tok.append(int(b[4].sum()))
T = float(np.mean(tok[a.warmup:]))
tr = bench.make_trainer(a.config, args, dev, False)
tr.set_train()
lib = os.environ.get("IKEA_REC_HIP_LIB", "tree") or "tree"
for r in range(a.reps):
    _, _, k2, _ = bench.timed_run(tr, batches, a.warmup if r == 0 else 0, a.steps, 1, True, "c2")
    t = bench.target_step(k2, T, B, args.negatives, E, E, 1, 6)
    print(f"lib={lib} rep {r}: gather {t['gather_ms'] * 1e3:.2f} us  sampled_fwd {t['sampled_fwd_ms'] * 1e3:.2f} us  "
          f"frac {t['frac']:.4f}", flush=True)
