"""Same-box A/B of the trunk GEMMs' arithmetic (Trunk.gemm_terms: 0 = the fp32
MFMA kernels, 6 = split-bf16 rg_gemm_x6 / rg_wgrad_x6) on one trainer per
config, alternating arms, timed like bench.py (pinned batches, H2D inside).

    python tools/ab_trunk_gemm.py [--configs c2 c3] [--reps 3] [--steps 20]
"""
import argparse
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "ikea-recommender-system_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from recommenders.data_utils.synthetic import SessionStream  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--configs", nargs="+", default=["c2", "c3"])
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--steps", type=int, default=20)
a = ap.parse_args()
sys.argv = [sys.argv[0]]
args = bench.parse()
dev = torch.device("cuda", 0)
B, N, L = args.batch, args.items, args.seq
st = SessionStream(N, L, B * (a.steps + 6), seed=2)
args.item_counts = st.item_counts()
batches = [bench.pinned(st.batch(i, B)) for i in range(a.steps + 5)]
for cfg in a.configs:
    tr = bench.make_trainer(cfg, args, dev, False)
    tr.set_train()
    nets = [getattr(tr, n) for n in ("gru_model", "SMORL_1", "SMORL_2") if hasattr(tr, n)]
    for r in range(a.reps):
        for terms in (0, 6):
            for n in nets:
                n.trunk.gemm_terms = terms
            dt, _, _, ps = bench.timed_run(tr, batches, 5, a.steps, 1, False, cfg)
            print(f"{cfg} gemm_terms={terms} rep {r}: {B * a.steps / dt:.1f} session-steps/s, "
                  f"{dt / a.steps * 1e3:.3f} ms/step (median {np.median(ps) * 1e3:.3f})", flush=True)
    del tr
    torch.cuda.empty_cache()
