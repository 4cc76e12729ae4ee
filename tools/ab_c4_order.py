"""Same-box A/B of the SMORL (C4) step order: qlearn.PASS2_BEFORE_TARGET True
(the supervised head's pass 2 launched right after pass 1) vs False (after
the double-Q target's join, the round-5 order).  One trainer, alternating
arms, timed like bench.py.

    python tools/ab_c4_order.py [--reps 3] [--steps 20] [--config c4]
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
from recommenders.hip import qlearn  # noqa: E402

ap = argparse.ArgumentParser()
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
tr = bench.make_trainer("c4", args, dev, False)
tr.set_train()
for r in range(a.reps):
    for arm in (False, True):
        qlearn.PASS2_BEFORE_TARGET = arm
        dt, _, _, ps = bench.timed_run(tr, batches, 5, a.steps, 1, False, "c4")
        print(f"PASS2_BEFORE_TARGET={arm} rep {r}: {B * a.steps / dt:.1f} session-steps/s, "
              f"{dt / a.steps * 1e3:.3f} ms/step (median {np.median(ps) * 1e3:.3f})", flush=True)
