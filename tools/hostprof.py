"""Host enqueue time vs GPU time per training step: is a config's step
launch-bound?  Builds bench.py's trainer for --config, runs --warmup steps,
then --steps steps timing each train_step call on the host (no sync inside)
and the whole run's wall time with one sync at the end.  A host time per step
close to the wall time per step means the GPU waits for launches.

    python tools/hostprof.py --config c3 [--steps 200] [--warmup 300]
"""
import argparse
import importlib.util
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
bench = importlib.util.module_from_spec(spec)
spec.loader.exec_module(bench)
import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c3")
ap.add_argument("--steps", type=int, default=200)
ap.add_argument("--warmup", type=int, default=300)
ap.add_argument("--nbatch", type=int, default=50)
ap.add_argument("--nosync", action="store_true",
                help="the loss read-back does not wait (zeros): the host's pure enqueue cost per step")
a = ap.parse_args()
sys.argv = [sys.argv[0], "--config", a.config]
args = bench.parse()
from recommenders.data_utils.synthetic import SessionStream  # noqa: E402
dev = torch.device("cuda", 0)
if a.nosync:
    from recommenders.hip import hostsync  # noqa: E402
    hostsync.HostScalars.get = lambda self: [0.0] * self._n
B, L, N = args.batch, args.seq, args.items
st = SessionStream(N, L, B * a.nbatch, seed=2)
args.item_counts = st.item_counts()
batches = [bench.pinned(st.batch(i, B)) for i in range(a.nbatch)]
tr = bench.make_trainer(a.config, args, dev, False)
tr.set_train()
for i in range(a.warmup):
    tr.train_step(*bench.step_args(a.config, batches[i % a.nbatch]))
torch.cuda.synchronize()
host = []
t0 = time.perf_counter()
for i in range(a.steps):
    h0 = time.perf_counter()
    tr.train_step(*bench.step_args(a.config, batches[i % a.nbatch]))
    host.append(time.perf_counter() - h0)
t_enq = time.perf_counter() - t0
torch.cuda.synchronize()
wall = time.perf_counter() - t0
host.sort()
print(f"{a.config}{' (no loss wait)' if a.nosync else ''}: B {B}, {a.steps} steps after {a.warmup}: wall {wall / a.steps * 1e3:.3f} ms/step, "
      f"host enqueue {t_enq / a.steps * 1e3:.3f} ms/step (median call {host[len(host) // 2] * 1e3:.3f}, "
      f"p90 {host[int(len(host) * 0.9)] * 1e3:.3f}), GPU queue drained {(wall - t_enq) * 1e3:.1f} ms after the "
      f"last call", flush=True)
