"""Training steps only, for a step-only rocprofv3 kernel summary (no trainer
construction): builds bench.py's trainer for --config, runs --warmup steps,
launches a 1-element marker kernel (k_f32_to_f16), runs --steps steps, and a
second marker.  tools/kwindow.py then keeps the kernels between the markers.

    rocprofv3 --kernel-trace --output-format csv -d OUT -o x -- python3 tools/stepprof.py --config c5
    python tools/kwindow.py OUT/**/x_kernel_trace.csv > stats.csv
"""
import argparse
import importlib.util
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
bench = importlib.util.module_from_spec(spec)
spec.loader.exec_module(bench)
import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c5")
ap.add_argument("--steps", type=int, default=4)
ap.add_argument("--warmup", type=int, default=2)
ap.add_argument("--nbatch", type=int, default=0, help="distinct batches, cycled (0: one per step)")
ap.add_argument("--shard", action="store_true",
                help="item-sharded trainer over a one-rank process group (RANK / WORLD_SIZE / MASTER_* from the env)")
a = ap.parse_args()
sys.argv = [sys.argv[0], "--config", "c2" if a.config == "c2s" else a.config]
args = bench.parse()
if a.config == "c5":
    args.items, args.dim, args.seq, args.batch = 5_000_000, 256, 100, 8192
from recommenders.data_utils.synthetic import SessionStream  # noqa: E402
from recommenders.hip import call, stream_ptr  # noqa: E402
dev = torch.device("cuda", 0)
if a.shard:
    torch.cuda.set_device(0)
    torch.distributed.init_process_group("nccl")
B, L, N = args.batch, args.seq, args.items
n = a.warmup + a.steps
nb = min(n, a.nbatch) if a.nbatch > 0 else n
st = SessionStream(N, L, B * nb, seed=2)
args.item_counts = st.item_counts()
batches = [bench.pinned(st.batch(i, B)) for i in range(nb)]
tr = bench.make_trainer(a.config, args, dev, a.shard)
tr.set_train()
x = torch.zeros(4, device=dev)
y = torch.zeros(8, dtype=torch.float16, device=dev)


def marker():
    torch.cuda.synchronize()
    call("rg_f32_to_f16", x.data_ptr(), 1, y.data_ptr(), stream_ptr())
    torch.cuda.synchronize()


for i in range(a.warmup):
    tr.train_step(*bench.step_args(a.config, batches[i % nb]))
marker()
for i in range(a.warmup, n):
    tr.train_step(*bench.step_args(a.config, batches[i % nb]))
marker()
print(f"stepprof: {a.config} {a.steps} steps between the markers", flush=True)
if a.shard:
    torch.distributed.destroy_process_group()
