"""Host time of each dist.Comm collective (one rank, nccl backend) while a long
kernel runs on another stream, and its device latency alone: does the call
return at once, or wait for the device?  RANK / WORLD_SIZE / MASTER_* from the env.

    RG_COMM=native|torch python tools/commlat.py
"""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "ikea-recommender-system_amd"))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

torch.cuda.set_device(0)
dist.init_process_group("nccl")
from recommenders.hip.dist import Comm  # noqa: E402

c = Comm()
dev = torch.device("cuda", 0)
x = torch.rand(4096, 128, device=dev)
y = torch.empty_like(x)
big = torch.rand(8192, 8192, device=dev)
side = torch.cuda.Stream()
ops = {
    "all_gather": lambda: c.all_gather(y.view(-1), x.view(-1)),
    "reduce_scatter": lambda: c.reduce_scatter(y.view(-1), x.view(-1)),
    "all_reduce": lambda: c.all_reduce(y),
    "all_to_all": lambda: c.all_to_all(y, x, [4096], [4096]),
    "plain_kernel": lambda: y.add_(1.0),   # (control: no collective)
}
main2 = torch.cuda.Stream()   # a non-default stream as the "main" one (--main-stream)
use_main2 = "--main-stream" in sys.argv
for name, op in ops.items():
  with torch.cuda.stream(main2 if use_main2 else torch.cuda.current_stream()):
      for _ in range(3):
          op()
      torch.cuda.synchronize()
      with torch.cuda.stream(side):
          for _ in range(20):
              big = big @ big * 1e-4
      t0 = time.perf_counter()
      op()
      t1 = time.perf_counter()
      done = torch.cuda.Event()
      done.record()              # on the current (main) stream, behind the collective
      done.synchronize()
      tm = time.perf_counter()   # the main stream's collective finished
      torch.cuda.synchronize()
      t2 = time.perf_counter()
      # device-side latency alone: 50 back-to-back calls
      torch.cuda.synchronize()
      t3 = time.perf_counter()
      for _ in range(50):
          op()
      torch.cuda.synchronize()
      t4 = time.perf_counter()
      print(f"{os.environ.get('RG_COMM', 'native'):6s} {'side-main' if use_main2 else 'null-main'} {name:15s} host call under a busy side stream "
            f"{(t1 - t0) * 1e3:8.3f} ms, done on its stream after {(tm - t0) * 1e3:8.3f} ms (side work "
            f"{(t2 - t0) * 1e3:7.2f} ms), alone {(t4 - t3) / 50 * 1e6:7.1f} us/call",
            flush=True)
dist.destroy_process_group()
