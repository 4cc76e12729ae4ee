"""Host cost of the item-sharded step's route computation (dist.host_routes:
owner counts of the host batch + one gloo all-gather), one rank, C2 shapes."""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "ikea-recommender-system_amd"))
os.environ.setdefault("RANK", "0")
os.environ.setdefault("WORLD_SIZE", "1")
os.environ.setdefault("LOCAL_RANK", "0")
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29541")
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from recommenders.data_utils.synthetic import SessionStream  # noqa: E402
from recommenders.hip.dist import host_routes, owner_counts  # noqa: E402
from recommenders.models.GRU4Rec.model import GRU4Rec_trainer  # noqa: E402

torch.cuda.set_device(0)
dist.init_process_group("nccl")
N, L, B = 1_000_000, 50, 4096
tr = GRU4Rec_trainer(hidden_dim=128, embedding_dim=128, gru_layers=1, train_pad_embed=True, use_packed_seq=True,
                     learning_rate=0.01, item_num=N, state_size=L, action_dim=N, device="cuda", shard_items=True)
st = SessionStream(N, L, B * 12, seed=2)
bs = [st.batch(i, B) for i in range(12)]
net = tr.gru_model
comm = net.comm
t = time.perf_counter()
for b in bs:
    owner_counts(b[0].numpy(), b[4].numpy(), L, True, net.trunk.N1, comm.world)
print(f"owner_counts {(time.perf_counter() - t) / len(bs) * 1e3:.2f} ms")
t = time.perf_counter()
for b in bs:
    host_routes(comm, net.trunk, [(b[0], b[4])])
print(f"host_routes {(time.perf_counter() - t) / len(bs) * 1e3:.2f} ms")
for b in bs[:3]:
    tr.train_step(b[0], b[1], b[4])
torch.cuda.synchronize()
t = time.perf_counter()
for b in bs[3:]:
    tr.train_step(b[0], b[1], b[4])
torch.cuda.synchronize()
print(f"train_step {(time.perf_counter() - t) / (len(bs) - 3) * 1e3:.2f} ms")
dist.destroy_process_group()
