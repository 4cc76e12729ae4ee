#!/usr/bin/env python3
"""Headline benchmark: GRU4Rec training steps at 1M items, dim 128,
seq_len <= 50, batch 4096, full-softmax logits (BASELINE.json configs[1]).

    python bench.py [--gpus N] [--steps K] [--warmup W]

metric: session-steps/sec (= batch rows × train_step calls per second, whole
job).  One step = one ``GRU4Rec_trainer.train_step(s, a, true_len)`` on the
MI355X (pack, gather, GRU fwd, logits + CE, backward, dense Adam over every
parameter, loss ``.item()``), inputs already resident in HBM.

Multi-GPU (torch.distributed.run, one rank per GPU, RCCL): weak scaling, each
rank trains its own 4096-row batch shard; the trunk is replicated (gradient
all-reduce), the output layer is sharded over ranks by item id (all-gather h,
LSE merge, reduce-scatter dh) — one optimizer step over the global batch
(see DESIGN.md §5).

Beside it, on rank 0 at N=1 only: the CPU oracle (the reference's PyTorch-CPU
math, oracle/) timed on a bounded sample of the same workload.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "ikea-recommender-system_amd"))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402
import torch  # noqa: E402

ITEMS, DIM, SEQ, BATCH = 1_000_000, 128, 50, 4096
FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: dense f32 MFMA (= f32 vector peak)
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--items", type=int, default=ITEMS)
    ap.add_argument("--dim", type=int, default=DIM)
    ap.add_argument("--seq", type=int, default=SEQ)
    ap.add_argument("--batch", type=int, default=BATCH)
    ap.add_argument("--cpu-batch", type=int, default=512)
    ap.add_argument("--cpu-steps", type=int, default=6)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-kernel-timing", action="store_true")
    ap.add_argument("--force-shard", action="store_true", help="item-sharded path even at world 1 (test)")
    return ap.parse_args()


def cpu_baseline(args):
    """The reference's per-step math on PyTorch-CPU (oracle/, restatement pinned
    to the reference's golden vectors) on a bounded sample: same item count,
    dims and seq_len, batch reduced to --cpu-batch rows."""
    from oracle.models import OracleSupervised
    from recommenders.data_utils.synthetic import SessionStream
    threads = torch.get_num_threads()
    B = args.cpu_batch
    orc = OracleSupervised(kind="gru4rec", hidden_dim=args.dim, embedding_dim=args.dim, gru_layers=1,
                           train_pad_embed=True, use_packed_seq=True, learning_rate=0.01, item_num=args.items,
                           state_size=args.seq, action_dim=args.items)
    st = SessionStream(args.items, args.seq, B * (args.cpu_steps + 1), seed=2)
    b = st.batch(0, B)
    orc.step(b[0], b[1], b[4])  # warm-up
    t0 = time.perf_counter()
    for i in range(1, args.cpu_steps + 1):
        b = st.batch(i, B)
        orc.step(b[0], b[1], b[4])
    dt = time.perf_counter() - t0
    return {"value": round(B * args.cpu_steps / dt, 2), "unit": "session-steps/sec", "cores": threads,
            "kind": "port",
            "sample": (f"oracle (reference PyTorch-CPU math) GRU4Rec {args.items} items dim{args.dim} "
                       f"L<={args.seq}, batch {B}, {args.cpu_steps} timed steps after 1 warm-up, "
                       f"{threads} threads, {dt:.1f} s")}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 or args.force_shard:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    from recommenders.data_utils.synthetic import SessionStream
    from recommenders.hip.timing import KernelTimer, timing
    from recommenders.models.GRU4Rec.model import GRU4Rec_trainer

    dev = torch.device("cuda", local)
    B, L, N, E = args.batch, args.seq, args.items, args.dim
    nsteps = args.warmup + args.steps
    # synthetic session stream (seeded per rank: each rank owns its batch shard)
    st = SessionStream(N, L, B * nsteps, seed=2 + rank)
    batches = []
    tok = []
    for i in range(nsteps):
        s, a, r, sn, ln, nln, e = st.batch(i, B)
        batches.append((s.to(dev), a.to(dev), ln.to(dev)))
        tok.append(int(ln.sum()))
    tr = GRU4Rec_trainer(hidden_dim=E, embedding_dim=E, gru_layers=1, train_pad_embed=True, use_packed_seq=True,
                         learning_rate=0.01, item_num=N, state_size=L, action_dim=N, device=dev,
                         shard_items=world > 1 or args.force_shard)
    tr.set_train()
    for i in range(args.warmup):
        tr.train_step(*batches[i])
    timer = KernelTimer()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    losses = []
    if args.no_kernel_timing:
        for i in range(args.warmup, nsteps):
            losses.append(tr.train_step(*batches[i]))
    else:
        with timing(timer):
            for i in range(args.warmup, nsteps):
                losses.append(tr.train_step(*batches[i]))
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        dt = float(t)
    if not all(np.isfinite(losses)):
        raise RuntimeError(f"non-finite loss {losses}")
    if rank != 0:
        if torch.distributed.is_initialized():
            torch.distributed.destroy_process_group()
        return
    ms = dt / args.steps * 1e3
    value = B * args.steps * world / dt
    flops_head = 2.0 * B * N * E  # one (B × E)·(E × A) contraction
    kern = {}
    roof = None
    if not args.no_kernel_timing:
        el = timer.elapsed_ms()
        kern = {k: round(float(np.mean(v)), 4) for k, v in el.items()}
        heads = {k: kern[k] for k in ("head_fwd", "head_dh", "head_dw_adam") if k in kern}
        dom = max(heads, key=heads.get)
        ach = flops_head / (heads[dom] * 1e-3) / 1e12
        traffic = None
        pmc = os.path.join(HERE, "profiles", "pmc_traffic.json")
        if os.path.exists(pmc):
            traffic = json.load(open(pmc)).get(dom)
        roof = {"bound": "mfma", "kernel": dom, "achieved": round(ach, 2), "peak": FP32_MFMA_PEAK_TFLOPS,
                "unit": "TFLOP/s", "frac": round(ach / FP32_MFMA_PEAK_TFLOPS, 4), "traffic": traffic,
                "flops_per_launch": flops_head}
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args)
    line = {
        "metric": "session-steps/sec at 1M items, dim128, batch 4096; HR@20/NDCG@20 parity",
        "value": round(value, 2), "unit": "session-steps/sec", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32", "data": "synthetic (seeded Zipf session stream, random-init weights)",
        "config": {"workload": f"GRU4Rec {N} items, dim{E}, seq_len<={L}, batch {B}/GPU, full-softmax logits",
                   "global_batch": B * world, "seq_len": L, "items": N, "dim": E,
                   "parallelism": (f"dp{world} trunk + {world}-way item-sharded head (RCCL)" if world > 1
                                   else "single"),
                   "tokens_per_batch": int(np.mean(tok))},
        "roofline": roof, "cpu_baseline": cpu, "kernel_ms": kern,
        "loss_first_last": [round(losses[0], 5), round(losses[-1], 5)],
    }
    print(json.dumps(line), flush=True)
    if torch.distributed.is_initialized():
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
