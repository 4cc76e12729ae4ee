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
BF16_MFMA_PEAK_TFLOPS = 2500.0  # dense bf16 MFMA (no sparsity)
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
    ap.add_argument("--config", choices=["c2", "c3"], default="c2",
                    help="c2: headline GRU4Rec full softmax; c3: BidirGRU4Rec with sampled softmax")
    ap.add_argument("--negatives", type=int, default=2048)
    # f32x6 (default): fp32 operands split exactly into three bf16 planes, the six
    # plane products above 2^-24 relative on bf16 MFMAs, fp32 accumulation;
    # tests/test_gpu_flash_head.py::test_flash_error_is_fp32_class measures it
    # against fp64 next to the native fp32-MFMA path ("f32")
    ap.add_argument("--precision", choices=["f32", "f32x9", "f32x6"], default="f32x6",
                    help="head GEMM arithmetic (hip/engine.py SPLIT_TERMS): native fp32 MFMA or split-bf16")
    ap.add_argument("--no-target", action="store_true", help="skip the north-star gather+sampled-logits side run")
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


def make_trainer(cfg, args, dev, shard):
    from recommenders.models.BidirGRU4Rec.model import BidirGRU4Rec_trainer
    from recommenders.models.GRU4Rec.model import GRU4Rec_trainer
    N, L, E = args.items, args.seq, args.dim
    common = dict(hidden_dim=E, embedding_dim=E, gru_layers=1, train_pad_embed=True, use_packed_seq=True,
                  learning_rate=0.01, item_num=N, state_size=L, action_dim=N, device=dev)
    if cfg == "c2":
        return GRU4Rec_trainer(shard_items=shard, matmul_precision=args.precision, **common)
    if cfg == "c2s":   # GRU4Rec at C2 shapes with the sampled head (north-star target step)
        return GRU4Rec_trainer(n_negatives=args.negatives, matmul_precision=args.precision, **common)
    if cfg == "c3":
        return BidirGRU4Rec_trainer(dropout=0.0, n_negatives=args.negatives, matmul_precision=args.precision,
                                    **common)
    raise ValueError(cfg)


def timed_run(tr, batches, warmup, steps, world, kernel_timing):
    """W untimed steps, then K steps between barrier + synchronize; max over ranks."""
    from recommenders.hip.timing import KernelTimer, timing
    for i in range(warmup):
        tr.train_step(*batches[i])
    timer = KernelTimer()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    losses = []
    if kernel_timing:
        with timing(timer):
            for i in range(warmup, warmup + steps):
                losses.append(tr.train_step(*batches[i]))
    else:
        for i in range(warmup, warmup + steps):
            losses.append(tr.train_step(*batches[i]))
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=torch.cuda.current_device())
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        dt = float(t)
    if not all(np.isfinite(losses)):
        raise RuntimeError(f"non-finite loss {losses}")
    kern = {}
    if kernel_timing:
        kern = {k: round(float(np.mean(v)), 4) for k, v in timer.elapsed_ms().items()}
    return dt, losses, kern


def gather_bytes(T, E):
    # per token: int64 id read, fp32 table row read, packed row write, int32 token-id write
    return T * (8 + 2 * 4 * E + 4)


def sampled_fwd_bytes(B, S, HF):
    # h read, negative ids, gathered W rows + bias read, Zᵀ write, (max, Σexp) partials, Wg/bg write
    nT = (S + 127) // 128
    return B * HF * 4 + S * 4 + 2 * S * (HF + 1) * 4 + B * S * 4 + nT * B * 8


def target_step(kern, T, B, S, E, HF, n_gather):
    """North-star target: embedding gather + sampled logits (fwd) against the
    HBM roofline, with the logits' flop rate beside it."""
    if "gather" not in kern or "sampled_fwd" not in kern:
        return None
    tg, ts = kern["gather"] * n_gather, kern["sampled_fwd"]
    by = n_gather * gather_bytes(T, E) + sampled_fwd_bytes(B, S, HF)
    gbs = by / ((tg + ts) * 1e-3) / 1e9
    fl = 2.0 * B * S * HF
    return {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(gbs / HBM_PEAK_GBS, 4), "bytes_per_step": int(by), "ms": round(tg + ts, 4),
            "gather_ms": round(tg, 4), "gather_GBs": round(n_gather * gather_bytes(T, E) / (tg * 1e-3) / 1e9, 1),
            "sampled_fwd_ms": round(ts, 4), "sampled_fwd_TFLOPs": round(fl / (ts * 1e-3) / 1e12, 2),
            "sampled_fwd_mfma_frac": round(fl / (ts * 1e-3) / 1e12 / FP32_MFMA_PEAK_TFLOPS, 4)}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    shard = (world > 1 or args.force_shard) and args.config == "c2"
    if world > 1 or args.force_shard:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    if world > 1 and args.config != "c2":
        raise SystemExit("multi-GPU bench runs the C2 headline workload only")
    from recommenders.data_utils.synthetic import SessionStream

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
    T = float(np.mean(tok[args.warmup:]))
    tr = make_trainer(args.config, args, dev, shard)
    tr.set_train()
    dt, losses, kern = timed_run(tr, batches, args.warmup, args.steps, world, not args.no_kernel_timing)
    if rank != 0:
        if torch.distributed.is_initialized():
            torch.distributed.destroy_process_group()
        return
    ms = dt / args.steps * 1e3
    value = B * args.steps * world / dt
    roof = None
    target = None
    HF = E * (2 if args.config == "c3" else 1)
    if args.config == "c2":
        flops_head = 2.0 * B * N * E  # one (B × E)·(E × A) contraction
        terms = {"f32x9": 9, "f32x6": 6}.get(args.precision, 0)
        if kern:
            heads = {k: kern[k] for k in ("head_fwd", "head_dh", "head_dw_adam") if k in kern}
            dom = max(heads, key=heads.get)
            t = heads[dom] * 1e-3
            traffic = None
            pmc = os.path.join(HERE, "profiles", "pmc_traffic.json")
            if os.path.exists(pmc):
                traffic = json.load(open(pmc)).get(f"{dom}:{args.precision}" if terms else dom)
            if terms:
                # fused split-bf16 head (csrc/head_flash.hip): pass 1 (head_fwd: Z and the softmax half of
                # dh) and pass 2 (head_dw_adam: Z recomputed, dW) each run two contractions, every fp32
                # product as `terms` exact bf16 plane products on v_mfma_f32_32x32x16_bf16
                ex = 2 * terms * flops_head if dom in ("head_fwd", "head_dw_adam") else 0.0
                alg = {"head_fwd": 2, "head_dw_adam": 1}.get(dom, 0) * flops_head
                ach = ex / t / 1e12
                roof = {"bound": "mfma", "kernel": dom, "achieved": round(ach, 2), "peak": BF16_MFMA_PEAK_TFLOPS,
                        "unit": "TFLOP/s", "frac": round(ach / BF16_MFMA_PEAK_TFLOPS, 4), "traffic": traffic,
                        "flops_per_launch": ex,
                        "mfma": f"bf16 MFMA, fp32 operands split exactly into 3 bf16 planes, {terms} plane products",
                        "algorithmic_fp32_TFLOPs": round(alg / t / 1e12, 2)}
            else:
                ach = flops_head / t / 1e12
                roof = {"bound": "mfma", "kernel": dom, "achieved": round(ach, 2), "peak": FP32_MFMA_PEAK_TFLOPS,
                        "unit": "TFLOP/s", "frac": round(ach / FP32_MFMA_PEAK_TFLOPS, 4), "traffic": traffic,
                        "flops_per_launch": flops_head}
        if world == 1 and not args.no_target and kern:
            # north-star target step measured on GRU4Rec at C2
            # shapes with the sampled head: a short side run, own trainer
            del tr
            torch.cuda.empty_cache()
            tr2 = make_trainer("c2s", args, dev, False)
            tr2.set_train()
            _, _, k2 = timed_run(tr2, batches, min(2, args.warmup), min(5, args.steps), 1, True)
            target = target_step(k2, T, B, args.negatives, E, E, 1)
            if target is not None:
                target["workload"] = f"GRU4Rec {N} items dim{E} batch {B}, {args.negatives} sampled negatives"
            del tr2
    else:
        target = target_step(kern, T, B, args.negatives, E, HF, 2)
        roof = dict(target) if target else None
        if roof:
            roof["kernel"] = "gather + sampled_fwd"
            # PMC HBM bytes of the same kernels per step (tools/pmc_c3.sh), committed under profiles/
            pmc = os.path.join(HERE, "profiles", "pmc_traffic.json")
            roof["traffic"] = None
            if os.path.exists(pmc) and (B, args.negatives, HF, args.precision) == (4096, 2048, 256, "f32x6"):
                roof["traffic"] = json.load(open(pmc)).get("c3:gather+sampled_fwd")
    cpu = None
    if world == 1 and not args.no_cpu_baseline and args.config == "c2":
        cpu = cpu_baseline(args)
    if args.config == "c2":
        metric = "session-steps/sec at 1M items, dim128, batch 4096; HR@20/NDCG@20 parity"
        workload = f"GRU4Rec {N} items, dim{E}, seq_len<={L}, batch {B}/GPU, full-softmax logits"
    else:
        metric = "session-steps/sec, BidirGRU4Rec 1M items, dim128, batch 4096, 2048 sampled negatives"
        workload = (f"BidirGRU4Rec {N} items, dim{E}, seq_len<={L}, batch {B}, {args.negatives} shared uniform "
                    f"negatives (sampled softmax), dropout 0")
    line = {
        "metric": metric,
        "value": round(value, 2), "unit": "session-steps/sec", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32", "matmul_precision": args.precision,
        "data": "synthetic (seeded Zipf session stream, random-init weights)",
        "config": {"workload": workload,
                   "global_batch": B * world, "seq_len": L, "items": N, "dim": E,
                   "parallelism": (f"dp{world} trunk + {world}-way item-sharded head (RCCL)" if world > 1
                                   else "single"),
                   "tokens_per_batch": int(T)},
        "roofline": roof, "cpu_baseline": cpu, "north_star_target": target, "kernel_ms": kern,
        "loss_first_last": [round(losses[0], 5), round(losses[-1], 5)],
    }
    print(json.dumps(line), flush=True)
    if torch.distributed.is_initialized():
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
