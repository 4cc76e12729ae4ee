#!/usr/bin/env python3
"""Headline benchmark: GRU4Rec training steps at 1M items, dim 128,
seq_len <= 50, batch 4096, full-softmax logits (BASELINE.json configs[1]).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c4|c5]

metric: session-steps/sec (= batch rows × train_step calls per second, whole
job).  One step = one ``GRU4Rec_trainer.train_step(s, a, true_len)`` on the
MI355X: H2D of the batch (pinned host tensors, as a DataLoader with
pin_memory hands them over), pack, gather, GRU fwd, logits + CE, backward,
dense Adam over every parameter, loss ``.item()``.  Per-step wall times give
the median / p10 / p90 beside the mean.

After the timed steps the trained model is evaluated on a held-out batch
(device top-20, HR@20 / NDCG@20).  On rank 0 at N=1 the CPU leg times the
oracle (the reference's PyTorch-CPU math, oracle/) on a bounded sample of the
same workload, and scores a 256-row slice of the held-out batch with the
reference CPU math on the GPU-trained weights: its canonical top-20 lists and
HR@20 / NDCG@20 next to the device's ("hr_ndcg_parity").

Configs: c2 (headline), c3 (BidirGRU4Rec, 2048 sampled negatives),
c4 (SMORL: GRU4Rec trunk + supervised head + 3 Q heads, 3-reward double-Q),
c5 (IKEA scale: SMORL at 5M items, d256, seq_len <= 100, global batch 8192
split over the ranks, fp16 item table; fits one MI355X at ~279 GiB peak).
Multi-GPU (torch.distributed.run, one rank per GPU, RCCL), item tables
sharded over the ranks: c2 weak scaling (each rank trains its
own 4096-row batch shard); c4 / c5 strong scaling (their global batch, 4096 /
8192, split over the ranks: per_rank_batch).
"""
from __future__ import annotations

import argparse
import json
import os
import platform
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
EVAL_K = 20
# bf16 plane products per fp32 product: logits-only GEMMs (hip/engine.py LOGIT_TERMS) and the
# fused head's two passes (two contractions each; csrc/common.h RG_TERMS_*)
LOGIT_TERMS = {"f32x9": 9, "f32x6": 6, "f32x6d3": 6}
PASS_PRODUCTS = {"f32x9": {"head_fwd": 18, "head_dw_adam": 18}, "f32x6": {"head_fwd": 12, "head_dw_adam": 12},
                 "f32x6d3": {"head_fwd": 9, "head_dw_adam": 12}}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--items", type=int, default=ITEMS)
    ap.add_argument("--dim", type=int, default=DIM)
    ap.add_argument("--seq", type=int, default=SEQ)
    ap.add_argument("--batch", type=int, default=BATCH)
    # CPU leg: batch 4096 when the host has >= 96 GiB of RAM (the
    # reference materialises the 16.4 GB logits, their log_softmax and grads),
    # else 512; plus the C1 line (BASELINE configs[0], 100 steps)
    ap.add_argument("--cpu-batch", type=int, default=0, help="0: 4096 if host RAM >= 96 GiB else 512")
    ap.add_argument("--cpu-steps", type=int, default=0,
                    help="timed CPU steps after 1 warm-up (0: 3 for c2 at batch 4096 (BASELINE.md §3), 6 below; "
                         "2 for c3 / c4)")
    ap.add_argument("--c1-steps", type=int, default=100)
    ap.add_argument("--c1-warmup", type=int, default=10)
    ap.add_argument("--harness-steps", type=int, default=10,
                    help="C2: per-batch train_step + update_train_metrics as trainGRU.py:195-224 runs them")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-kernel-timing", action="store_true")
    ap.add_argument("--no-eval", action="store_true")
    ap.add_argument("--force-shard", action="store_true", help="item-sharded path even at world 1 (test)")
    ap.add_argument("--config", choices=["c2", "c3", "c4", "c5"], default="c2",
                    help="c2: headline GRU4Rec full softmax; c3: BidirGRU4Rec with sampled softmax; "
                         "c4: SMORL 3-reward double-Q; c5: IKEA-scale SMORL (5M items, d256, L<=100, global "
                         "batch 8192, fp16 item table)")
    ap.add_argument("--negatives", type=int, default=2048)
    # f32x6d3 (default): fp32 operands split exactly into three bf16 planes; the logits and dW
    # contractions keep the six plane products above 2^-24 relative (f32x6), pass 1's O = P·W
    # (-> dh) the three leading ones; fp32 accumulation on bf16 MFMAs.
    # tests/test_gpu_flash_head.py::test_flash_error_is_fp32_class holds every output (lse, CE,
    # dh, dW, db) within 4x of the native fp32-MFMA path ("f32") and 2x of the reference's CPU
    # fp32 path against fp64, and tests/test_gpu_model_parity.py holds it to the oracle's
    # top-20 / HR@20
    ap.add_argument("--precision", choices=["f32", "f32x9", "f32x6", "f32x6d3"], default="f32x6d3",
                    help="head GEMM arithmetic (hip/engine.py SPLIT_TERMS): native fp32 MFMA or split-bf16")
    ap.add_argument("--stored-logits", choices=["auto", "off"], default="auto",
                    help="fused head: pass 1 stores the logits for pass 2 (auto: where they fit, HF <= 128; "
                         "hip/engine.py ZSTORE_MAX_BYTES) or pass 2 recomputes them (off)")
    ap.add_argument("--no-target", action="store_true", help="skip the north-star gather+sampled-logits side run")
    ap.add_argument("--no-native-side", action="store_true", help="skip the native-f32 side run")
    ap.add_argument("--extra-steps", type=int, default=20,
                    help="C2 at N=1: timed steps of the short C3 / C4 side lines (configs_extra); 0 skips them")
    ap.add_argument("--settle", type=int, default=0,
                    help="untimed steps (batches cycled) before the warmup of this run's own line (C3 in a "
                         "child process: the catch-up Adam's steady state)")
    ap.add_argument("--extra-settle", type=int, default=1500,
                    help="untimed steps before the C3 side line's warmup (the catch-up Adam's steady state, "
                         "about 3·A/S steps for the sampled head's negatives)")
    return ap.parse_args()


def host_ram_gib():
    try:
        with open("/proc/meminfo") as f:
            for line in f:
                if line.startswith("MemTotal:"):
                    return round(int(line.split()[1]) / 2**20, 1)
    except OSError:
        pass
    return None


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


# ------------------------------------------------------------ CPU leg ------
def host_threads():
    """(threads the CPU leg uses, how they were found): the CPUs this process
    may run on (sched_getaffinity), capped by a cgroup CPU quota when one is
    set (a GPU box's share of a larger host)."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = max(1, int(-(-int(q) // int(per))))
    except (OSError, ValueError):
        pass
    n = min(aff, quota) if quota else aff
    return n, {"affinity_cpus": aff, "cgroup_cpu_quota": quota, "os_cpu_count": os.cpu_count()}


def _cpu_oracle(cfg, items, dim, seq, counts=None):
    from oracle.models import OracleSMORL, OracleSupervised
    common = dict(hidden_dim=dim, embedding_dim=dim, train_pad_embed=True, use_packed_seq=True, learning_rate=0.01,
                  item_num=items, state_size=seq, action_dim=items)
    if cfg in ("c2", "c1"):
        return OracleSupervised(kind="gru4rec", gru_layers=1, **common)
    if cfg == "c3":
        return OracleSupervised(kind="bidir", gru_layers=1, dropout=0.0, n_negatives=2048, **common)
    from recommenders.data_utils.synthetic import unpopular_items
    g = torch.Generator().manual_seed(7)
    div = torch.randn(items + 1, 64, generator=g) * 0.01
    return OracleSMORL(padding_pos="end", gamma=0.5, gru_layers=1, q_weights=[1.0, 1.0, 1.0], alpha=1.0,
                       div_embedding=div, unpopular_actions_set=unpopular_items(counts), topk_div=1,
                       topk_nov=1, nov_rew_sig=1.0, **common)


def _cpu_run(cfg, items, dim, seq, B, steps, seed, warmup=1, batches=None, counts=None):
    """Oracle steps of config ``cfg`` on the host: per-step seconds after
    ``warmup`` untimed steps, every step's loss, and the oracle.  ``batches``
    (with ``counts``): the GPU run's own host batches (the loss-parity leg);
    else a stream of its own (seed ``seed``)."""
    if batches is None:
        from recommenders.data_utils.synthetic import SessionStream
        st = SessionStream(items, seq, B * (steps + warmup), seed=seed)
        batches = [st.batch(i, B) for i in range(warmup + steps)]
        counts = st.item_counts()
    orc = _cpu_oracle(cfg, items, dim, seq, counts)

    def one(i):
        b = batches[i]
        return orc.step(*b) if cfg in ("c4", "c5") else orc.step(b[0], b[1], b[4])
    losses = [one(i) for i in range(warmup)]
    times = []
    for i in range(warmup, warmup + steps):
        t0 = time.perf_counter()
        losses.append(one(i))
        times.append(time.perf_counter() - t0)
    return times, losses, orc


CPU_NAMES = {"c2": "GRU4Rec", "c3": "BidirGRU4Rec (2048 shared sampled negatives, dropout 0)",
             "c4": "SMORL_trainer (sup head + 3 Q heads, 3 rewards, topk 1)",
             "c5": "SMORL_trainer (sup head + 3 Q heads, 3 rewards, topk 1; fp32 item table as the reference)"}
# C5's CPU sample ("Configs 4-5: CPU numbers ... single-process
# restatement at a reduced batch, stated"): the full 5M x 256 tables of both
# double-Q nets with their Adam moments and gradients (~200 GB) do not fit a
# few-minute host run, so the sample keeps dim 256 and seq_len 100 at a tenth
# of the items and batch 256
C5_CPU_ITEMS, C5_CPU_BATCH = 500_000, 256


def cpu_sample(args, cfg):
    """(items, batch, timed steps) of the CPU leg's bounded sample: C2 at batch
    4096 when the host RAM allows it (1 warm-up + 3 timed steps,
    BASELINE.md §3), else 512 (6 steps), C3 at batch 4096 and C4 at batch 512
    (3 timed steps each: one C4 step scores 1M items for the supervised head and
    the Q target), C5 at 500k items and batch 256 (dim 256, L <= 100, 2 timed
    steps; C5_CPU_ITEMS)."""
    ram = host_ram_gib()
    items = args.items
    if cfg == "c2":
        B = args.cpu_batch or (4096 if ram is not None and ram >= 96 else 512)
        steps = args.cpu_steps or (3 if B >= 4096 else 6)
    elif cfg == "c5":
        items = min(items, C5_CPU_ITEMS)
        B = args.cpu_batch or C5_CPU_BATCH
        steps = args.cpu_steps or 2
    else:
        B = args.cpu_batch or (4096 if cfg == "c3" else 512)
        steps = args.cpu_steps or 3
    return items, B, steps


def cpu_baseline(args, cfg="c2", batches=None, counts=None):
    """The reference's per-step math on PyTorch-CPU (oracle/, restatement pinned
    to the reference's golden vectors), timed on this host with every CPU the
    process may use (host_threads) on the bounded sample of ``cpu_sample`` —
    plus, with C2, the C1 line (BASELINE configs[0]: 10k items, dim32, L<=20,
    batch 64, --c1-warmup + --c1-steps steps).  ``batches``: the GPU run's
    first host batches at the sample's batch size (C2: the loss-parity leg
    trains the oracle on exactly what the GPU trainer saw); the oracle's
    per-step losses and final parameters come back in ``out["_oracle"]``."""
    threads, how = host_threads()
    torch.set_num_threads(threads)
    ram = host_ram_gib()
    items, B, steps = cpu_sample(args, cfg)
    if batches is not None:
        batches = batches[:1 + steps]
    times, losses, orc = _cpu_run(cfg, items, args.dim, args.seq, B, steps, 2, batches=batches, counts=counts)
    dt = float(np.sum(times))
    red = [x for x, full in (("items", items == args.items), ("batch", B == args.batch)) if not full]
    out = {"value": round(B * steps / dt, 2), "unit": "session-steps/sec", "cores": threads, "threads": how,
           "cpu_model": cpu_model(), "host_ram_gib": ram, "kind": "port", "batch": B, "items": items, "steps": steps,
           "median_ms_per_step": round(float(np.median(times)) * 1e3, 1),
           "sample": (f"oracle (reference PyTorch-CPU math) {CPU_NAMES[cfg]} {items} items dim{args.dim} "
                      f"L<={args.seq}, batch {B}{' (reduced ' + ' and '.join(red) + ')' if red else ''}, {steps} "
                      f"timed steps after 1 warm-up, torch.set_num_threads({threads}), {dt:.1f} s"
                      f"{'; on the first batches the GPU trainer saw' if batches is not None else ''}")}
    if batches is not None:
        out["_oracle"] = (losses, orc)
    if cfg == "c2" and args.c1_steps > 0:
        t1, _, _ = _cpu_run("c1", 10_000, 32, 20, 64, args.c1_steps, 1, warmup=args.c1_warmup)
        d1 = float(np.sum(t1))
        out["c1"] = {"value": round(64 * args.c1_steps / d1, 2), "unit": "session-steps/sec",
                     "ms_per_step": round(d1 / args.c1_steps * 1e3, 3), "steps": args.c1_steps,
                     "warmup": args.c1_warmup,
                     "workload": "GRU4Rec 10k items, dim32, seq_len<=20, batch 64 (BASELINE configs[0]), "
                                 f"{threads} threads"}
    return out


def cpu_eval_parity(net, ev, dev_idx, rows=256):
    """Reference CPU math (oracle.Net: nn.Embedding, packed nn.GRU, nn.Linear)
    on the GPU-trained weights for ``rows`` held-out rows: canonical top-20
    lists and HR@20 / NDCG@20 beside the device's."""
    from oracle import metrics as om
    from oracle.models import Net
    s, a, ln = ev[0][:rows], ev[1][:rows], ev[2][:rows]
    cpu = Net("gru4rec", net.item_num, net.action_dim, net.embedding_dim, net.hidden_dim)
    cpu.load_state_dict({k: v.detach().cpu() for k, v in net.state_dict().items()})
    cpu.eval()
    with torch.no_grad():
        z = cpu(s, ln).numpy()
    ref = om.canonical_topk_fast(z, EVAL_K)
    got = dev_idx[:rows]
    h_c, n_c = om.hits_from_lists(ref, a.numpy(), [EVAL_K])
    h_g, n_g = om.hits_from_lists(got, a.numpy(), [EVAL_K])
    same = int((ref == got).all(1).sum())
    return {"rows": rows, "top20_rows_identical": same, "hr20_cpu": h_c[0] / rows, "hr20_gpu": h_g[0] / rows,
            "ndcg20_cpu": round(n_c[0] / rows, 6), "ndcg20_gpu": round(n_g[0] / rows, 6),
            "note": "reference CPU math on the GPU-trained weights vs the device top-20 (canonical ties)"}


def gpu_parity_run(args, dev, batches):
    """The benched C2 trainer (same precision and stored-logit mode as the
    line) built afresh — the same seeds, so the reference's initial weights —
    and trained on ``batches``, the CPU leg's batches: per-step losses and the
    parameters after the last step (host copies)."""
    tr = make_trainer("c2", args, dev, False)
    apply_stored_logits(tr, args.stored_logits)
    tr.set_train()
    losses = [float(tr.train_step(*step_args("c2", b))) for b in batches]
    sd = {k: v.detach().cpu() for k, v in tr.gru_model.state_dict().items()}
    del tr
    torch.cuda.empty_cache()
    return losses, sd


# the trainer-vs-oracle bars of tests/test_gpu_supervised.py:33-43 / 79-100: losses within 1e-4;
# parameters within 2·lr everywhere and within 1e-4 for all but 0.1 % of the elements (Adam's first
# steps are sign-like, so a gradient that is zero up to summation order may move one element by 2·lr)
PARITY_LOSS_TOL, PARITY_PARAM_TOL, PARITY_PARAM_FRAC = 1e-4, 1e-4, 1e-3


def loss_parity(gpu_losses, cpu_losses, gpu_sd, cpu_sd, lr, batch):
    """GPU trainer vs the CPU oracle on the same batches, seeds and init:
    per-step |Δloss|, and per parameter tensor max |Δ| and the fraction of
    elements more than 1e-4 apart."""
    dl = [abs(a - b) for a, b in zip(gpu_losses, cpu_losses)]
    params = {}
    for k, v in gpu_sd.items():
        d = (v.float() - cpu_sd[k].float()).abs()
        params[k] = {"max_abs": float(d.max()), "frac_gt_1e-4": float((d > PARITY_PARAM_TOL).float().mean())}
    ok = (max(dl) <= PARITY_LOSS_TOL and
          all(p["max_abs"] <= 2 * lr + 1e-5 and p["frac_gt_1e-4"] < PARITY_PARAM_FRAC for p in params.values()))
    return {"steps": len(dl), "batch": batch, "gpu_losses": [round(x, 6) for x in gpu_losses],
            "cpu_losses": [round(x, 6) for x in cpu_losses], "max_abs_dloss": max(dl),
            "abs_dloss": [float(f"{x:.3g}") for x in dl], "params": params, "pass": bool(ok),
            "bars": {"loss": PARITY_LOSS_TOL, "param_max": 2 * lr + 1e-5, "param_tol": PARITY_PARAM_TOL,
                     "param_frac_over_tol": PARITY_PARAM_FRAC},
            "note": "the benched trainer (fresh, seeds 118 / 999) and the oracle (the reference's PyTorch-CPU "
                    "math) trained side by side on the same first batches of the bench stream at the same lr; "
                    "bars as tests/test_gpu_supervised.py"}


# ------------------------------------------------------------ GPU runs -----
def make_trainer(cfg, args, dev, shard):
    from recommenders.models.BidirGRU4Rec.model import BidirGRU4Rec_trainer
    from recommenders.models.GRU4Rec.model import GRU4Rec_trainer
    N, L, E = args.items, args.seq, args.dim
    common = dict(hidden_dim=E, embedding_dim=E, gru_layers=1, train_pad_embed=True, use_packed_seq=True,
                  learning_rate=0.01, item_num=N, state_size=L, action_dim=N, device=dev)
    if cfg == "c2":
        return GRU4Rec_trainer(shard_items=shard, matmul_precision=args.precision, **common)
    if cfg == "c2native":
        return GRU4Rec_trainer(matmul_precision="f32", **common)
    if cfg == "c2s":   # GRU4Rec at C2 shapes with the sampled head (north-star target step)
        return GRU4Rec_trainer(n_negatives=args.negatives, matmul_precision=args.precision, shard_items=shard,
                               **common)
    if cfg == "c3":
        return BidirGRU4Rec_trainer(dropout=0.0, n_negatives=args.negatives, matmul_precision=args.precision,
                                    **common)
    if cfg in ("c4", "c5"):
        from recommenders.data_utils.synthetic import unpopular_items
        from recommenders.models.SMORL.smorl_gru import SMORL_trainer
        common.pop("device")
        g = torch.Generator().manual_seed(7)
        div = torch.randn(N + 1, 64, generator=g) * 0.01     # frozen div table
        return SMORL_trainer(padding_pos="end", gamma=0.5, q_weights=[1.0, 1.0, 1.0], alpha=1.0, div_embedding=div,
                             unpopular_actions_set=unpopular_items(args.item_counts), topk_div=1, topk_nov=1,
                             device=dev, shard_items=shard, matmul_precision=args.precision,
                             fp16_embeddings=(cfg == "c5"), **common)
    raise ValueError(cfg)


def apply_stored_logits(tr, mode):
    """--stored-logits off: every fused full-softmax head recomputes its logits in pass 2."""
    if mode == "auto":
        return
    from recommenders.hip.engine import SoftmaxHead
    for name in ("gru_model", "SMORL_1", "SMORL_2", "DQN_1", "DQN_2"):
        for h in getattr(getattr(tr, name, None), "heads", {}).values():
            if isinstance(h, SoftmaxHead):
                h.zstore = False


def step_args(cfg, b):
    s, a, r, sn, ln, nln, e = b
    if cfg in ("c4", "c5"):
        return (s, a, r, sn, ln, nln, e)
    return (s, a, ln)


def top_scanned(tr, reset=False):
    """Rows whose exact top-k / argmax candidates overflowed the cap and were
    scanned whole (engine.SoftmaxHead.top_scanned), summed over the trainer's
    heads; reset zeroes the counters."""
    n = 0
    for name in ("gru_model", "SMORL_1", "SMORL_2", "DQN_1", "DQN_2"):
        for h in getattr(getattr(tr, name, None), "heads", {}).values():
            t = h.__dict__.get("_top_scanned")
            if t is not None:
                n += int(t.item())
                if reset:
                    t.zero_()
    return n


def timed_run(tr, batches, warmup, steps, world, kernel_timing, cfg):
    """W untimed steps, then K steps between barrier + synchronize; max over ranks.
    Batches are host (pinned) tensors: the H2D copy is inside every step."""
    from recommenders.hip.timing import KernelTimer, timing
    for i in range(warmup):
        tr.train_step(*step_args(cfg, batches[i]))
    top_scanned(tr, reset=True)
    timer = KernelTimer()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    losses, per_step = [], []
    ctx = timing(timer) if kernel_timing else None
    if ctx is not None:
        ctx.__enter__()
    try:
        t_prev = t0
        for i in range(warmup, warmup + steps):
            out = tr.train_step(*step_args(cfg, batches[i]))   # ends with .item(): a device sync
            t_now = time.perf_counter()
            per_step.append(t_now - t_prev)
            t_prev = t_now
            losses.append(out[0] if isinstance(out, tuple) else out)
    finally:
        if ctx is not None:
            ctx.__exit__(None, None, None)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        native = torch.distributed.get_backend() == "nccl"
        t = torch.tensor([dt], device=torch.cuda.current_device() if native else "cpu")
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        dt = float(t)
    if not all(np.isfinite(losses)):
        raise RuntimeError(f"non-finite loss {losses}")
    kern = {}
    if kernel_timing:
        kern = {k: round(float(np.mean(v)), 4) for k, v in timer.elapsed_ms().items()}
    return dt, losses, kern, per_step


def device_eval(net, ev):
    """Device top-20 and HR@20 / NDCG@20 of the trained model on the held-out batch."""
    from recommenders.hip.evalpath import eval_batch
    s, a, ln = ev
    net.eval()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = eval_batch(net, s, ln, a, K=EVAL_K, ks=[EVAL_K], want_loss=True)
    out = {"rows": int(len(a)), "hr20": float(r.hits[0].item()) / len(a), "ndcg20": float(r.ndcg[0].item()) / len(a),
           "ce": round(float(r.loss.item()), 5), "ms": round((time.perf_counter() - t0) * 1e3, 2),
           "note": "evaluate()'s device path on the held-out batch: no (B, A) logits (DESIGN §4c)"}
    idx = r.idx.cpu().numpy()
    net.train()
    return out, idx


def gather_bytes(T, E):
    # per token: int64 id read, fp32 table row read, packed row write, int32 token-id write
    return T * (8 + 2 * 4 * E + 4)


def sampled_fwd_bytes(B, S, HF):
    # h, targets, negative ids, target + negative W rows and biases, logits B·(S+1)
    return B * HF * 4 + B * 4 + S * 4 + (B + S) * (HF + 1) * 4 + B * (S + 1) * 4


def exchange_bytes(U, B, S, E, HF):
    """Collective payload per rank of the item-sharded gather + sampled logits
    (DESIGN §5): the batch's U distinct ids out and their table rows back
    (rg_shard_dedup), the negatives' rows + biases all-reduced, the targets'
    ids out and rows + biases back (HF + 4 floats per row, one all-to-all)."""
    return {"distinct_ids": int(4 * U), "distinct_rows": int(4 * E * U), "neg_rows_allreduce": int(4 * S * (HF + 1)),
            "target_ids": int(4 * B), "target_rows": int(4 * B * (HF + 4))}


def target_step(kern, T, B, S, E, HF, n_gather, terms, U=None):
    """North-star target: embedding gather + sampled logits (fwd) against the
    HBM roofline, with the logits' MFMA rate beside it.  On an
    item-sharded run the gather region is the whole exchange (route, id / row
    all-to-alls, owner gather, placement) and the negatives' / targets' row
    exchange (neg_exchange) is timed into the step too; the algorithmic bytes
    stay the one-GPU ones, the exchanged bytes are stated beside them."""
    if "gather" not in kern or "sampled_fwd" not in kern:
        return None
    tg, ts, tx = kern["gather"] * n_gather, kern["sampled_fwd"], kern.get("neg_exchange", 0.0)
    by = n_gather * gather_bytes(T, E) + sampled_fwd_bytes(B, S, HF)
    gbs = by / ((tg + ts + tx) * 1e-3) / 1e9
    fl = 2.0 * B * S * HF
    out = {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(gbs / HBM_PEAK_GBS, 4), "bytes_per_step": int(by), "ms": round(tg + ts + tx, 4),
           "gather_ms": round(tg, 4), "gather_GBs": round(n_gather * gather_bytes(T, E) / (tg * 1e-3) / 1e9, 1),
           "sampled_fwd_ms": round(ts, 4), "sampled_fwd_alg_TFLOPs": round(fl / (ts * 1e-3) / 1e12, 2)}
    if "neg_exchange" in kern:
        out["neg_exchange_ms"] = round(tx, 4)
        out["exchange_bytes_per_rank"] = exchange_bytes(T if U is None else U, B, S, E, HF)
        out["tokens_per_rank"], out["unique_ids_per_rank"] = int(T), (None if U is None else int(U))
    if terms:
        out["sampled_fwd_mfma_frac"] = round(terms * fl / (ts * 1e-3) / 1e12 / BF16_MFMA_PEAK_TFLOPS, 4)
        out["mfma"] = f"bf16 MFMA, {terms} plane products per fp32 product"
    else:
        out["sampled_fwd_mfma_frac"] = round(fl / (ts * 1e-3) / 1e12 / FP32_MFMA_PEAK_TFLOPS, 4)
    return out


# HBM traffic from the PMC passes (tools/pmc_head.sh, tools/pmc_ns.sh; profiles/pmc_traffic.json):
# an entry {"bytes": per launch / per step, "src": hash, "file": the PMC output under profiles/} counts
# only while "src" equals the hash of the sources that define the kernels measured (kernel_src_hash),
# so a kernel edited after its PMC pass reports traffic null instead of a stale number
KERNEL_SRC = {"head": ("head_flash.hip", "common.h"),
              "gather+sampled_fwd": ("pack_gather.hip", "sampled.hip", "common.h")}


def kernel_src_hash(group):
    import hashlib
    h = hashlib.sha256()
    for f in KERNEL_SRC[group]:
        with open(os.path.join(HERE, "ikea-recommender-system_amd", "csrc", f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def pmc_traffic(key, group):
    """Measured HBM bytes of ``key`` when its PMC pass ran on the current
    sources of ``group``, else None."""
    pmc = os.path.join(HERE, "profiles", "pmc_traffic.json")
    if not os.path.exists(pmc):
        return None
    e = json.load(open(pmc)).get(key)
    if not isinstance(e, dict) or e.get("src") != kernel_src_hash(group):
        return None
    return int(e["bytes"])


def head_roofline(kern, precision, B, N, E, zs=False, cfg="c2"):
    """zs: the stored-logit head (pass 1 stores z, pass 2 reads it and runs
    the dW contraction only: half of PASS_PRODUCTS' pass-2 products)."""
    flops_head = 2.0 * B * N * E  # one (B × E)·(E × A) contraction
    terms = LOGIT_TERMS.get(precision, 0)
    heads = {k: kern[k] for k in ("head_fwd", "head_dh", "head_dw_adam") if k in kern}
    if not heads:
        return None
    dom = max(heads, key=heads.get)
    t = heads[dom] * 1e-3
    # the PMC passes ran at the C2 shapes (B 4096, 1M items, d128), stored-logit head
    traffic = (pmc_traffic(f"{dom}:{precision}:zs", "head") if (B, N, E) == (BATCH, ITEMS, DIM) and zs and cfg == "c2"
               else None)
    if terms:
        # fused split-bf16 head (csrc/head_flash.hip): pass 1 (head_fwd: Z and the softmax half of
        # dh) and pass 2 (head_dw_adam: Z recomputed — or read back when stored — and dW), every fp32
        # product as exact bf16 plane products on v_mfma_f32_16x16x32_bf16 (PASS_PRODUCTS per pass)
        nprod = PASS_PRODUCTS[precision].get(dom, 0) // (2 if zs and dom == "head_dw_adam" else 1)
        ex = nprod * flops_head
        alg = {"head_fwd": 2, "head_dw_adam": 1}.get(dom, 0) * flops_head
        ach = ex / t / 1e12
        out = {"bound": "mfma", "kernel": dom, "achieved": round(ach, 2), "peak": BF16_MFMA_PEAK_TFLOPS,
               "unit": "TFLOP/s", "frac": round(ach / BF16_MFMA_PEAK_TFLOPS, 4), "traffic": traffic,
               "flops_per_launch": ex,
               "mfma": f"bf16 MFMA, fp32 operands split exactly into 3 bf16 planes, "
                       f"{nprod} plane products per fp32 product of the pass",
               "stored_logits": bool(zs),
               "algorithmic_fp32_TFLOPs": round(alg / t / 1e12, 2)}
        if zs and dom == "head_dw_adam":
            # the stored-logit pass 2 reads the logits (16.4 GB at C2) and streams the Adam state: it is priced
            # against both ceilings and reported on the one it comes closer to (the other one beside it)
            hb = (-(-N // 32) * 32 * B * 4 + N * E * (24 + 12) + N * (24 + 4))
            hbm = {"bound": "hbm", "kernel": dom, "achieved": round(hb / t / 1e9, 1), "peak": HBM_PEAK_GBS,
                   "unit": "GB/s", "frac": round(hb / t / 1e9 / HBM_PEAK_GBS, 4), "traffic": traffic,
                   "bytes_per_launch": hb, "stored_logits": True}
            mf = {k: out[k] for k in ("bound", "achieved", "peak", "unit", "frac", "flops_per_launch")}
            if hbm["frac"] > out["frac"]:
                out = dict(out, **hbm)
                out["other"] = mf
            else:
                out["other"] = {k: hbm[k] for k in ("bound", "achieved", "peak", "unit", "frac", "bytes_per_launch")}
        if "head_fwd" in kern and "head_dw_adam" in kern:   # the two passes together (the head's step share)
            p1 = PASS_PRODUCTS[precision].get("head_fwd", 0) * flops_head
            p2 = PASS_PRODUCTS[precision].get("head_dw_adam", 0) // (2 if zs else 1) * flops_head
            tt = (kern["head_fwd"] + kern["head_dw_adam"]) * 1e-3
            out["both_passes"] = {"ms": round(tt * 1e3, 4), "executed_bf16_TFLOP": round((p1 + p2) / 1e12, 3),
                                  "achieved": round((p1 + p2) / tt / 1e12, 2), "unit": "TFLOP/s",
                                  "frac": round((p1 + p2) / tt / 1e12 / BF16_MFMA_PEAK_TFLOPS, 4)}
        if dom == "head_dw_adam":
            out["note"] = ("pass 2 runs on a side stream beside the trunk backward (and, in the SMORL step, the "
                           "target and Q-head passes): its event time is the kernel's duration while sharing "
                           "the CUs, not a standalone launch (DESIGN §4b)")
        return out
    ach = flops_head / t / 1e12
    return {"bound": "mfma", "kernel": dom, "achieved": round(ach, 2), "peak": FP32_MFMA_PEAK_TFLOPS,
            "unit": "TFLOP/s", "frac": round(ach / FP32_MFMA_PEAK_TFLOPS, 4), "traffic": traffic,
            "flops_per_launch": flops_head}


def describe(cfg, N, E, L, B, world, S):
    """(metric, workload) of a config's line."""
    if cfg == "c2":
        return ("session-steps/sec at 1M items, dim128, batch 4096; HR@20/NDCG@20 parity",
                f"GRU4Rec {N} items, dim{E}, seq_len<={L}, batch {B}/GPU, full-softmax logits")
    if cfg == "c3":
        return ("session-steps/sec, BidirGRU4Rec 1M items, dim128, batch 4096, 2048 sampled negatives",
                f"BidirGRU4Rec {N} items, dim{E}, seq_len<={L}, batch {B}, {S} shared uniform "
                f"negatives (sampled softmax), dropout 0")
    if cfg == "c4":
        return ("session-steps/sec, SMORL (SQN double-Q, 3 rewards) 1M items, dim128, batch 4096",
                f"SMORL_trainer {N} items, dim{E}, seq_len<={L}, global batch {B * world} ({B}/GPU), sup head + "
                f"Q heads acc/div/nov, topk_div=topk_nov=1, q_weights [1,1,1], gamma 0.5, alpha 1")
    return ("session-steps/sec, IKEA-scale SMORL (SQN double-Q, 3 rewards) 5M items, dim256, batch 8192",
            f"SMORL_trainer {N} items, dim{E}, seq_len<={L}, global batch {B * world} ({B}/GPU), fp16 item "
            f"table (fp32 master + Adam), sup head + Q heads acc/div/nov, topk_div=topk_nov=1, "
            f"q_weights [1,1,1], gamma 0.5, alpha 1")


def side_line(cfg, args, dev, batches, tok, steps, warmup, settle=0):
    """A short line of another BASELINE config on one GPU, same stream and
    device as the C2 line (C3: BidirGRU4Rec with 2048 sampled negatives,
    configs[2]; C4: SMORL 3-reward double-Q, configs[3] at its global batch on
    one GPU): value, step times, roofline and kernel times — no CPU leg.
    ``settle`` untimed steps first (the stream's batches cycled): the catch-up
    Adam's replay of a sampled head's negatives grows over the first ~3·A/S
    steps, so the C3 line is timed at that steady state, not on a
    fresh table."""
    B, N, E, L = args.batch, args.items, args.dim, args.seq
    tr = make_trainer(cfg, args, dev, False)
    apply_stored_logits(tr, args.stored_logits)
    tr.set_train()
    for i in range(settle):
        tr.train_step(*step_args(cfg, batches[i % len(batches)]))
    dt, losses, kern, per_step = timed_run(tr, batches, warmup, steps, 1, True, cfg)
    terms = LOGIT_TERMS.get(args.precision, 0)
    roof = None
    if cfg == "c3":
        T = float(np.mean(tok[warmup:warmup + steps]))
        roof = target_step(kern, T, B, args.negatives, E, 2 * E, 2, terms)
        if roof:
            roof["kernel"] = "gather + sampled_fwd"
            roof["traffic"] = (pmc_traffic("c3:gather+sampled_fwd", "gather+sampled_fwd")
                               if (B, args.negatives, E) == (4096, 2048, 128) and terms == 6 else None)
    elif kern:
        sup = tr.SMORL_1.sup_head_output
        roof = head_roofline(kern, args.precision if sup.flash_terms(B) else "f32", B, N, E,
                             zs=sup.stored_logits(), cfg=cfg)
    scanned = top_scanned(tr)
    del tr
    torch.cuda.empty_cache()
    metric, workload = describe(cfg, N, E, L, B, 1, args.negatives)
    ps = np.array(per_step) * 1e3
    return {"metric": metric, "workload": workload, "value": round(B * steps / dt, 2), "unit": "session-steps/sec",
            "n_gpus": 1, "steps": steps, "warmup": warmup, "settle_steps": settle,
            "ms_per_step": round(dt / steps * 1e3, 3), "step_ms": {"median": round(float(np.median(ps)), 3), "p10": round(float(np.percentile(ps, 10)), 3),
                        "p90": round(float(np.percentile(ps, 90)), 3)},
            "roofline": roof, "kernel_ms": kern, "loss_first_last": [round(losses[0], 5), round(losses[-1], 5)],
            "top_scanned_rows": scanned}


# side lines timed in a child process (RG_SIDE_CHILD, comma-separated configs)
SIDE_CHILD = tuple(c for c in os.environ.get("RG_SIDE_CHILD", "c3,c4").split(",") if c)
SIDE_KEYS = ("metric", "workload", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "step_ms", "roofline",
             "kernel_ms", "loss_first_last", "top_scanned_rows")


def side_line_process(cfg, args, steps, warmup, settle=0):
    """The side line of ``cfg`` in a child process: ``bench.py --config cfg``
    with the C2 line's precision / stored-logit settings, same seeded stream.
    A step that spreads its kernels over several HIP streams measures what it
    would in a process of its own only if its streams get their own hardware
    queues; after the C2 and C3 trainers created theirs, the C4 trainer's
    streams are assigned round-robin onto queues those already hold (C4 in
    process 217.0K, median 18.81 ms, against 224.5K, median 18.11 ms, as its
    own line on the same box, profiles/r07/bench_c4_side_in_process.json).
    None when the child fails (the caller then times it in process)."""
    import subprocess
    cmd = [sys.executable, os.path.join(HERE, "bench.py"), "--config", cfg, "--steps", str(steps), "--warmup",
           str(warmup), "--no-cpu-baseline", "--no-eval", "--no-native-side", "--no-target", "--extra-steps", "0",
           "--precision", args.precision, "--stored-logits", args.stored_logits, "--settle", str(settle)]
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE")}
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env)
        d = json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else None
    except (subprocess.SubprocessError, ValueError, IndexError):
        d = None
    if not d or "value" not in d:
        return None
    out = {k: d.get(k) for k in SIDE_KEYS}
    out.update(settle_steps=settle, process="child")
    return out


def pinned(b):
    return tuple(x.pin_memory() for x in b)


# ------------------------------------------------------ multi-rank launch ---
def free_port():
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch_cmd(nproc, argv, port):
    """torch.distributed.run command starting one rank per GPU of this node."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]


def relay_json(stdout_text):
    """The one JSON result line among the ranks' merged stdout (rank 0's)."""
    found = None
    for line in stdout_text.splitlines():
        line = line.strip()
        if line.startswith("{"):
            try:
                d = json.loads(line)
            except ValueError:
                continue
            if isinstance(d, dict) and "metric" in d:
                found = line
    return found


def launch_ranks(args, argv, runner=None):
    """``bench.py --gpus N`` without a torch.distributed launcher: start the N
    ranks as child processes (torch.distributed.run, before this process
    touches any GPU) and relay rank 0's JSON line.  Returns the exit code."""
    import subprocess
    runner = runner or subprocess.run
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    r = runner(launch_cmd(args.gpus, argv, free_port()), stdout=subprocess.PIPE, env=env, text=True)
    line = relay_json(r.stdout or "")
    if r.returncode != 0 or line is None:
        sys.stderr.write(r.stdout or "")
        return r.returncode or 1
    sys.stdout.write(line + "\n")
    sys.stdout.flush()
    return 0


def check_world(args):
    """None when this process is a rank of the right world size; otherwise the
    action: ("launch", N) or ("error", message)."""
    ws = os.environ.get("WORLD_SIZE")
    if ws is None:
        return ("launch", args.gpus) if args.gpus > 1 else None
    if int(ws) != args.gpus:
        return ("error", f"bench.py: WORLD_SIZE={ws} but --gpus {args.gpus}")
    return None


def max_over_ranks(vals, op="max"):
    """Element-wise max (or sum) of a list of floats over the ranks."""
    if not torch.distributed.is_initialized():
        return list(vals)
    native = torch.distributed.get_backend() == "nccl"
    t = torch.tensor(vals, dtype=torch.float64, device=torch.cuda.current_device() if native else "cpu")
    torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX if op == "max" else torch.distributed.ReduceOp.SUM)
    return [float(x) for x in t.cpu()]


def harness_run(tr, batches, n, args, item_counts):
    """The reference training loop's per-batch pair (trainGRU.py:195-224):
    ``train_step`` then ``update_train_metrics`` on the same batch (top-k
    [10, 20] HR / NDCG, coverage [1, 5, 10], diversity + novelty top-1 with a
    frozen 64-wide div table).  Returns per-batch ms statistics."""
    from recommenders.data_utils.synthetic import unpopular_items
    from recommenders.evaluate.eval_protocol import update_train_metrics
    g = torch.Generator().manual_seed(7)
    div = torch.nn.Embedding.from_pretrained(torch.randn(args.items + 1, 64, generator=g) * 0.01, freeze=True)
    unpop = unpopular_items(item_counts)
    cov = {k: set() for k in (1, 5, 10)}
    t_all, t_met = [], []
    for i in range(n):
        s, a, _, _, ln, _, _ = batches[i % len(batches)]
        t0 = time.perf_counter()
        tr.set_train()
        tr.train_step(s, a, ln)
        t1 = time.perf_counter()
        hr, nd, cov, dv, nv, reps = update_train_metrics(
            s=s, a=a, s_len=ln, model=tr.gru_model, device=tr.device, padding_pos="end", diversity_embedding=div,
            unpopular_actions_set=unpop, actions_covered_topk_dict=cov, head_idx=0, topk_hr_ndcg=[10, 20],
            topk_to_consider_cov=[1, 5, 10], topk_to_consider_div=1, topk_to_consider_nov=1, novelty_rew_signal=1)
        float(dv)   # the harness accumulates it on the host
        t2 = time.perf_counter()
        t_all.append(t2 - t0)
        t_met.append(t2 - t1)
    tr.set_train()
    B = batches[0][0].shape[0]
    ta, tm = np.array(t_all[1:]) * 1e3, np.array(t_met[1:]) * 1e3
    return {"harness_ms_per_step": round(float(np.median(ta)), 3),
            "update_train_metrics_ms": round(float(np.median(tm)), 3),
            "value": round(B / (float(np.median(ta)) * 1e-3), 2), "unit": "session-steps/sec", "batches": n - 1,
            "note": "median per batch of train_step + update_train_metrics (trainGRU.py:195-224), after 1 untimed "
                    "batch; metrics: HR/NDCG@[10,20], coverage [1,5,10], div/nov top-1; update_train_metrics_ms is "
                    "the host time from train_step's return (at its loss readout, the backward still queued) to "
                    "the metrics, so it includes the step's remaining GPU work"}


def per_rank_batch(config, batch, world):
    """Rows each rank trains per step.  C4 / C5 name a GLOBAL batch on 8 GPUs
    (BASELINE configs[3]: batch 4096 embedding-sharded across 8×MI355X, SURVEY
    §8e: B/8 = 512 sessions per rank; configs[4]: batch 8192), so their ranks
    split it (strong scaling); C2 / C3 are 1-GPU configs whose multi-GPU lines
    keep the batch per GPU (weak scaling)."""
    if config in ("c4", "c5"):
        if batch % (32 * world):
            raise SystemExit(f"{config}: the global batch must split into multiples of 32 rows per rank")
        return batch // world
    return batch


def main():
    args = parse()
    act = check_world(args)
    if act is not None:
        if act[0] == "error":
            raise SystemExit(act[1])
        # no torch.distributed launcher around us: start the ranks as children
        sys.exit(launch_ranks(args, sys.argv[1:]))
    # the ONE JSON line goes to the real stdout; everything else that writes to
    # fd 1 while the job runs (RCCL's version banner at init, library logs)
    # is sent to stderr
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.config == "c5":
        # BASELINE configs[4]: 5M items, d256, seq_len <= 100, batch 8192, fp16
        # item table; flags that were left at the C2 defaults take the C5 values
        for k, c2v, c5v in (("items", ITEMS, 5_000_000), ("dim", DIM, 256), ("seq", SEQ, 100),
                            ("batch", BATCH, 8192)):
            if getattr(args, k) == c2v:
                setattr(args, k, c5v)
    args.batch = per_rank_batch(args.config, args.batch, world)
    shard = (world > 1 or args.force_shard) and args.config in ("c2", "c4", "c5")
    if world > 1 or args.force_shard:
        import torch.distributed as dist
        # RCCL in production; RG_BENCH_BACKEND=gloo rehearses the N-rank path with
        # several ranks on one GPU (host-staged collectives, hip/dist.py)
        backend = os.environ.get("RG_BENCH_BACKEND", "nccl")
        if backend != "nccl":
            local %= torch.cuda.device_count()
        torch.cuda.set_device(local)
        dist.init_process_group(backend)
    if world > 1 and args.config == "c3":
        raise SystemExit("multi-GPU bench runs the C2 / C4 / C5 workloads")
    from recommenders.data_utils.synthetic import SessionStream

    dev = torch.device("cuda", local)
    B, L, N, E = args.batch, args.seq, args.items, args.dim
    nsteps = args.warmup + args.steps
    # synthetic session stream (seeded per rank: each rank owns its batch shard);
    # one extra batch is held out for evaluation
    st = SessionStream(N, L, B * (nsteps + 1), seed=2 + rank)
    args.item_counts = st.item_counts()
    batches, tok, uniq = [], [], []
    for i in range(nsteps):
        b = st.batch(i, B)
        batches.append(pinned(b))
        tok.append(int(b[4].sum()))
        ln = np.clip(b[4].numpy(), 1, L)
        uniq.append(int(np.unique(b[0].numpy()[np.arange(L)[None, :] < ln[:, None]]).size))
    hb = st.batch(nsteps, B)
    held = (hb[0], hb[1], hb[4])
    T = float(np.mean(tok[args.warmup:]))
    U = float(np.mean(uniq[args.warmup:]))   # distinct items per batch (the sharded exchange's rows)
    t_init = time.perf_counter()
    tr = make_trainer(args.config, args, dev, shard)
    apply_stored_logits(tr, args.stored_logits)
    tr.set_train()
    print(f"bench: trainer built in {time.perf_counter() - t_init:.1f} s, "
          f"{torch.cuda.memory_allocated(dev) / 2**30:.1f} GiB on the device", file=sys.stderr, flush=True)
    for i in range(args.settle):
        tr.train_step(*step_args(args.config, batches[i % len(batches)]))
    dt, losses, kern, per_step = timed_run(tr, batches, args.warmup, args.steps, world, not args.no_kernel_timing,
                                           args.config)
    scanned = top_scanned(tr)   # over the timed steps (exact either way; each costs one whole-row scan)
    print(f"bench: peak device memory {torch.cuda.max_memory_allocated(dev) / 2**30:.1f} GiB", file=sys.stderr,
          flush=True)
    net = getattr(tr, "gru_model", None)
    harness = None
    if args.config == "c2" and not shard and args.harness_steps > 1 and not args.no_eval:
        harness = harness_run(tr, batches, args.harness_steps, args, args.item_counts)
    ev, dev_idx = None, None
    if not args.no_eval and not shard and net is not None:
        ev, dev_idx = device_eval(net, held)
    elif not args.no_eval and not shard and args.config in ("c4", "c5"):
        # the supervised head of the trained SMORL net (evaluate(head_idx=0));
        # at C5 (5M items, batch 8192) the held-out evaluation must fit beside
        # the trainer: the target-side trunk workspaces are dropped first
        for q in (tr.SMORL_1, tr.SMORL_2):
            for k in [k for k in q.trunk._ws if k[0] in ("next", "boot")]:
                del q.trunk._ws[k]
        torch.cuda.empty_cache()
        ev, _ = device_eval(tr.SMORL_1, held)
    ms = dt / args.steps * 1e3
    value = B * args.steps * world / dt
    roof = None
    target = None
    native = None
    parity_net = None
    gpar = None
    extra = None
    HF = E * (2 if args.config == "c3" else 1)
    terms = LOGIT_TERMS.get(args.precision, 0)
    want_cpu = world == 1 and rank == 0 and not args.no_cpu_baseline
    cpu_items, cpu_B, cpu_steps = cpu_sample(args, args.config)
    # the loss-parity leg (C2): the CPU leg's sample is the first batches of THIS stream at the
    # CPU leg's batch size, trained by the oracle and by a fresh copy of the benched GPU trainer
    par_batches = None
    if want_cpu and args.config == "c2" and cpu_items == N and (1 + cpu_steps) * cpu_B <= len(st):
        par_batches = [st.batch(i, cpu_B) for i in range(1 + cpu_steps)]
    if args.config in ("c2", "c4", "c5"):
        if kern:
            sup = net.heads["output"] if net is not None else tr.SMORL_1.sup_head_output
            prec = args.precision if sup.flash_terms(B * world) else "f32"
            roof = head_roofline(kern, prec, B * world, N // world, E, zs=sup.stored_logits(), cfg=args.config)
        if args.config == "c2":
            if world == 1 and not args.no_cpu_baseline and not args.no_eval and net is not None:
                parity_net = net
            else:
                del net
            del tr
            torch.cuda.empty_cache()
            if world == 1 and not args.no_native_side and args.precision != "f32":
                # the native fp32 MFMA head (precision "f32"), short side run
                trn = make_trainer("c2native", args, dev, False)
                trn.set_train()
                dtn, _, _, psn = timed_run(trn, batches, 2, min(10, args.steps), 1, False, "c2")
                native = {"value": round(B * min(10, args.steps) / dtn, 2),
                          "ms_per_step": round(dtn / min(10, args.steps) * 1e3, 3), "matmul_precision": "f32",
                          "note": "native fp32 MFMA head (matmul_precision f32), 10 steps"}
                del trn
                torch.cuda.empty_cache()
            if not args.no_target and kern:
                # north-star target step measured on GRU4Rec at C2
                # shapes with the sampled head: a short side run, own trainer, on
                # every rank (its own batch shard); at N > 1 item-sharded like the
                # C2 line (row-sharded table, engine.ShardedSampledHead)
                tr2 = make_trainer("c2s", args, dev, shard)
                tr2.set_train()
                _, _, k2, _ = timed_run(tr2, batches, min(5, args.warmup), min(30, args.steps), world, True, "c2")
                target = target_step(k2, T, B, args.negatives, E, E, 1, terms, U=U)
                if target is not None and world > 1:
                    by_sum, = max_over_ranks([float(target["bytes_per_step"])], op="sum")
                    tg, ts, tx = max_over_ranks([k2["gather"], k2["sampled_fwd"], k2.get("neg_exchange", 0.0)])
                    gbs = by_sum / ((tg + ts + tx) * 1e-3) / 1e9
                    target.update({"achieved": round(gbs, 1), "peak": HBM_PEAK_GBS * world,
                                   "frac": round(gbs / (HBM_PEAK_GBS * world), 4), "bytes_per_step": int(by_sum),
                                   "ms": round(tg + ts + tx, 4), "gather_ms": round(tg, 4),
                                   "sampled_fwd_ms": round(ts, 4), "neg_exchange_ms": round(tx, 4), "ranks": world,
                                   "note": "item-sharded: every rank's gather (route, id / row all-to-alls, owner "
                                           "gather, placement) + the negatives' / targets' row exchange + the "
                                           "sampled logits over its own batch shard; algorithmic bytes (one-GPU "
                                           "definition) summed over ranks, region times max over ranks, peak = "
                                           "ranks x 8 TB/s; exchange_bytes_per_rank beside"})
                if target is not None:
                    target["workload"] = f"GRU4Rec {N} items dim{E} batch {B}/GPU, {args.negatives} sampled negatives"
                    target["kernel_ms"] = k2
                    # HBM bytes of the two kernels per step from the PMC passes (tools/pmc_ns.sh), which
                    # measured the one-GPU kernels at these shapes
                    target["traffic"] = None
                    if (N, E, B, args.negatives) == (1_000_000, 128, 4096, 2048) and terms == 6 and not shard:
                        target["traffic"] = pmc_traffic("c2:gather+sampled_fwd", "gather+sampled_fwd")
                del tr2
                torch.cuda.empty_cache()
            if par_batches is not None:
                gpar = gpu_parity_run(args, dev, par_batches)
            if world == 1 and args.extra_steps > 0:
                # driver-visible C3 / C4 lines (BASELINE configs[2] / [3] on one GPU) on the same stream
                extra = {}
                wx = min(5, args.warmup)
                nx = min(args.extra_steps, len(batches) - wx)
                for c in ("c3", "c4"):
                    # C3 and C4 (several side streams per step) each in a process of its own
                    ln = (side_line_process(c, args, nx, wx, args.extra_settle if c == "c3" else 0)
                          if c in SIDE_CHILD else None)
                    extra[c] = ln if ln is not None else side_line(c, args, dev, batches, tok, nx, wx,
                                                                   settle=args.extra_settle if c == "c3" else 0)
    else:
        target = target_step(kern, T, B, args.negatives, E, HF, 2, terms)
        roof = dict(target) if target else None
        if roof:
            roof["kernel"] = "gather + sampled_fwd"
            roof["traffic"] = None
            if (B, args.negatives, HF) == (4096, 2048, 256) and terms == 6:
                roof["traffic"] = pmc_traffic("c3:gather+sampled_fwd", "gather+sampled_fwd")
    if rank != 0:
        if torch.distributed.is_initialized():
            torch.distributed.destroy_process_group()
        return
    cpu = None
    lparity = None
    if want_cpu:
        cpu = cpu_baseline(args, args.config, batches=par_batches, counts=args.item_counts)
        orc_out = cpu.pop("_oracle", None)
        if gpar is not None and orc_out is not None:
            lparity = loss_parity(gpar[0], orc_out[0], gpar[1], orc_out[1].net.state_dict(), 0.01, cpu_B)
        del orc_out
        if ev is not None and dev_idx is not None and parity_net is not None:
            cpu["hr_ndcg_parity"] = cpu_eval_parity(parity_net, held, dev_idx)
    metric, workload = describe(args.config, N, E, L, B, world, args.negatives)
    ps = np.array(per_step) * 1e3
    line = {
        "metric": metric,
        "value": round(value, 2), "unit": "session-steps/sec", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, **({"settle_steps": args.settle} if args.settle else {}),
        "ms_per_step": round(ms, 3), "higher_is_better": True,
        "scaling": "strong" if args.config in ("c4", "c5") else "weak",
        "vs_baseline": None, "dtype": "f32", "matmul_precision": args.precision, "stored_logits": args.stored_logits,
        "data": "synthetic (seeded Zipf session stream, random-init weights)",
        "config": {"workload": workload,
                   "global_batch": B * world, "seq_len": L, "items": N, "dim": E,
                   "parallelism": (f"dp{world} trunk + {world}-way item-sharded tables "
                                   f"({torch.distributed.get_backend() if torch.distributed.is_initialized() else ''})"
                                   if shard else "single"),
                   "tokens_per_batch": int(T), "distinct_items_per_batch": int(U)},
        "step_ms": {"median": round(float(np.median(ps)), 3), "p10": round(float(np.percentile(ps, 10)), 3),
                    "p90": round(float(np.percentile(ps, 90)), 3), "mean": round(float(ps.mean()), 3)},
        "roofline": roof, "cpu_baseline": cpu, "north_star_target": target, "eval_heldout": ev,
        "harness": harness, "native_f32": native, "kernel_ms": kern,
        "loss_first_last": [round(losses[0], 5), round(losses[-1], 5)],
        "top_scanned_rows": scanned, "loss_parity": lparity, "configs_extra": extra,
    }
    os.write(json_fd, (json.dumps(line) + "\n").encode())
    if torch.distributed.is_initialized():
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
