"""ctypes binding of the gfx950 C-ABI library (include/ikea_rec_hip.h).

This is the only route to compute in the package: there is no CPU or
PyTorch fallback.  If the library is missing, or no MI355X is visible, the
trainers raise instead of silently running something else.
"""
from __future__ import annotations

import ctypes as C
import os

import torch

LIB_PATH = os.environ.get("IKEA_REC_HIP_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                                "libikea_rec_hip.so")

P = C.c_void_p
I = C.c_int
I64 = C.c_int64
F = C.c_float
D = C.c_double
I32 = C.c_int32
U64 = C.c_uint64

# entry points returning int64_t (all others return int)
RESTYPE_I64 = {"rg_sampled_work_bytes", "rg_head_work_bytes", "rg_head_plane_bytes", "rg_gru_wide_work_bytes",
               "rg_scatter_rows_work_bytes", "rg_flash_dw_work_bytes", "rg_shard_dedup_work_bytes",
               "rg_flash_topk_work_bytes", "rg_flash_zs_bytes"}

# name -> argtypes
SIGNATURES = {
    "rg_abi_version": [],
    "rg_partial_block": [],
    "rg_pack": [P, I, I, I, P, P, P, P],
    "rg_gather": [P, I, I, P, P, P, P, I64, I, I, P, P, P, P],
    "rg_scatter_rows_work_bytes": [I, I, I64],
    "rg_scatter_rows": [P, P, I, I, P, I, I, P, I64, P, I32, I, P, I64, P],
    "rg_gemm_f32": [P, I64, I64, P, I64, I64, P, I64, P, I, P, I, I, P, I, P],
    "rg_reduce_slabs": [P, I, I64, P, P, I, I, P],
    "rg_colsum": [P, I, I, P, I, P, P],
    "rg_wgrad": [P, I, P, I, I, P, I, P, P, P],
    "rg_gru_fwd": [P, P, P, P, P, P, I, I, P, I, I, P, I64, P],
    "rg_gru_bwd": [P, I64, P, P, P, P, I, I, P, I, I, P, P, P],
    "rg_head_fwd": [P, P, P, I, I, I, P, I64, P, P, P, I, P],
    "rg_head_work_bytes": [I, I],
    "rg_head_fwd_x": [P, P, P, I, I, I, I, P, I64, P, P, P, I, P, P],
    "rg_head_fwd_xp": [P, P, P, I, I, I, I, I, P, I64, P, P, P, I, P],
    "rg_head_plane_bytes": [I, I],
    "rg_head_planes": [P, I, I, P, P, P, P, P],
    "rg_flash_fwd": [P, P, P, P, I, I, I, I, I, P, P, P, P],
    "rg_flash_rows_per_block": [I],
    "rg_remap_ids": [P, I64, P, I64, P, P, P],
    "rg_build_transitions": [P, P, P, P, P, I, I, I64, I, P, P, P, P, P, P, P, P],
    "rg_flash_fwd_top": [P, P, P, P, I, I, I, I, I, P, P, P, P, P, P, P, P],
    "rg_flash_zs_bytes": [I, I],
    "rg_flash_argmax": [P, P, I, I, P, P, P],
    "rg_flash_amax_fwd": [P, P, P, I, I, I, I, I, P, P, P],
    "rg_flash_score": [P, P, P, I, I, I, I, I, P, P, P, P, P, P],
    "rg_flash_amax_screen": [P, P, P, I, I, I, I, I, P, P, P, P],
    "rg_row_norm_max": [P, I64, I, P, P],
    "rg_comm_id_bytes": [],
    "rg_comm_unique_id": [P],
    "rg_comm_init": [P, I, I, I, P],
    "rg_comm_destroy": [P],
    "rg_comm_alltoallv": [P, P, P, P, P, I, P],
    "rg_comm_allreduce": [P, P, P, I64, I, P],
    "rg_comm_allgather": [P, P, P, I64, I, P],
    "rg_comm_reduce_scatter": [P, P, P, I64, I, P],
    "rg_flash_argmax_exact": [P, I, I, P, P, P, I, P, F, P, P, P, P, P, P, P],
    "rg_flash_topk_cap": [],
    "rg_flash_topk": [P, I, I, I, I, F, F, P, P, P, I, P, P, P, P, P, P, P],
    "rg_flash_topk_work_bytes": [I, I, I],
    "rg_flash_topk_screened": [P, I, I, I, I, F, P, P, P, P, I, P, P, P, P, P, P, P],
    "rg_flash_lse": [P, P, I, P, P, P, P, I64, I, I64, I, I, P, P, P],
    "rg_flash_rows": [P, P, I64, I, I, P, P],
    "rg_flash_dh": [P, P, P, I, P, F, I, I, P, P],
    "rg_flash_dw_adam": [P, P, P, P, P, F, I, I, I, I, P, P, P, P, P, P, P, P, P, P],
    "rg_flash_dw_adam_planes": [P, P, P, P, P, F, I, I, I, I, P, P, P, P, P, P, P, P, P, P, P, P, P, I64, P, P],
    "rg_flash_dw_work_bytes": [I, I, I],
    "rg_timing_events": [P, P],
    "rg_lse_combine": [P, P, P, I, I, P, P, I64, P, I, P, P, P, P, P],
    "rg_sum_scale": [P, I, F, P, P, P],
    "rg_lse_merge_ranks": [P, I, I, P, P],
    "rg_shard_targets": [P, I64, P, I64, I64, I, P, P, P],
    "rg_shard_index": [P, P, I, I64, I64, P, P],
    "rg_argmax_merge_ranks": [P, P, I, I, I64, P, P, P],
    "rg_topk_merge_ranks": [P, P, I, I, I, I64, P, P, P],
    "rg_sub": [P, P, I, P, P],
    "rg_head_dh": [P, I64, P, P, F, P, I, I, I, I, P, P],
    "rg_head_dw_adam": [P, I64, P, P, F, P, I, I, I, P, P, P, P, P, P, P, P, P, P],
    "rg_adam_dense": [P, P, P, P, I64, P, I, P],
    "rg_adam_rows": [P, P, P, P, P, I32, I64, I, P, P],
    "rg_adam_slabs": [P, P, P, P, I, I64, P, P, P],
    "rg_q_gather": [P, I, P, P, I, P, P, I, P, P],
    "rg_q_backward": [P, I, P, I, P, I, P, P, P, P, P, P, P],
    "rg_sqn_td": [P, P, P, P, F, I, D, P, P, P],
    "rg_smorl_td": [P, P, P, P, P, I, F, F, I, P, P, P],
    "rg_sum64": [P, I, D, P, P, P],
    "rg_diversity": [P, I, P, I, P, I, I, P, I64, I, F, I, P, P],
    "rg_novelty": [P, I, I, P, I, F, I, P, P],
    "rg_topk": [P, I64, P, I, I, I, P, P, P, P],
    "rg_hits_ndcg": [P, I, P, I, P, I, P, P],
    "rg_repetitions": [P, I, P, I, I, P, I, P, P],
    "rg_mask_scale": [P, P, F, I64, P, P],
    "rg_gru_wide_work_bytes": [I],
    "rg_gru_fwd_dirs": [P, P, P, P, I, P, P, P, I, I, P, I, I, I64, P],
    "rg_gru_fwd_dirs_planes": [P, P, P, P, I, P, P, P, I, I, P, I, I, I64, P, P],
    "rg_gru_bwd_dirs": [P, P, P, P, I, I64, P, P, P, I, I, P, I, I, P],
    "rg_gru_fwd_wide": [P, P, P, P, P, P, I, I, P, I, I, P, I64, P, P],
    "rg_gru_bwd_wide": [P, I64, P, P, P, P, I, I, P, I, I, P, P, P, P],
    "rg_gather_h": [P, I, I, P, P, P, P, I64, I, I, P, P, P, P],
    "rg_adam_rows_h": [P, P, P, P, P, I32, I64, I, P, P, P],
    "rg_f32_to_f16": [P, I64, P, P],
    "rg_sample_uniform": [U64, U64, I, I64, P, P],
    "rg_sampled_nparts": [I, I, I],
    "rg_sampled_work_bytes": [I, I, I],
    "rg_sampled_fwd_x": [P, P, P, P, I, U64, U64, I64, I, I, I, I, P, I64, P, P, P, P, P, P],
    "rg_sampled_logits": [P, P, P, P, I, U64, U64, I64, I, I, I, I, P, I64, P, P, P, P, P, P, P],
    "rg_gather_neg": [P, I, I, P, P, P, P, I, I64, I, I, P, P, P, P, P, U64, U64, I64, I, I, P, P, P, P, I, P],
    "rg_sampled_dz_rows": [P, I64, P, I, I, F, P, P, P],
    "rg_sampled_fwd": [P, P, P, P, I, I, I, P, I64, P, P, P, P, P],
    "rg_sampled_lse": [P, P, P, P, I, I64, I, P, P, I, F, P, P, P, P, P, P, P],
    "rg_sampled_dz": [P, I64, P, I, I, F, P, P],
    "rg_bpr_rows": [P, P, P, P, I, I64, I, P, I64, I64, I, F, P, P, P, P, P, P, P],
    "rg_bpr_dz": [P, I64, I64, P, I, I, F, P, P, P],
    "rg_weighted_sum": [P, P, I, I64, P, P],
    "rg_stack_rewards": [P, P, P, I, P, P],
    "rg_token_ids": [P, I, I, P, P, P, I64, P, P, P],
    "rg_shard_route": [P, P, I64, I, P, P, P, P],
    "rg_rows_gather": [P, I, I64, I64, P, I, I, P, P, P],
    "rg_place_rows": [P, I, P, P, P, I, I, I, P, P],
    "rg_combine_dirs": [P, P, P, P, I, I, P],
    "rg_qcomb": [P, P, P, I, I, I, I, P, P, P, P, P, P],
    "rg_shard_dedup_work_bytes": [I, I, I64],
    "rg_shard_dedup": [P, P, I, I64, I, I, P, P, P, P, P, I64, P],
    "rg_shard_dedup_grads": [P, I, I, I64, P, P, I64, P],
    "rg_shard_dedup_ids": [P, I, I, P, P, P, P, I, I64, P, I, P, P, P, P, I, P, I64, P],
    "rg_neg_pick": [U64, U64, I64, I, I, I64, I64, P, P, P, P, P, P, P],
    "rg_neg_planes": [P, I, I, P, P],
    "rg_target_ids": [P, I, I64, P, P, P],
    "rg_head_rows_gather": [P, I, I64, I64, P, P, I, I, P, P, P],
    "rg_rows_unslot": [P, I, P, P, I, I, P, P, P, P],
    "rg_rows_slot": [P, P, P, I, I, I, P, P],
    "rg_gemm_x6": [P, I64, P, I64, I, P, I64, P, I, P, I, I, I, P],
    "rg_gemm_x6_sk": [P, I64, I, P, I64, I, P, I64, I64, I, I, I, I, I, P],
    "rg_wgrad_x6": [P, I, P, I, I, P, I, P, P, I, P],
    "rg_lazy_mark_rows": [P, I64, I64, U64, U64, I, P, I32, P],
    "rg_lazy_mark_rows32": [P, I, I64, I64, P, I32, P],
    "rg_lazy_catch_up": [P, P, P, I, P, P, P, P, I64, P, P, I32, I32, P, P],
    "rg_lazy_adam_rows": [P, P, P, P, I, P, P, P, P, P, I64, P, P, I32, I32, P, P, P],
}

_lib = None


def load_library(path: str = LIB_PATH):
    """Load the .so and type every exported entry point (works without a GPU)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError(
            f"MI355X kernel library not built: {path} (run ikea-recommender-system_amd/build.py)")
    lib = C.CDLL(path)
    for name, argtypes in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes = argtypes
        fn.restype = C.c_int64 if name in RESTYPE_I64 else C.c_int
    _lib = lib
    return lib


def require_gpu(device) -> torch.device:
    dev = torch.device(device)
    if dev.type != "cuda" or not torch.cuda.is_available():
        raise RuntimeError(
            "the GRU4Rec/SQN/SMORL step path runs only on an MI355X (HIP device); "
            f"got device={device!r}, torch.cuda.is_available()={torch.cuda.is_available()}")
    load_library()
    return dev


def stream_ptr(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t) -> int | None:
    return None if t is None else t.data_ptr()


def call(name: str, *args) -> int:
    lib = load_library()
    rc = getattr(lib, name)(*args)
    if rc < 0:
        raise RuntimeError(f"{name} failed with status {rc}")
    return rc


def host_ptr_array(tensors):
    """HOST array of device pointers (for the multi-head entry points)."""
    arr = (C.c_void_p * len(tensors))(*[None if t is None else t.data_ptr() for t in tensors])
    return arr


def host_floats(vals):
    return (C.c_float * len(vals))(*[float(v) for v in vals])
