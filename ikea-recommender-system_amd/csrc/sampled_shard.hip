// Item-sharded sampled softmax for the multi-GPU step ("the
// embedding table and session minibatches shard naturally across the 8
// GPUs"; the sampled head itself is the build-defined C3 extension,
// csrc/sampled.hip, replacing the output layer of GRU4Rec/model.py:58-60, 80).
//
// Rank r holds output rows [lo, hi) of W (A × HF) and b, with their Adam
// moments; every rank trains its own B session rows.  Rows move to the data,
// never the logits or an item-sized gradient (recommenders/hip/sampled_shard.py):
//
//   forward   the S shared negatives are drawn from the same counter-based
//             stream on every rank; each rank writes the rows it owns
//             (k_neg_pick, zero rows elsewhere), one SUM all-reduce of
//             S·(HF+1) floats leaves every negative's row and bias on every
//             rank (exact: one nonzero term per element), k_neg_planes cuts
//             them into the logits' fragment-order bf16 planes; the rank's B
//             targets go to their owners (all-to-all of ids, k_head_rows_gather
//             on the owner, ONE all-to-all of the rows with their biases
//             back, k_rows_unslot)
//   backward  the negatives' row gradients (S × HF, summed over the rank's
//             rows) SUM all-reduced, each owner scatters the rows it holds;
//             the targets' row and bias gradients go back to their owners
//             by one all-to-all (k_rows_slot) and are scattered there
#include "common.h"

namespace {

// one thread per (negative x, 8-value group g): the draw's id, and its row /
// bias when this rank owns it (zeros otherwise); nloc = id − lo or −1
__global__ __launch_bounds__(256) void k_neg_pick(uint64_t seed, uint64_t counter, uint64_t A, int S, int HF,
                                                  int64_t lo, int64_t hi, const float* __restrict__ W,
                                                  const float* __restrict__ bias, int32_t* __restrict__ ids,
                                                  int32_t* __restrict__ nloc, float* __restrict__ Wg,
                                                  float* __restrict__ bg) {
  const int G = HF >> 3;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)S * G) return;
  const int x = (int)(i / G), g = (int)(i % G);
  const int id = draw_id(seed, counter, S, x, A);
  const bool own = id >= lo && id < hi;
  f4 a = {0.f, 0.f, 0.f, 0.f}, c = a;
  if (own) {
    const float* src = W + (int64_t)(id - lo) * HF + 8 * g;
    a = *reinterpret_cast<const f4*>(src);
    c = *reinterpret_cast<const f4*>(src + 4);
  }
  float* dst = Wg + (int64_t)x * HF + 8 * g;
  *reinterpret_cast<f4*>(dst) = a;
  *reinterpret_cast<f4*>(dst + 4) = c;
  if (g == 0) {
    ids[x] = id;
    nloc[x] = own ? (int32_t)(id - lo) : -1;
    bg[x] = own ? bias[id - lo] : 0.f;
  }
}

// the gathered rows' fragment-order bf16 planes (rg_sampled_logits draw = 2;
// the layout of csrc/pack_gather.hip neg_prep): a wave covers 32 negatives ×
// 2 groups = one 16-deep slice, each plane store one contiguous 1 KB fragment
__global__ __launch_bounds__(256) void k_neg_planes(const float* __restrict__ Wg, int S, int HF,
                                                    bf16x8* __restrict__ Wp) {
  const int G = HF >> 3, NS = HF >> 4;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)S * G) return;
  const int blk = (int)(i / (32 * G));
  const int rem = (int)(i - (int64_t)blk * 32 * G);
  const int x = blk * 32 + (rem & 31), g = rem >> 5;
  const float* src = Wg + (int64_t)x * HF + 8 * g;
  const f4 a = *reinterpret_cast<const f4*>(src);
  const f4 c = *reinterpret_cast<const f4*>(src + 4);
  bf16x8 p0, p1, p2;
  split3x8(a, c, p0, p1, p2);
  const int lane = (g & 1) * 32 + (x & 31);
  Wp[plane_idx(blk, g >> 1, 0, lane, NS)] = p0;
  Wp[plane_idx(blk, g >> 1, 1, lane, NS)] = p1;
  Wp[plane_idx(blk, g >> 1, 2, lane, NS)] = p2;
}

// targets as int32 routing ids (−1 outside [0, A): routed to rank 0, which
// returns a zero row; the requester marks the row invalid) and their count
__global__ void k_target_ids(const int64_t* __restrict__ tgt, int n, int64_t A, int32_t* __restrict__ out,
                             int32_t* __restrict__ n_out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) *n_out = n;
  if (i >= n) return;
  const int64_t t = tgt[i];
  out[i] = (t >= 0 && t < A) ? (int32_t)t : -1;
}

// Exchange rows carry the bias too: ld = HF + 4 floats per row (row, bias,
// 3 pad: 16-B aligned rows), so each direction is ONE all-to-all.
//
// owner side: W rows and biases of n received item ids from the local shard
// [lo, lo + n_local) into rows[k·ld ..]: the row, then the bias at + HF;
// local_ids[k] = id − lo (−1 and zeros when not held)
__global__ __launch_bounds__(256) void k_head_rows_gather(const int32_t* __restrict__ ids, int n, int64_t lo,
                                                          int64_t n_local, const float* __restrict__ W,
                                                          const float* __restrict__ bias, int HF, int ld,
                                                          float* __restrict__ rows, int32_t* __restrict__ local_ids) {
  const int per = HF / 4;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)n * per) return;
  const int k = (int)(i / per), c = (int)(i % per);
  const int64_t l = (int64_t)ids[k] - lo;
  const bool ok = ids[k] >= 0 && l >= 0 && l < n_local;
  f4 v = {0.f, 0.f, 0.f, 0.f};
  if (ok) v = reinterpret_cast<const f4*>(W + l * HF)[c];
  reinterpret_cast<f4*>(rows + (int64_t)k * ld)[c] = v;
  if (c == 0) {
    local_ids[k] = ok ? (int32_t)l : -1;
    rows[(int64_t)k * ld + HF] = ok ? bias[l] : 0.f;
  }
}

// requester side: tW[b] = row slot[b], tb[b] = its bias, trow[b] = b: the
// CE's target table is tW / tb, row b's target is entry b.  A row whose target
// was invalid gets a zero row and trow[b] = −1, so k_sampled_lse's range
// guard gives it a NaN loss row with zero gradients — as on one GPU, where
// the same guard sees the invalid id itself
__global__ __launch_bounds__(256) void k_rows_unslot(const float* __restrict__ rows, int ld,
                                                     const int32_t* __restrict__ slot,
                                                     const int32_t* __restrict__ tid32, int n, int HF,
                                                     float* __restrict__ tW, float* __restrict__ tb,
                                                     int64_t* __restrict__ trow) {
  const int per = HF / 4;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)n * per) return;
  const int b = (int)(i / per), c = (int)(i % per);
  const bool ok = tid32[b] >= 0;
  const float* src = rows + (int64_t)slot[b] * ld;
  f4 v = {0.f, 0.f, 0.f, 0.f};
  if (ok) v = reinterpret_cast<const f4*>(src)[c];
  reinterpret_cast<f4*>(tW + (int64_t)b * HF)[c] = v;
  if (c == 0) {
    tb[b] = ok ? src[HF] : 0.f;
    trow[b] = ok ? b : -1;
  }
}

// backward: row slot[b] of gsend = grows[b], its bias entry (+ HF) = gb[b]
__global__ __launch_bounds__(256) void k_rows_slot(const float* __restrict__ grows, const float* __restrict__ gb,
                                                   const int32_t* __restrict__ slot, int n, int HF, int ld,
                                                   float* __restrict__ gsend) {
  const int per = HF / 4;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)n * per) return;
  const int b = (int)(i / per), c = (int)(i % per);
  float* dst = gsend + (int64_t)slot[b] * ld;
  reinterpret_cast<f4*>(dst)[c] = reinterpret_cast<const f4*>(grows + (int64_t)b * HF)[c];
  if (c == 0) dst[HF] = gb[b];
}

inline unsigned blocks(int64_t n) { return (unsigned)((n + 255) / 256); }

}  // namespace

// ---------------------------------------------------------------- ABI ----
extern "C" int rg_neg_pick(uint64_t seed, uint64_t counter, int64_t A, int S, int HF, int64_t lo, int64_t hi,
                           const float* W, const float* bias, int32_t* ids, int32_t* nloc, float* Wg, float* bg,
                           hipStream_t stream) {
  if (S <= 0 || A <= 0 || A > INT32_MAX || HF <= 0 || (HF % 8) || lo < 0 || hi < lo || hi > A) return RG_ERR_ARG;
  if (!ids || !nloc || !Wg || !bg || (hi > lo && (!W || !bias))) return RG_ERR_ARG;
  hipLaunchKernelGGL(k_neg_pick, dim3(blocks((int64_t)S * (HF / 8))), dim3(256), 0, stream, seed, counter,
                     (uint64_t)A, S, HF, lo, hi, W, bias, ids, nloc, Wg, bg);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_neg_planes(const float* Wg, int S, int HF, void* Wp, hipStream_t stream) {
  if (S <= 0 || (S % 32) || !Wg || !Wp) return RG_ERR_ARG;
  if (HF != 32 && HF != 64 && HF != 128 && HF != 256) return RG_ERR_SHAPE;
  hipLaunchKernelGGL(k_neg_planes, dim3(blocks((int64_t)S * (HF / 8))), dim3(256), 0, stream, Wg, S, HF,
                     reinterpret_cast<bf16x8*>(Wp));
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_target_ids(const int64_t* tgt, int n, int64_t A, int32_t* out, int32_t* n_out,
                             hipStream_t stream) {
  if (n <= 0 || A <= 0 || !tgt || !out || !n_out) return RG_ERR_ARG;
  hipLaunchKernelGGL(k_target_ids, dim3(blocks(n)), dim3(256), 0, stream, tgt, n, A, out, n_out);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_head_rows_gather(const int32_t* ids, int n, int64_t lo, int64_t n_local, const float* W,
                                   const float* bias, int HF, int ld, float* rows, int32_t* local_ids,
                                   hipStream_t stream) {
  if (n < 0 || HF <= 0 || (HF & 3) || ld < HF + 1 || (ld & 3) || !local_ids || (n > 0 && (!ids || !rows)))
    return RG_ERR_ARG;
  if (n == 0) return RG_OK;
  if (n_local > 0 && (!W || !bias)) return RG_ERR_ARG;
  hipLaunchKernelGGL(k_head_rows_gather, dim3(blocks((int64_t)n * (HF / 4))), dim3(256), 0, stream, ids, n, lo,
                     n_local, W, bias, HF, ld, rows, local_ids);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_rows_unslot(const float* rows, int ld, const int32_t* slot, const int32_t* tid32, int n, int HF,
                              float* tW, float* tb, int64_t* trow, hipStream_t stream) {
  if (n <= 0 || HF <= 0 || (HF & 3) || ld < HF + 1 || (ld & 3) || !rows || !slot || !tid32 || !tW || !tb || !trow)
    return RG_ERR_ARG;
  hipLaunchKernelGGL(k_rows_unslot, dim3(blocks((int64_t)n * (HF / 4))), dim3(256), 0, stream, rows, ld, slot, tid32,
                     n, HF, tW, tb, trow);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_rows_slot(const float* grows, const float* gb, const int32_t* slot, int n, int HF, int ld,
                            float* gsend, hipStream_t stream) {
  if (n <= 0 || HF <= 0 || (HF & 3) || ld < HF + 1 || (ld & 3) || !grows || !gb || !slot || !gsend)
    return RG_ERR_ARG;
  hipLaunchKernelGGL(k_rows_slot, dim3(blocks((int64_t)n * (HF / 4))), dim3(256), 0, stream, grows, gb, slot, n, HF,
                     ld, gsend);
  RG_LAUNCH_CHECK();
  return RG_OK;
}
