// Row-sharded item-embedding table for the multi-GPU step (SURVEY §8e;
// reference table: recommenders/models/GRU4Rec/model.py:35-47 nn.Embedding,
// gathered at :69, dense gradient + Adam at :150-153).
//
// Rank r owns the contiguous rows [lo_r, hi_r) of the (N+1) × E table with
// lo_r = ⌊r·(N+1)/world⌋ (recommenders/hip/dist.py item_shard), plus their
// Adam moments and gradient rows.  A trunk pass exchanges each DISTINCT id of
// its batch once (a C2 batch: ~88K tokens, ~1.7K distinct items):
//
//   rg_token_ids      packed token t -> item id (forward time order)
//   rg_shard_dedup    (csrc/segsum.hip) the distinct ids sorted — grouped by
//                     owner — uslot[t] = the token's distinct index, counts
//   (host: all_to_all of the distinct ids; the splits come from the host batch)
//   rg_rows_gather    owner side: rows of the received ids from the local
//                     shard (fp32 or the fp16 storage copy), local row ids
//   (host: all_to_all of the rows back)
//   rg_place_rows     requester: X[d][t] = rows_in[uslot[t]] (d = 1: the
//                     row's valid prefix reversed, BidirGRU4Rec)
// and in the backward:
//   rg_combine_dirs   (Bidir) dX[0][t] += dX[1][rev t]
//   rg_shard_dedup_grads  gsend[u] = Σ over the tokens of distinct id u, in
//                     token order (csrc/segsum.hip)
//   (host: all_to_all of the per-id row-gradients to their owners)
//   then rg_scatter_rows into the local gradient rows and rg_adam_rows over
//   the local shard (csrc/segsum.hip, csrc/optim.hip).
// No item-sized table is ever all-reduced.  (rg_shard_route, a per-row stable
// partition by owner, routes the sharded sampled head's B targets.)
#include "common.h"
#include <hip/hip_fp16.h>

namespace {

// one workgroup per sorted row r: tok_id[offs[r] + t] = s[perm[r]][t] (ids
// outside [0, n_rows) -> -1 and the err flag, as nn.Embedding raises)
__global__ __launch_bounds__(256) void k_token_ids(const int64_t* __restrict__ s, int L,
                                                   const int32_t* __restrict__ perm,
                                                   const int32_t* __restrict__ lsort,
                                                   const int32_t* __restrict__ offs, int64_t n_rows,
                                                   int32_t* __restrict__ tok_id, int32_t* __restrict__ err) {
  const int r = blockIdx.x;
  const int b = perm[r], len = lsort[r], base = offs[r];
  for (int t = threadIdx.x; t < len; t += blockDim.x) {
    const int64_t id = s[(int64_t)b * L + t];
    const bool ok = id >= 0 && id < n_rows;
    tok_id[base + t] = ok ? (int32_t)id : -1;
    if (!ok && err) atomicOr(err, 1);
  }
}

// Stable partition of the T tokens by owner (one workgroup, 1024 threads,
// each a contiguous token range; the per-owner offsets by a shuffle scan):
// counts[o], slot[t], send_ids[slot[t]].
// Invalid ids (-1) go to rank 0, whose gather returns a zero row for them.
// Deterministic: the send order is the packed token order within each owner.
constexpr int RT_THREADS = 1024;
constexpr int RT_MAXW = 8;    // ranks of one node

__global__ __launch_bounds__(RT_THREADS) void k_shard_route(const int32_t* __restrict__ tok_id,
                                                            const int32_t* __restrict__ ntok_ptr, int64_t N1, int W,
                                                            int32_t* __restrict__ slot,
                                                            int32_t* __restrict__ send_ids,
                                                            int32_t* __restrict__ counts) {
  __shared__ int wtot[RT_THREADS / 64][RT_MAXW];   // per (wave, owner) totals
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int T = *ntok_ptr;
  const int per = (T + RT_THREADS - 1) / RT_THREADS;
  const int t0 = min(T, tid * per), t1 = min(T, t0 + per);
  // owner boundaries ⌊r·N1/W⌋ (the owner of id is the number of boundaries
  // r >= 1 at or below it): compares per token instead of a 64-bit division
  int bnd[RT_MAXW];
#pragma unroll
  for (int r = 1; r < RT_MAXW; ++r) bnd[r] = r < W ? (int)(((int64_t)r * N1) / W) : INT32_MAX;
  auto owner = [&](int id) {
    int o = 0;
#pragma unroll
    for (int r = 1; r < RT_MAXW; ++r) o += id >= bnd[r];
    return id < 0 ? 0 : o;
  };
  int cnt[RT_MAXW];
#pragma unroll
  for (int o = 0; o < RT_MAXW; ++o) cnt[o] = 0;
  for (int t = t0; t < t1; ++t) {
    const int id = tok_id[t];
    const int o = owner(id);
#pragma unroll
    for (int q = 0; q < RT_MAXW; ++q) cnt[q] += q == o;
  }
  // exclusive scan over the threads (token order), per owner: wave shuffles,
  // then the waves' totals through LDS
  int pre[RT_MAXW];
#pragma unroll
  for (int o = 0; o < RT_MAXW; ++o) {
    int x = cnt[o];
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int y = __shfl_up(x, d);
      if (lane >= d) x += y;
    }
    pre[o] = x - cnt[o];
    if (lane == 63) wtot[wv][o] = x;
  }
  __syncthreads();
  int base = 0;
#pragma unroll
  for (int o = 0; o < RT_MAXW; ++o) {
    int tot = 0, before = 0;
#pragma unroll
    for (int q = 0; q < RT_THREADS / 64; ++q) {
      const int v = wtot[q][o];
      before += q < wv ? v : 0;
      tot += v;
    }
    if (tid == 0 && o < W) counts[o] = tot;
    pre[o] += base + before;   // the owner's base in the send buffer + the earlier threads' tokens
    base += o < W ? tot : 0;
  }
  for (int t = t0; t < t1; ++t) {
    const int id = tok_id[t];
    const int o = owner(id);
    int p = 0;
#pragma unroll
    for (int q = 0; q < RT_MAXW; ++q)
      if (q == o) p = pre[q]++;
    slot[t] = p;
    send_ids[p] = id;
  }
}

// owner side: rows of n received ids (global row ids) from the local shard
// [lo, lo + n_local); local_ids[i] = id − lo (−1 and a zero row when the id
// is not held here: an invalid token).  half: the table and the rows are fp16.
template <typename TE>
__global__ __launch_bounds__(256) void k_rows_gather(const int32_t* __restrict__ ids, int n, int64_t lo,
                                                     int64_t n_local, const TE* __restrict__ table, int E,
                                                     TE* __restrict__ rows, int32_t* __restrict__ local_ids) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int per = E / 4;  // 4 values per thread
  if (i >= (int64_t)n * per) return;
  const int k = (int)(i / per), c = (int)(i % per);
  const int64_t l = (int64_t)ids[k] - lo;
  const bool ok = ids[k] >= 0 && l >= 0 && l < n_local;
  if (c == 0) local_ids[k] = ok ? (int32_t)l : -1;
  if (sizeof(TE) == 4) {
    f4 v = {0.f, 0.f, 0.f, 0.f};
    if (ok) v = reinterpret_cast<const f4*>(table + l * E)[c];
    reinterpret_cast<f4*>(rows + (int64_t)k * E)[c] = v;
  } else {
    uint2 v = {0u, 0u};
    if (ok) v = reinterpret_cast<const uint2*>(table + l * E)[c];
    reinterpret_cast<uint2*>(rows + (int64_t)k * E)[c] = v;
  }
}

__device__ __forceinline__ f4 load_row4(const float* p, int c) { return reinterpret_cast<const f4*>(p)[c]; }
__device__ __forceinline__ f4 load_row4(const __half* p, int c) {
  const uint2 u = reinterpret_cast<const uint2*>(p)[c];
  const float2 a = __half22float2(*reinterpret_cast<const __half2*>(&u.x));
  const float2 b = __half22float2(*reinterpret_cast<const __half2*>(&u.y));
  return f4{a.x, a.y, b.x, b.y};
}

// requester side: X[offs[r] + τ] = rows_in[slot[offs[r] + (reverse ? len−1−τ : τ)]]
template <typename TE>
__global__ __launch_bounds__(256) void k_place_rows(const TE* __restrict__ rows_in, const int32_t* __restrict__ slot,
                                                    const int32_t* __restrict__ lsort,
                                                    const int32_t* __restrict__ offs, int E, int reverse,
                                                    float* __restrict__ X) {
  const int r = blockIdx.x;
  const int len = lsort[r], base = offs[r];
  const int v4 = E / 4;
  for (int e = threadIdx.x; e < len * v4; e += blockDim.x) {
    const int tau = e / v4, c = e % v4;
    const int t = base + (reverse ? len - 1 - tau : tau);
    reinterpret_cast<f4*>(X + (int64_t)(base + tau) * E)[c] = load_row4(rows_in + (int64_t)slot[t] * E, c);
  }
}

// backward, Bidir: dX0[t] += dX1[rev(t)] in place (the token's gradient of both
// directions, before the per-distinct-id sums of rg_shard_dedup_grads)
__global__ __launch_bounds__(256) void k_combine_dirs(float* __restrict__ dX0, const float* __restrict__ dX1,
                                                      const int32_t* __restrict__ lsort,
                                                      const int32_t* __restrict__ offs, int E) {
  rg_main_prio();
  const int r = blockIdx.x;
  const int len = lsort[r], base = offs[r];
  const int v4 = E / 4;
  for (int e = threadIdx.x; e < len * v4; e += blockDim.x) {
    const int tau = e / v4, c = e % v4;
    f4* d = reinterpret_cast<f4*>(dX0 + (int64_t)(base + tau) * E) + c;
    *d += reinterpret_cast<const f4*>(dX1 + (int64_t)(base + len - 1 - tau) * E)[c];
  }
}

}  // namespace

// ---------------------------------------------------------------- ABI ----
extern "C" int rg_token_ids(const int64_t* s, int B, int L, const int32_t* perm, const int32_t* lsort,
                            const int32_t* offs, int64_t n_rows, int32_t* tok_id, int32_t* err, hipStream_t stream) {
  if (B <= 0 || L <= 0 || !s || !perm || !lsort || !offs || !tok_id) return RG_ERR_ARG;
  hipLaunchKernelGGL(k_token_ids, dim3(B), dim3(64), 0, stream, s, L, perm, lsort, offs, n_rows, tok_id, err);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_shard_route(const int32_t* tok_id, const int32_t* ntok_ptr, int64_t n_rows, int world,
                              int32_t* slot, int32_t* send_ids, int32_t* counts, hipStream_t stream) {
  if (world <= 0 || world > RT_MAXW || n_rows < world || !tok_id || !ntok_ptr || !slot || !send_ids || !counts)
    return RG_ERR_ARG;
  hipLaunchKernelGGL(k_shard_route, dim3(1), dim3(RT_THREADS), 0, stream, tok_id, ntok_ptr, n_rows, world, slot,
                     send_ids, counts);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_rows_gather(const int32_t* ids, int n, int64_t lo, int64_t n_local, const void* table, int E,
                              int half, void* rows, int32_t* local_ids, hipStream_t stream) {
  if (n < 0 || E <= 0 || (E & 3) || !table || !local_ids || (n > 0 && (!ids || !rows))) return RG_ERR_ARG;
  if (n == 0) return RG_OK;
  const unsigned grid = (unsigned)(((int64_t)n * (E / 4) + 255) / 256);
  if (half)
    hipLaunchKernelGGL(k_rows_gather<__half>, dim3(grid), dim3(256), 0, stream, ids, n, lo, n_local,
                       (const __half*)table, E, (__half*)rows, local_ids);
  else
    hipLaunchKernelGGL(k_rows_gather<float>, dim3(grid), dim3(256), 0, stream, ids, n, lo, n_local,
                       (const float*)table, E, (float*)rows, local_ids);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_place_rows(const void* rows_in, int half, const int32_t* slot, const int32_t* lsort,
                             const int32_t* offs, int B, int E, int reverse, float* X, hipStream_t stream) {
  if (B <= 0 || E <= 0 || (E & 3) || !rows_in || !slot || !lsort || !offs || !X) return RG_ERR_ARG;
  if (half)
    hipLaunchKernelGGL(k_place_rows<__half>, dim3(B), dim3(256), 0, stream, (const __half*)rows_in, slot, lsort,
                       offs, E, reverse, X);
  else
    hipLaunchKernelGGL(k_place_rows<float>, dim3(B), dim3(256), 0, stream, (const float*)rows_in, slot, lsort, offs,
                       E, reverse, X);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_combine_dirs(float* dX0, const float* dX1, const int32_t* lsort, const int32_t* offs, int B, int E,
                               hipStream_t stream) {
  if (B <= 0 || E <= 0 || (E & 3) || !dX0 || !dX1 || !lsort || !offs) return RG_ERR_ARG;
  hipLaunchKernelGGL(k_combine_dirs, dim3(B), dim3(256), 0, stream, dX0, dX1, lsort, offs, E);
  RG_LAUNCH_CHECK();
  return RG_OK;
}
