// Item-sharded heads across ranks: rank r of nr holds
// items [lo_r, hi_r) = [r·A/nr, (r+1)·A/nr) of every head.  Helpers for the
// multi-GPU double-Q step (recommenders/hip/sharded.py):
//
//  k_shard_index       : global action -> local row (or −1 when another rank
//                        holds it); the Q gathers/backward skip −1 rows, so a
//                        SUM all-reduce returns the owner's value bit-exactly.
//  k_argmax_merge_ranks: per row, the global argmax from every rank's (row
//                        maximum, local argmax): larger value wins, equal
//                        values go to the lower rank = the lower global index,
//                        which is torch.argmax's first-maximum rule over the
//                        whole row (every logit is the same k-ordered fma chain
//                        on any rank, so the values compared are identical).
//  k_topk_merge_ranks  : per row, merge nr canonical (value desc, index asc)
//                        local top-k lists into the global canonical top-k.
#include "common.h"

__device__ __forceinline__ int64_t shard_lo(int r, int nr, int64_t A) { return ((int64_t)r * A) / nr; }

__global__ void k_shard_index(const int64_t* __restrict__ idx64, const int32_t* __restrict__ idx32, int n,
                              int64_t lo, int64_t hi, int64_t* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t j = idx64 ? idx64[i] : (int64_t)idx32[i];
  out[i] = (j >= lo && j < hi) ? j - lo : -1;
}

extern "C" int rg_shard_index(const int64_t* idx64, const int32_t* idx32, int n, int64_t lo, int64_t hi,
                              int64_t* out, hipStream_t stream) {
  if (n <= 0 || hi <= lo || (idx64 == nullptr) == (idx32 == nullptr)) return RG_ERR_ARG;
  hipLaunchKernelGGL(k_shard_index, dim3((n + 255) / 256), dim3(256), 0, stream, idx64, idx32, n, lo, hi, out);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

__global__ void k_argmax_merge_ranks(const float* __restrict__ mx, const int32_t* __restrict__ am, int nr, int n,
                                     int64_t A, int32_t* __restrict__ out, float* __restrict__ out_max) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float best = -__builtin_inff();
  int64_t arg = -1;
  for (int r = 0; r < nr; ++r) {
    const int32_t a = am[(int64_t)r * n + i];
    if (a < 0 || a == INT32_MAX) continue;  // empty shard row
    const float v = mx[(int64_t)r * n + i];
    if (arg < 0 || v > best) {  // strict: ties keep the lower rank (lower index)
      best = v;
      arg = shard_lo(r, nr, A) + a;
    }
  }
  out[i] = (int32_t)arg;
  if (out_max) out_max[i] = best;
}

extern "C" int rg_argmax_merge_ranks(const float* mx, const int32_t* am, int nr, int n, int64_t A, int32_t* out,
                                     float* out_max, hipStream_t stream) {
  if (nr <= 0 || n <= 0 || A <= 0) return RG_ERR_ARG;
  hipLaunchKernelGGL(k_argmax_merge_ranks, dim3((n + 255) / 256), dim3(256), 0, stream, mx, am, nr, n, A, out,
                     out_max);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

// One thread per row; the nr lists are each sorted canonically, so a k-step
// merge with (value desc, global index asc) picks the global canonical top-k.
#define TKM_MAXR 64
__global__ void k_topk_merge_ranks(const float* __restrict__ vals, const int32_t* __restrict__ idx, int nr, int n,
                                   int K, int64_t A, int32_t* __restrict__ out_idx, float* __restrict__ out_val) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int pos[TKM_MAXR];
  for (int r = 0; r < nr; ++r) pos[r] = 0;
  for (int q = 0; q < K; ++q) {
    int br = -1;
    float bv = 0.f;
    int64_t bg = 0;
    for (int r = 0; r < nr; ++r) {
      if (pos[r] >= K) continue;
      const int64_t o = ((int64_t)r * n + i) * K + pos[r];
      const int32_t a = idx[o];
      if (a < 0) continue;  // list exhausted (shard smaller than k)
      const float v = vals[o];
      const int64_t g = shard_lo(r, nr, A) + a;
      if (br < 0 || v > bv || (v == bv && g < bg)) {
        br = r;
        bv = v;
        bg = g;
      }
    }
    out_idx[(int64_t)i * K + q] = br < 0 ? -1 : (int32_t)bg;
    if (out_val) out_val[(int64_t)i * K + q] = br < 0 ? -__builtin_inff() : bv;
    if (br >= 0) ++pos[br];
  }
}

extern "C" int rg_topk_merge_ranks(const float* vals, const int32_t* idx, int nr, int n, int K, int64_t A,
                                   int32_t* out_idx, float* out_val, hipStream_t stream) {
  if (nr <= 0 || nr > TKM_MAXR || n <= 0 || K <= 0 || A <= 0) return RG_ERR_ARG;
  hipLaunchKernelGGL(k_topk_merge_ranks, dim3((n + 127) / 128), dim3(128), 0, stream, vals, idx, nr, n, K, A,
                     out_idx, out_val);
  RG_LAUNCH_CHECK();
  return RG_OK;
}
