// Exact full-row top-K scan: the fallback of the candidate-based top-K
// selections (rg_flash_topk / rg_flash_topk_screened / rg_flash_argmax_exact
// in head_flash.hip, rg_topk in topk.hip) for a row whose candidate set
// overflowed its buffer (massive exact or near ties).  The reference takes
// torch.topk of the full fp32 logit row (evaluate/diversity.py:15-73,
// novelty.py:12-47, eval_protocol.py:75) and torch.argmax for the double-Q
// target (SQN/sqn_gru.py:222-226); a bounded candidate list cannot decide such
// a row, so the row is scanned whole instead of keeping a screened pick.
//
// One 256-thread workgroup per overflowing row: thread t visits items t,
// t + 256, ... (increasing), keeps its own canonical (value desc, index asc)
// top-K list in registers, then K rounds merge the 256 list heads in LDS.
// Cost: one pass over the row's logits (A·HF fp32 reads for the fused head's
// re-scoring) on one CU; only rows that overflowed run it.
#pragma once
#include "common.h"

constexpr int TS_MAX = 32;   // K <= TS_MAX

// logit source: src.prepare(row) once (may stage operands in LDS, ends with
// a barrier), then src(item) for every item of the row
template <class Src>
__device__ __forceinline__ void topk_scan_row(Src& src, int row, int A, int K, int32_t* __restrict__ out_idx,
                                              float* __restrict__ out_val) {
  __shared__ float lv[TS_MAX][256];
  __shared__ int li[TS_MAX][256];
  __shared__ float rv[4];
  __shared__ int ri[4], rt[4];
  __shared__ int s_win;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const float ninf = -__builtin_inff();
  src.prepare(row);
  float tv[TS_MAX];
  int ti[TS_MAX];
#pragma unroll
  for (int i = 0; i < TS_MAX; ++i) {
    tv[i] = ninf;
    ti[i] = INT32_MAX;
  }
  float thr = ninf;   // tv[K-1]
  bool full = false;  // K entries held
  for (int j = tid; j < A; j += 256) {
    const float z = src(j);
    // items arrive in increasing order: an equal value never displaces an
    // entry (that one has the smaller index)
    if (z > thr || (!full && z == z)) {
      float cv = z;
      int ci = j;
      bool ins = false;
#pragma unroll
      for (int i = 0; i < TS_MAX; ++i) {
        if (ins || cv > tv[i] || ti[i] == INT32_MAX) {
          const float t = tv[i];
          const int u = ti[i];
          tv[i] = cv;
          ti[i] = ci;
          cv = t;
          ci = u;
          ins = true;
        }
      }
#pragma unroll
      for (int i = 0; i < TS_MAX; ++i)
        if (i == K - 1) {
          thr = tv[i];
          full = ti[i] != INT32_MAX;
        }
    }
  }
#pragma unroll
  for (int i = 0; i < TS_MAX; ++i) {
    lv[i][tid] = tv[i];
    li[i][tid] = ti[i];
  }
  __syncthreads();
  int pos = 0;
  for (int k = 0; k < K; ++k) {
    float bv = pos < K ? lv[pos][tid] : ninf;
    int bi = pos < K ? li[pos][tid] : INT32_MAX;
    int bt = bi == INT32_MAX ? -1 : tid;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      const float v2 = __shfl_xor(bv, o);
      const int i2 = __shfl_xor(bi, o), t2 = __shfl_xor(bt, o);
      if (t2 >= 0 && (bt < 0 || v2 > bv || (v2 == bv && i2 < bi))) {
        bv = v2;
        bi = i2;
        bt = t2;
      }
    }
    if (lane == 0) {
      rv[w] = bv;
      ri[w] = bi;
      rt[w] = bt;
    }
    __syncthreads();
    if (tid == 0) {
      for (int q = 1; q < 4; ++q)
        if (rt[q] >= 0 && (rt[0] < 0 || rv[q] > rv[0] || (rv[q] == rv[0] && ri[q] < ri[0]))) {
          rv[0] = rv[q];
          ri[0] = ri[q];
          rt[0] = rt[q];
        }
      out_idx[(int64_t)row * K + k] = rt[0] >= 0 ? ri[0] : -1;
      if (out_val) out_val[(int64_t)row * K + k] = rt[0] >= 0 ? rv[0] : ninf;
      s_win = rt[0];
    }
    __syncthreads();
    if (tid == s_win) ++pos;
    __syncthreads();
  }
}
