// Row top-k over the stored logits Zᵀ (SURVEY §8 A12/A13 top-k rewards, A14
// HR@k / NDCG@k).
//
// Reference: torch.topk(preds, k) on a (B, A) tensor copied to the host
// (recommenders/evaluate/eval_protocol.py:75, :199; diversity.py:51;
// novelty.py:33).  Here the (B, A) logits never leave HBM:
//   1. the forward kernel already produced, per row, the maximum of every
//      RG_PBLK-item block (pmax, nJ × B);
//   2. per row, the k-th largest block maximum τ is a lower bound of the row's
//      k-th largest logit (the top-k block maxima are k distinct elements);
//      radix-select it over the (coarsened) block maxima in LDS;
//   3. only blocks whose maximum is ≥ τ can hold a top-k element: scan those
//      blocks' logits, keep the ones ≥ τ as (value, index) candidates;
//   4. bitonic-sort the candidates by (value desc, index asc) and emit k.
// Exact for any data; ties are broken by the smaller index (canonical order).
// A row with more than TK_MAXCAND logits >= tau (massive ties) is scanned
// whole instead (k <= TS_MAX, k_topk_zscan, topk_scan.h); beyond that k it
// raises err |= 2.
#include "common.h"
#include "topk_scan.h"

#define TK_THREADS 256
#define TK_MAXSEL 8192
#define TK_MAXCAND 2048
#define TK_SCAN_MARK INT32_MIN

__device__ __forceinline__ uint32_t f2key(float f) {
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);  // order-preserving
}
__device__ __forceinline__ float key2f(uint32_t k) {
  uint32_t u = (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k;
  return __uint_as_float(u);
}

// one workgroup per row b
__global__ __launch_bounds__(TK_THREADS) void k_topk(const float* __restrict__ ZT, int64_t ldz,
                                                     const float* __restrict__ pmax, int B, int A, int nJ, int coarse,
                                                     int k, int32_t* __restrict__ out_idx,
                                                     float* __restrict__ out_val, int32_t* __restrict__ err) {
  __shared__ uint32_t sel[TK_MAXSEL];
  __shared__ uint32_t hist[256];
  __shared__ uint64_t cand[TK_MAXCAND];
  __shared__ uint32_t s_prefix, s_rank, s_ncand;
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const int nS = (nJ + coarse - 1) / coarse;  // coarsened block count (≤ TK_MAXSEL)
  for (int i = tid; i < nS; i += TK_THREADS) {
    float m = -__builtin_inff();
    for (int c = 0; c < coarse; ++c) {
      int jb = i * coarse + c;
      if (jb < nJ) m = fmaxf(m, pmax[(int64_t)jb * B + b]);
    }
    sel[i] = f2key(m);
  }
  // k <= nS: select over the block maxima (a lower bound of the k-th logit);
  // otherwise (tiny A) select directly over the row's A logits.
  const bool by_block = k <= nS;
  const int nsel = by_block ? nS : A;
  if (tid == 0) {
    s_prefix = 0;
    s_rank = (uint32_t)min(k, nsel);  // want the s_rank-th largest key
  }
  __syncthreads();
  // radix select, 8 bits per pass, most significant first
  for (int shift = 24; shift >= 0; shift -= 8) {
    hist[tid] = 0;
    __syncthreads();
    const uint32_t pre = s_prefix;
    const uint32_t mask = (shift == 24) ? 0u : (0xffffffffu << (shift + 8));
    for (int i = tid; i < nsel; i += TK_THREADS) {
      const uint32_t key = by_block ? sel[i] : f2key(ZT[(int64_t)i * ldz + b]);
      if ((key & mask) == (pre & mask)) atomicAdd(&hist[(key >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (tid == 0) {
      uint32_t r = s_rank, acc = 0;
      int d = 255;
      for (; d > 0; --d) {
        if (acc + hist[d] >= r) break;
        acc += hist[d];
      }
      s_prefix = pre | ((uint32_t)d << shift);
      s_rank = r - acc;
    }
    __syncthreads();
  }
  const float tau = key2f(s_prefix);
  if (tid == 0) s_ncand = 0;
  __syncthreads();
  // gather candidates ≥ τ from qualifying blocks (one wave per block)
  const int wv = tid >> 6, lane = tid & 63;
  for (int i = wv; i < nS; i += TK_THREADS / 64) {
    if (by_block && sel[i] < s_prefix) continue;  // block maximum < τ
    const int j0 = i * coarse * RG_PBLK;
    const int j1 = min(A, j0 + coarse * RG_PBLK);
    for (int j = j0 + lane; j < j1; j += 64) {
      const float z = ZT[(int64_t)j * ldz + b];
      if (z >= tau) {
        uint32_t slot = atomicAdd(&s_ncand, 1u);
        // pack (key desc, index asc) so that a descending sort is the canonical order
        if (slot < TK_MAXCAND) cand[slot] = ((uint64_t)f2key(z) << 32) | (uint32_t)(0x7fffffffu - (uint32_t)j);
      }
    }
  }
  __syncthreads();
  uint32_t n = s_ncand;
  if (n > TK_MAXCAND) {
    if (k <= TS_MAX) {   // left to k_topk_zscan
      if (tid == 0) out_idx[(int64_t)b * k] = TK_SCAN_MARK;
      return;
    }
    if (tid == 0 && err) atomicOr(err, 2);
    n = TK_MAXCAND;
  }
  int np2 = 1;
  while (np2 < (int)n) np2 <<= 1;
  for (int i = n + tid; i < np2; i += TK_THREADS) cand[i] = 0;  // smallest possible
  __syncthreads();
  // bitonic sort, descending
  for (int size = 2; size <= np2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = tid; i < np2; i += TK_THREADS) {
        int p = i ^ stride;
        if (p > i) {
          const bool desc = (i & size) == 0;
          uint64_t x = cand[i], y = cand[p];
          if ((x < y) == desc) {
            cand[i] = y;
            cand[p] = x;
          }
        }
      }
      __syncthreads();
    }
  }
  for (int q = tid; q < k; q += TK_THREADS) {
    const uint64_t c = (q < (int)n) ? cand[q] : 0;
    out_idx[(int64_t)b * k + q] = (q < (int)n) ? (int32_t)(0x7fffffffu - (uint32_t)(c & 0xffffffffu)) : -1;
    if (out_val) out_val[(int64_t)b * k + q] = (q < (int)n) ? key2f((uint32_t)(c >> 32)) : -__builtin_inff();
  }
}

// the rows k_topk marked (candidate overflow): full scan of the stored row
struct ZtRowSrc {
  const float* ZT;
  int64_t ldz;
  int row;
  __device__ void prepare(int r) { row = r; }
  __device__ float operator()(int item) const { return ZT[(int64_t)item * ldz + row]; }
};

__global__ __launch_bounds__(256) void k_topk_zscan(const float* __restrict__ ZT, int64_t ldz, int A, int k,
                                                    int32_t* __restrict__ out_idx, float* __restrict__ out_val) {
  const int b = blockIdx.x;
  if (out_idx[(int64_t)b * k] != TK_SCAN_MARK) return;
  ZtRowSrc src{ZT, ldz, b};
  topk_scan_row(src, b, A, k, out_idx, out_val);
}

extern "C" int rg_topk(const float* ZT, int64_t ldz, const float* pmax, int B, int A, int k, int32_t* out_idx,
                       float* out_val, int32_t* err, hipStream_t stream) {
  if (B <= 0 || A <= 0 || k <= 0 || k > 1024 || k > A) return RG_ERR_ARG;
  const int nJ = (A + RG_PBLK - 1) / RG_PBLK;
  const int coarse = (nJ + TK_MAXSEL - 1) / TK_MAXSEL;
  hipLaunchKernelGGL(k_topk, dim3(B), dim3(TK_THREADS), 0, stream, ZT, ldz, pmax, B, A, nJ, coarse, k, out_idx,
                     out_val, err);
  if (k <= TS_MAX)
    hipLaunchKernelGGL(k_topk_zscan, dim3(B), dim3(TK_THREADS), 0, stream, ZT, ldz, A, k, out_idx, out_val);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

// HR@k / NDCG@k sums over a batch (eval_protocol.py:26-100): rank = 1 + first
// position of the target in the top-max(k) list, hit if rank <= k,
// ndcg += 1/log2(rank+1).  ks: HOST array (≤ 16 values).  out (2*nk doubles)
// = [hits_k..., ndcg_k...] accumulated (+=) so a whole eval set can be summed.
struct KList {
  int k[16];
};
__global__ __launch_bounds__(256) void k_hits(const int32_t* __restrict__ idx, int K, const int64_t* __restrict__ tgt,
                                              int B, KList ks, int nk, double* __restrict__ out) {
  __shared__ double red[2 * 16][256];
  double h[16], n[16];
  for (int q = 0; q < nk; ++q) h[q] = n[q] = 0.0;
  for (int b = threadIdx.x; b < B; b += 256) {
    int rank = 0;
    for (int q = 0; q < K; ++q)
      if (idx[(int64_t)b * K + q] == tgt[b]) {
        rank = q + 1;
        break;
      }
    for (int q = 0; q < nk; ++q)
      if (rank > 0 && rank <= ks.k[q]) {
        h[q] += 1.0;
        n[q] += 1.0 / log2((double)rank + 1.0);
      }
  }
  for (int q = 0; q < nk; ++q) {
    red[q][threadIdx.x] = h[q];
    red[16 + q][threadIdx.x] = n[q];
  }
  __syncthreads();
  if (threadIdx.x < 2 * nk) {
    const int row = threadIdx.x < nk ? threadIdx.x : 16 + threadIdx.x - nk;
    double s = 0.0;
    for (int i = 0; i < 256; ++i) s += red[row][i];
    out[threadIdx.x] += s;
  }
}

extern "C" int rg_hits_ndcg(const int32_t* idx, int K, const int64_t* tgt, int B, const int* ks, int nk, double* out,
                            hipStream_t stream) {
  if (B <= 0 || nk <= 0 || nk > 16) return RG_ERR_ARG;
  KList kl{};
  for (int q = 0; q < nk; ++q) {
    if (ks[q] <= 0 || ks[q] > K) return RG_ERR_ARG;
    kl.k[q] = ks[q];
  }
  hipLaunchKernelGGL(k_hits, dim3(1), dim3(256), 0, stream, idx, K, tgt, B, kl, nk, out);
  RG_LAUNCH_CHECK();
  return RG_OK;
}
