// Double-Q heads, TD losses and the SMORL online rewards.
//
// Only row a_b of a Q head ever receives gradient (sqn_gru.py:221-222 gathers
// Q(s, a) from the full (B, A) output), so Q(s, a) and its backward are B dot
// products plus a row-sparse scatter — identical math to the reference's
// full GEMM + gather, without the (B, A) tensor.
#include "common.h"

#define MAXH 4
struct HeadPtrs {
  const float* W[MAXH];
  const float* b[MAXH];
};

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) v += __shfl_xor(v, d);
  return v;
}

// q[b*nh + i] = h[b]·W_i[idx_b] + b_i[idx_b]; one wave per batch row.
__global__ __launch_bounds__(256) void k_q_gather(const float* __restrict__ h, int HF, HeadPtrs hp, int nh,
                                                  const int64_t* __restrict__ idx64,
                                                  const int32_t* __restrict__ idx32, int B,
                                                  float* __restrict__ q) {
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (b >= B) return;
  const int64_t j = idx64 ? idx64[b] : (int64_t)idx32[b];
  if (j < 0) {  // not held here (item-sharded head): contributes 0 to the all-reduce
    if (lane < nh) q[(int64_t)b * nh + lane] = 0.f;
    return;
  }
  for (int i = 0; i < nh; ++i) {
    const float* wr = hp.W[i] + j * HF;
    float s = 0.f;
    for (int c = lane; c < HF; c += 64) s += h[(int64_t)b * HF + c] * wr[c];
    s = wave_sum(s);
    if (lane == 0) q[(int64_t)b * nh + i] = s + hp.b[i][j];
  }
}

extern "C" int rg_q_gather(const float* h, int HF, const float* const* W, const float* const* bias, int nh,
                           const int64_t* idx64, const int32_t* idx32, int B, float* q, hipStream_t stream) {
  if (nh <= 0 || nh > MAXH || B <= 0) return RG_ERR_ARG;
  HeadPtrs hp{};
  for (int i = 0; i < nh; ++i) {
    hp.W[i] = W[i];
    hp.b[i] = bias[i];
  }
  hipLaunchKernelGGL(k_q_gather, dim3((B + 3) / 4), dim3(256), 0, stream, h, HF, hp, nh, idx64, idx32, B, q);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

// Backward of q = h·W_i[a] + b_i[a] without float atomics: dh[b] +=
// Σ_i dq_bi W_i[a_b] (heads in order), and the per-row gradient contributions
// rows[i][b] = dq_bi h_b, rows_b[i][b] = dq_bi with ids[b] = a_b (-1 where the
// row's action is not held here, item-sharded heads), n_rows[0] = B.  The
// caller sums them into G_i / Gb_i through the deterministic sorted scatter
// (csrc/segsum.hip rg_scatter_rows, one sort shared by every head): several
// rows of a batch share an action, and an atomic sum would depend on arrival
// order.
__global__ __launch_bounds__(256) void k_q_backward(const float* __restrict__ h, int HF, HeadPtrs hp, int nh,
                                                    const int64_t* __restrict__ idx, int B,
                                                    const float* __restrict__ dq, float* __restrict__ dh,
                                                    float* __restrict__ rows, float* __restrict__ rows_b,
                                                    int32_t* __restrict__ ids, int32_t* __restrict__ n_rows) {
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (blockIdx.x == 0 && threadIdx.x == 0) n_rows[0] = B;
  if (b >= B) return;
  const int64_t j = idx[b];
  if (lane == 0) ids[b] = j < 0 ? -1 : (int32_t)j;
  if (j < 0) return;  // skipped by the scatter (its rows are never read)
  for (int c = lane; c < HF; c += 64) {
    float acc = dh[(int64_t)b * HF + c];
    const float hv = h[(int64_t)b * HF + c];
    for (int i = 0; i < nh; ++i) {
      const float g = dq[(int64_t)b * nh + i];
      acc += g * hp.W[i][j * HF + c];
      rows[((int64_t)i * B + b) * HF + c] = g * hv;
    }
    dh[(int64_t)b * HF + c] = acc;
  }
  if (lane < nh) rows_b[(int64_t)lane * B + b] = dq[(int64_t)b * nh + lane];
}

extern "C" int rg_q_backward(const float* h, int HF, const float* const* W, int nh, const int64_t* idx, int B,
                             const float* dq, float* dh, float* rows, float* rows_b, int32_t* ids, int32_t* n_rows,
                             hipStream_t stream) {
  if (nh <= 0 || nh > MAXH || B <= 0 || HF <= 0 || !rows || !rows_b || !ids || !n_rows) return RG_ERR_ARG;
  HeadPtrs hp{};
  for (int i = 0; i < nh; ++i) hp.W[i] = W[i];
  hipLaunchKernelGGL(k_q_backward, dim3((B + 3) / 4), dim3(256), 0, stream, h, HF, hp, nh, idx, B, dq, dh, rows,
                     rows_b, ids, n_rows);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

// SQN TD term (sqn_gru.py:225-239): qn := 0 where is_end;
// d = r + γ·qn − q evaluated like the reference: γ·qn in f32, then promoted
// to f64 by the f64 reward.  sq[b] = d² (f64), dq[b] = f32(−2·d·scale).
__global__ void k_sqn_td(const float* __restrict__ q, float* __restrict__ qn, const double* __restrict__ r,
                         const uint8_t* __restrict__ is_end, float gamma, int B, double scale, double* __restrict__ sq,
                         float* __restrict__ dq) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  float n = is_end[b] ? 0.0f : qn[b];
  qn[b] = n;
  const float gq = gamma * n;
  const double d = (r[b] + (double)gq) - (double)q[b];
  sq[b] = d * d;
  dq[b] = (float)(-(2.0 * d * scale));
}

extern "C" int rg_sqn_td(const float* q, float* qn, const double* r, const uint8_t* is_end, float gamma, int B,
                         double scale, double* sq, float* dq, hipStream_t stream) {
  if (B <= 0) return RG_ERR_ARG;
  hipLaunchKernelGGL(k_sqn_td, dim3((B + 255) / 256), dim3(256), 0, stream, q, qn, r, is_end, gamma, B, scale, sq,
                     dq);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

// SMORL multi-head TD term (smorl_gru.py:295,317-325 with 3 heads):
// per_head = (r + γ·qn − q)²  (f32), row_b = per_head·w, dq = α/B · w_i · (−2x).
__global__ void k_smorl_td(const float* __restrict__ q, float* __restrict__ qn, const float* __restrict__ r,
                           const uint8_t* __restrict__ is_end, const float* __restrict__ w, int nh, float gamma,
                           float grad_row, int B, float* __restrict__ row_loss, float* __restrict__ dq) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  float acc = 0.f;
  for (int i = 0; i < nh; ++i) {
    const int64_t o = (int64_t)b * nh + i;
    const float n = is_end[b] ? 0.0f : qn[o];
    qn[o] = n;
    const float x = (r[o] + gamma * n) - q[o];
    const float ph = x * x;
    acc = (i == 0) ? ph * w[i] : acc + ph * w[i];
    dq[o] = -((grad_row * w[i]) * 2.0f * x);
  }
  row_loss[b] = acc;
}

extern "C" int rg_smorl_td(const float* q, float* qn, const float* r, const uint8_t* is_end, const float* w, int nh,
                           float gamma, float grad_row, int B, float* row_loss, float* dq, hipStream_t stream) {
  if (B <= 0 || nh <= 0) return RG_ERR_ARG;
  hipLaunchKernelGGL(k_smorl_td, dim3((B + 255) / 256), dim3(256), 0, stream, q, qn, r, is_end, w, nh, gamma,
                     grad_row, B, row_loss, dq);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

// Σ x (f64) · scale, one workgroup, fixed tree.
__global__ __launch_bounds__(1024) void k_sum64(const double* __restrict__ x, int n, double scale,
                                                double* __restrict__ out64, float* __restrict__ out32) {
  __shared__ double red[1024];
  double s = 0.0;
  for (int i = threadIdx.x; i < n; i += 1024) s += x[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int d = 512; d > 0; d >>= 1) {
    if ((int)threadIdx.x < d) red[threadIdx.x] += red[threadIdx.x + d];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    if (out64) out64[0] = red[0] * scale;
    if (out32) out32[0] = (float)(red[0] * scale);
  }
}

extern "C" int rg_sum64(const double* x, int n, double scale, double* out64, float* out32, hipStream_t stream) {
  if (n <= 0) return RG_ERR_ARG;
  hipLaunchKernelGGL(k_sum64, dim3(1), dim3(1024), 0, stream, x, n, scale, out64, out32);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

// Diversity reward (diversity.py:4-73): last = s[b, len_b−1] (end padding)
// or s[b, L−1] (beg); r = 1 − mean_k cos(D[last], D[idx_bk]), cos with
// per-vector norms clamped at eps (torch cosine_similarity).  One wave per row.
// An id outside the table's Drows rows (e.g. -1 from an unmapped tokenizer
// remap, where the reference's stoi raises KeyError) gives a NaN reward and
// is never dereferenced.
__global__ __launch_bounds__(256) void k_diversity(const int64_t* __restrict__ s, int L,
                                                   const int64_t* __restrict__ lens, int pad_end,
                                                   const int32_t* __restrict__ idx, int k, int ldi,
                                                   const float* __restrict__ D, int64_t Drows, int Ed, float eps,
                                                   int B, float* __restrict__ out) {
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (b >= B) return;
  const int64_t li = pad_end ? lens[b] - 1 : L - 1;
  const int64_t last = (li >= 0 && li < L) ? s[(int64_t)b * L + li] : -1;
  bool bad = last < 0 || last >= Drows;
  for (int q = 0; q < k; ++q) {
    const int64_t j = idx[(int64_t)b * ldi + q];
    bad |= j < 0 || j >= Drows;
  }
  if (bad) {   // wave-uniform (every lane read the same ids)
    if (lane == 0) out[b] = __builtin_nanf("");
    return;
  }
  const float* x1 = D + last * Ed;
  float n1 = 0.f;
  for (int c = lane; c < Ed; c += 64) n1 += x1[c] * x1[c];
  n1 = fmaxf(sqrtf(wave_sum(n1)), eps);
  float tot = 0.f;
  for (int q = 0; q < k; ++q) {
    const float* x2 = D + (int64_t)idx[(int64_t)b * ldi + q] * Ed;
    float n2 = 0.f;
    for (int c = lane; c < Ed; c += 64) n2 += x2[c] * x2[c];
    n2 = fmaxf(sqrtf(wave_sum(n2)), eps);
    float d = 0.f;
    for (int c = lane; c < Ed; c += 64) d += (x1[c] / n1) * (x2[c] / n2);
    tot += wave_sum(d);
  }
  if (lane == 0) out[b] = 1.0f - tot / (float)k;
}

extern "C" int rg_diversity(const int64_t* s, int L, const int64_t* lens, int pad_end, const int32_t* idx, int k,
                            int ldi, const float* D, int64_t Drows, int Ed, float eps, int B, float* out,
                            hipStream_t stream) {
  if (B <= 0 || k <= 0 || ldi < k || Drows <= 0 || L <= 0) return RG_ERR_ARG;
  hipLaunchKernelGGL(k_diversity, dim3((B + 3) / 4), dim3(256), 0, stream, s, L, lens, pad_end, idx, k, ldi, D, Drows,
                     Ed, eps, B, out);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

// Novelty reward (novelty.py:12-47): mean_k [idx_bk ∈ U]·reward, U as a bitmap.
__global__ void k_novelty(const int32_t* __restrict__ idx, int k, int ldi, const uint32_t* __restrict__ bitmap,
                          int n_items, float reward, int B, float* __restrict__ out) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  double acc = 0.0;
  for (int q = 0; q < k; ++q) {
    const int j = idx[(int64_t)b * ldi + q];
    if (j < 0 || j >= n_items) {   // not an item (never read from the bitmap): NaN reward
      out[b] = __builtin_nanf("");
      return;
    }
    const bool u = (bitmap[j >> 5] >> (j & 31)) & 1u;
    acc += u ? (double)reward : 0.0;
  }
  out[b] = (float)(acc / k);
}

extern "C" int rg_novelty(const int32_t* idx, int k, int ldi, const uint32_t* bitmap, int n_items, float reward, int B,
                          float* out, hipStream_t stream) {
  if (B <= 0 || k <= 0 || ldi < k || n_items <= 0) return RG_ERR_ARG;
  hipLaunchKernelGGL(k_novelty, dim3((B + 255) / 256), dim3(256), 0, stream, idx, k, ldi, bitmap, n_items, reward, B,
                     out);
  RG_LAUNCH_CHECK();
  return RG_OK;
}
