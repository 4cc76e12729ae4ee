// Small elementwise helpers on the step path (dropout mask, SMORL head
// combination) and the ABI version probe.
#include "common.h"

__global__ void k_mask_scale(const float* __restrict__ x, const float* __restrict__ mask, float scale, int64_t n,
                             float* __restrict__ y) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    y[i] = x[i] * (mask[i] * scale);
}

extern "C" int rg_mask_scale(const float* x, const float* mask, float scale, int64_t n, float* y,
                             hipStream_t stream) {
  if (n <= 0) return RG_ERR_ARG;
  int blocks = (int)((n + 255) / 256);
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(k_mask_scale, dim3(blocks), dim3(256), 0, stream, x, mask, scale, n, y);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

struct Ptr4 {
  const float* p[4];
  float w[4];
};

__global__ void k_weighted_sum(Ptr4 in, int nh, int64_t n, float* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float s = in.p[0][i] * in.w[0];
    for (int k = 1; k < nh; ++k) s = s + in.p[k][i] * in.w[k];
    out[i] = s;
  }
}

// X: HOST array of nh device pointers; w: HOST array of nh weights.
extern "C" int rg_weighted_sum(const float* const* X, const float* w, int nh, int64_t n, float* out,
                               hipStream_t stream) {
  if (nh <= 0 || nh > 4 || n <= 0) return RG_ERR_ARG;
  Ptr4 in{};
  for (int k = 0; k < nh; ++k) {
    in.p[k] = X[k];
    in.w[k] = w[k];
  }
  int blocks = (int)((n + 255) / 256);
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL(k_weighted_sum, dim3(blocks), dim3(256), 0, stream, in, nh, n, out);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

// The SMORL double-Q target's combined head in one pass over the nh Q heads
// (tensor_operations.py:50-70 through the weighted argmax): per (item row x,
// 8-value group g) the same fp32 sum as k_weighted_sum (W_0·w_0 + W_1·w_1 +
// ..., in head order: bitwise rg_weighted_sum's W_comb), written as fp32
// (the exact re-scoring reads it) and as its three bf16 K-planes (the
// screening argmax's operand, common.h kplane16: bitwise rg_head_planes);
// the biases likewise into b_comb and the −inf-padded bias; and the largest
// row norm ||W_comb[x]||₂ (the screening's error bound): a running max per
// lane over a grid-stride loop, reduced per block through LDS, then one
// atomicMax of the non-negative float bits per block (order-independent:
// deterministic; one atomic per wave serialised ~A/4 atomics on one address).
// Replaces rg_weighted_sum (W, b) + rg_head_planes + rg_row_norm_max: the Q
// heads are read once and W_comb is not re-read.
template <int HF, int NP>
__global__ __launch_bounds__(256) void k_qcomb(Ptr4 in, Ptr4 inb, int nh, int A, int Ap, float* __restrict__ Wc,
                                               float* __restrict__ bc, bf16x8* __restrict__ P,
                                               float* __restrict__ bias_pad, float* __restrict__ wnorm) {
  constexpr int G = HF / 8;   // threads per item row (a power of two dividing 64)
  __shared__ float red[4];
  float best = 0.f;
  // Ap·G is a multiple of 64 and the stride of 256, so every wave is wholly
  // inside or outside the range: the shuffles below see full waves.
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < (int64_t)Ap * G; i += (int64_t)gridDim.x * 256) {
    const int x = (int)(i / G), g = (int)(i % G);
    f4 lo = {0.f, 0.f, 0.f, 0.f}, hi = lo;
    float ss = 0.f;
    if (x < A) {
      const int64_t off = (int64_t)x * HF + 8 * g;
      lo = *reinterpret_cast<const f4*>(in.p[0] + off) * in.w[0];
      hi = *reinterpret_cast<const f4*>(in.p[0] + off + 4) * in.w[0];
      for (int k = 1; k < nh; ++k) {
        lo = lo + *reinterpret_cast<const f4*>(in.p[k] + off) * in.w[k];
        hi = hi + *reinterpret_cast<const f4*>(in.p[k] + off + 4) * in.w[k];
      }
      *reinterpret_cast<f4*>(Wc + off) = lo;
      *reinterpret_cast<f4*>(Wc + off + 4) = hi;
#pragma unroll
      for (int u = 0; u < 4; ++u) ss = fmaf(lo[u], lo[u], fmaf(hi[u], hi[u], ss));
      if (g == 0) {
        float sb = inb.p[0][x] * inb.w[0];
        for (int k = 1; k < nh; ++k) sb = sb + inb.p[k][x] * inb.w[k];
        bc[x] = sb;
        bias_pad[x] = sb;
      }
    } else if (g == 0) {
      bias_pad[x] = -__builtin_inff();
    }
    // (rows past A: zero planes, as rg_head_planes pads the last chunk)
    bf16x8 p0, p1, p2;
    split3x8(lo, hi, p0, p1, p2);
    const int64_t base = kplane16(x, g, HF);
    P[base] = p0;
    if (NP == 3) {   // (NP = 1: the one-product screening reads plane 0 only)
      P[base + 64] = p1;
      P[base + 128] = p2;
    }
#pragma unroll
    for (int o = G / 2; o >= 1; o >>= 1) ss += __shfl_xor(ss, o);
    best = fmaxf(best, sqrtf(ss));
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) best = fmaxf(best, __shfl_xor(best, o));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = best;
  __syncthreads();
  if (threadIdx.x == 0)
    atomicMax(reinterpret_cast<unsigned int*>(wnorm),
              __float_as_uint(fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]))));
}

extern "C" int rg_qcomb(const float* const* W, const float* const* b, const float* w, int nh, int A, int HF,
                        int nplanes, float* Wc, float* bc, void* planes_k, float* bias_pad, float* wnorm,
                        hipStream_t stream) {
  if (nh <= 0 || nh > 4 || A <= 0 || (nplanes != 1 && nplanes != 3) || !W || !b || !w || !Wc || !bc || !planes_k ||
      !bias_pad || !wnorm)
    return RG_ERR_ARG;
  if (HF != 32 && HF != 64 && HF != 128 && HF != 256) return RG_ERR_SHAPE;
  Ptr4 in{}, inb{};
  for (int k = 0; k < nh; ++k) {
    in.p[k] = W[k];
    inb.p[k] = b[k];
    in.w[k] = inb.w[k] = w[k];
  }
  if (hipMemsetAsync(wnorm, 0, sizeof(float), stream) != hipSuccess) return RG_ERR_LAUNCH;
  const int Ap = (A + 31) / 32 * 32;
  int64_t need = ((int64_t)Ap * (HF / 8) + 255) / 256;
  const unsigned grid = (unsigned)(need < 4096 ? need : 4096);
#define QC1(HFV, NPV)                                                                                     \
  hipLaunchKernelGGL((k_qcomb<HFV, NPV>), dim3(grid), dim3(256), 0, stream, in, inb, nh, A, Ap, Wc, bc,  \
                     reinterpret_cast<bf16x8*>(planes_k), bias_pad, wnorm)
#define QC(HFV)        \
  if (nplanes == 1) {  \
    QC1(HFV, 1);       \
  } else {             \
    QC1(HFV, 3);       \
  }
  switch (HF) {
    case 32: QC(32); break;
    case 64: QC(64); break;
    case 128: QC(128); break;
    case 256: QC(256); break;
  }
#undef QC
#undef QC1
  RG_LAUNCH_CHECK();
  return RG_OK;
}

// 2: the changes listed in INTEGRATION.md §3 (argument lists of rg_scatter_rows, rg_gather_neg,
// rg_flash_amax_screen, rg_head_rows_gather, rg_rows_unslot, rg_rows_slot; rg_collect_grads
// removed; rg_flash_rows' per-chunk record layout; the catch-up Adam entry points)
extern "C" int rg_abi_version(void) { return 2; }

// SMORL reward matrix r = stack([r_acc, r_div, r_nov], 1).to(float32)
// (smorl_gru.py:311-314 with the third reward): f64 -> f32 per column.
__global__ void k_stack_rewards(const double* __restrict__ r_acc, const float* __restrict__ r_div,
                                const float* __restrict__ r_nov, int B, float* __restrict__ r) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  r[3 * b + 0] = (float)r_acc[b];
  r[3 * b + 1] = r_div[b];
  r[3 * b + 2] = r_nov[b];
}

extern "C" int rg_stack_rewards(const double* r_acc, const float* r_div, const float* r_nov, int B, float* r,
                                hipStream_t stream) {
  if (B <= 0) return RG_ERR_ARG;
  hipLaunchKernelGGL(k_stack_rewards, dim3((B + 255) / 256), dim3(256), 0, stream, r_acc, r_div, r_nov, B, r);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

// Tokenizer remap of predicted ids (output vocabulary -> input vocabulary,
// diversity.py:55-60, repetitiveness.py:42-47): out[i] = lut[idx[i]] with
// lut[j] = input_tokenizer.stoi(output_tokenizer.itos(j)) built once on the
// host.  An id outside the table or mapped to -1 (no such string, no <unk>:
// the reference raises there) gives -1 and sets err.
__global__ void k_remap_ids(const int32_t* __restrict__ idx, int64_t n, const int32_t* __restrict__ lut,
                            int64_t lut_n, int32_t* __restrict__ out, int32_t* __restrict__ err) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int32_t j = idx[i];
  const int32_t v = (j >= 0 && j < lut_n) ? lut[j] : -1;
  out[i] = v;
  if (v < 0 && err) atomicOr(err, 1);
}

extern "C" int rg_remap_ids(const int32_t* idx, int64_t n, const int32_t* lut, int64_t lut_n, int32_t* out,
                            int32_t* err, hipStream_t stream) {
  if (n <= 0 || lut_n <= 0 || !idx || !lut || !out) return RG_ERR_ARG;
  hipLaunchKernelGGL(k_remap_ids, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, idx, n, lut, lut_n, out,
                     err);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

// Repetition counts (repetitiveness.py:21-57): for every k of ks, the number
// of (state slot, top-k prediction) pairs with s[b, t] == idx[b, j], j < k,
// summed over the batch.  One wave per row, lanes over the L slots; integer
// counts (order-free atomics on 64-bit integers: deterministic).
constexpr int REP_MAXK = 16;
struct RepKs {
  int k[REP_MAXK];
};
__global__ __launch_bounds__(256) void k_repetitions(const int64_t* __restrict__ s, int L,
                                                     const int32_t* __restrict__ idx, int K, int B, RepKs ks, int nk,
                                                     unsigned long long* __restrict__ out) {
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (b >= B) return;
  unsigned cnt[REP_MAXK];
#pragma unroll
  for (int q = 0; q < REP_MAXK; ++q) cnt[q] = 0;
  for (int t = lane; t < L; t += 64) {
    const int64_t v = s[(int64_t)b * L + t];
    for (int j = 0; j < K; ++j) {
      if (v == (int64_t)idx[(int64_t)b * K + j]) {
#pragma unroll
        for (int q = 0; q < REP_MAXK; ++q)
          if (q < nk && j < ks.k[q]) ++cnt[q];
      }
    }
  }
#pragma unroll
  for (int q = 0; q < REP_MAXK; ++q) {
    if (q >= nk) break;
    unsigned c = cnt[q];
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) c += __shfl_xor(c, o);
    if (lane == 0 && c) atomicAdd(&out[q], (unsigned long long)c);
  }
}

extern "C" int rg_repetitions(const int64_t* s, int L, const int32_t* idx, int K, int B, const int* ks, int nk,
                              unsigned long long* out, hipStream_t stream) {
  if (B <= 0 || L <= 0 || K <= 0 || nk <= 0 || nk > REP_MAXK || !s || !idx || !ks || !out) return RG_ERR_ARG;
  RepKs kk{};
  for (int q = 0; q < nk; ++q) {
    if (ks[q] <= 0 || ks[q] > K) return RG_ERR_ARG;
    kk.k[q] = ks[q];
  }
  hipLaunchKernelGGL(k_repetitions, dim3((B + 3) / 4), dim3(256), 0, stream, s, L, idx, K, B, kk, nk, out);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

// items per online-softmax partial block of rg_head_fwd (pmax/psum/parg are
// ceil(A / rg_partial_block()) × B)
extern "C" int rg_partial_block(void) { return RG_PBLK; }

hipEvent_t rg_tev0 = nullptr, rg_tev1 = nullptr;

// arm (or, with NULLs, disarm) kernel-exact timing for the next RG_TLAUNCH
// launch; returns 1 when the previous arming was still pending (no RG_TLAUNCH
// launch consumed it), else 0
extern "C" int rg_timing_events(void* start, void* stop) {
  if ((start == nullptr) != (stop == nullptr)) return RG_ERR_ARG;
  const int pending = rg_tev0 != nullptr ? 1 : 0;
  rg_tev0 = (hipEvent_t)start;
  rg_tev1 = (hipEvent_t)stop;
  return pending;
}
