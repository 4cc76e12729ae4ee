// Dense Adam sweeps.
//
// Reference: torch.optim.Adam over every parameter, dense gradients
// (GRU4Rec/model.py:124-127,149-153; sqn_gru.py:173-181,248-252).  The
// embedding and Q-head tables receive row-sparse gradients, but the reference
// materialises them densely, so every row's moments decay and every row with
// non-zero m moves.  k_adam_rows reproduces that exactly without a dense
// gradient tensor: rows tagged with this step's epoch read their gradient
// from the (kept-zero) accumulation table and clear it; every other row takes
// g = 0.  28 B/param of HBM traffic (p, m, v read+write, tag / gradient rows
// only where touched).
#include "common.h"
#include <hip/hip_fp16.h>

static inline AdamArgs to_args(const float* a6) { return AdamArgs{a6[0], a6[1], a6[2], a6[3], a6[4], a6[5]}; }

__global__ void k_adam_dense(float* __restrict__ P, float* __restrict__ M, float* __restrict__ V,
                             float* __restrict__ G, int64_t n, AdamArgs a, int zero_grad) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float p = P[i], m = M[i], v = V[i];
    adam_elem(p, m, v, G[i], a);
    P[i] = p;
    M[i] = m;
    V[i] = v;
    if (zero_grad) G[i] = 0.f;
  }
}

extern "C" int rg_adam_dense(float* P, float* M, float* V, float* G, int64_t n, const float* adam6, int zero_grad,
                             hipStream_t stream) {
  if (n <= 0) return RG_ERR_ARG;
  int blocks = (int)((n + 255) / 256);
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL(k_adam_dense, dim3(blocks), dim3(256), 0, stream, P, M, V, G, n, to_args(adam6), zero_grad);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

// Row-sparse-gradient dense Adam.  cols % 4 == 0: one float4 per thread.
// The row of float4 i is i >> sh when cols / 4 is a power of two (sh >= 0),
// else i / (cols / 4); P / M / V stream through once per step (9 GB at C3),
// so they are loaded and stored non-temporally: 1.234 -> 1.138 ms for the
// 1M × 256 output layer (5.0 -> 5.4 TB/s, tools/adambench.py).
__global__ void k_adam_rows4(float* __restrict__ P, float* __restrict__ M, float* __restrict__ V,
                             float* __restrict__ G, const int32_t* __restrict__ tags, int32_t tag, int64_t rows,
                             int cols, int sh, AdamArgs a) {
  const int c4n = cols >> 2;
  const int64_t n4 = rows * c4n;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = sh >= 0 ? i >> sh : i / c4n;
    const bool hit = tags[row] == tag;
    f4 p = __builtin_nontemporal_load(reinterpret_cast<f4*>(P) + i);
    f4 m = __builtin_nontemporal_load(reinterpret_cast<f4*>(M) + i);
    f4 v = __builtin_nontemporal_load(reinterpret_cast<f4*>(V) + i);
    f4 g = {0.f, 0.f, 0.f, 0.f};
    if (hit) {
      g = reinterpret_cast<f4*>(G)[i];
      reinterpret_cast<f4*>(G)[i] = f4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float pq = p[q], mq = m[q], vq = v[q];
      adam_elem(pq, mq, vq, g[q], a);
      p[q] = pq;
      m[q] = mq;
      v[q] = vq;
    }
    __builtin_nontemporal_store(p, reinterpret_cast<f4*>(P) + i);
    __builtin_nontemporal_store(m, reinterpret_cast<f4*>(M) + i);
    __builtin_nontemporal_store(v, reinterpret_cast<f4*>(V) + i);
  }
}

typedef int32_t i4 __attribute__((ext_vector_type(4)));

// One-column tables (the heads' biases): four rows per thread, tags read
// as int4, so the sweep streams like the wide tables; rows past the last
// multiple of 4 go to k_adam_rows1.
__global__ void k_adam_bias4(float* __restrict__ P, float* __restrict__ M, float* __restrict__ V,
                             float* __restrict__ G, const int32_t* __restrict__ tags, int32_t tag, int64_t n4,
                             AdamArgs a) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    const i4 t = reinterpret_cast<const i4*>(tags)[i];
    f4 p = __builtin_nontemporal_load(reinterpret_cast<f4*>(P) + i);
    f4 m = __builtin_nontemporal_load(reinterpret_cast<f4*>(M) + i);
    f4 v = __builtin_nontemporal_load(reinterpret_cast<f4*>(V) + i);
    f4 g = {0.f, 0.f, 0.f, 0.f};
    if (t[0] == tag || t[1] == tag || t[2] == tag || t[3] == tag) {
      const f4 gr = reinterpret_cast<f4*>(G)[i];
      f4 gz = gr;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        g[q] = t[q] == tag ? gr[q] : 0.f;
        gz[q] = t[q] == tag ? 0.f : gr[q];
      }
      reinterpret_cast<f4*>(G)[i] = gz;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float pq = p[q], mq = m[q], vq = v[q];
      adam_elem(pq, mq, vq, g[q], a);
      p[q] = pq;
      m[q] = mq;
      v[q] = vq;
    }
    __builtin_nontemporal_store(p, reinterpret_cast<f4*>(P) + i);
    __builtin_nontemporal_store(m, reinterpret_cast<f4*>(M) + i);
    __builtin_nontemporal_store(v, reinterpret_cast<f4*>(V) + i);
  }
}

__global__ void k_adam_rows1(float* __restrict__ P, float* __restrict__ M, float* __restrict__ V,
                             float* __restrict__ G, const int32_t* __restrict__ tags, int32_t tag, int64_t rows,
                             int cols, AdamArgs a) {
  const int64_t n = rows * cols;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = cols == 1 ? i : i / cols;
    float g = 0.f;
    if (tags[row] == tag) {
      g = G[i];
      G[i] = 0.f;
    }
    float p = P[i], m = M[i], v = V[i];
    adam_elem(p, m, v, g, a);
    P[i] = p;
    M[i] = m;
    V[i] = v;
  }
}

extern "C" int rg_adam_rows(float* P, float* M, float* V, float* G, const int32_t* tags, int32_t tag, int64_t rows,
                            int cols, const float* adam6, hipStream_t stream) {
  if (rows <= 0 || cols <= 0) return RG_ERR_ARG;
  // the 16-B paths need 16-B aligned tables (torch allocations are; views at odd offsets take the scalar path)
  const bool a16 = ((reinterpret_cast<uintptr_t>(P) | reinterpret_cast<uintptr_t>(M) | reinterpret_cast<uintptr_t>(V) |
                     reinterpret_cast<uintptr_t>(G)) & 15) == 0;
  const bool wide = cols % 4 == 0 && a16;
  const int64_t n = wide ? rows * (cols / 4) : rows * cols;
  // about one float4 per thread up to 64M float4s (a 1M × 256 table): a 32768-block grid-stride
  // sweep ran 1.14 ms there, this one 1.07 ms (profiles/r06/adam_sweep_grid.txt)
  int blocks = (int)((n + 255) / 256);
  if (blocks > 262144) blocks = 262144;
  if (wide) {
    const int c4n = cols / 4;
    const int sh = (c4n & (c4n - 1)) == 0 ? __builtin_ctz((unsigned)c4n) : -1;
    hipLaunchKernelGGL(k_adam_rows4, dim3(blocks), dim3(256), 0, stream, P, M, V, G, tags, tag, rows, cols, sh,
                       to_args(adam6));
  }
  else if (cols == 1 && rows >= 4 && a16 && (reinterpret_cast<uintptr_t>(tags) & 15) == 0) {
    const int64_t n4 = rows / 4, r4 = n4 * 4;
    int b4 = (int)((n4 + 255) / 256);
    if (b4 > 32768) b4 = 32768;
    hipLaunchKernelGGL(k_adam_bias4, dim3(b4), dim3(256), 0, stream, P, M, V, G, tags, tag, n4, to_args(adam6));
    if (r4 < rows)
      hipLaunchKernelGGL(k_adam_rows1, dim3(1), dim3(256), 0, stream, P + r4, M + r4, V + r4, G + r4, tags + r4, tag,
                         rows - r4, 1, to_args(adam6));
  } else
    hipLaunchKernelGGL(k_adam_rows1, dim3(blocks), dim3(256), 0, stream, P, M, V, G, tags, tag, rows, cols,
                       to_args(adam6));
  RG_LAUNCH_CHECK();
  return RG_OK;
}

// Row-sparse dense Adam that also refreshes an fp16 copy of the table
// (config C5: the gather reads fp16 rows, Adam keeps fp32 master + moments).
__global__ void k_adam_rows4_h(float* __restrict__ P, float* __restrict__ M, float* __restrict__ V,
                               float* __restrict__ G, const int32_t* __restrict__ tags, int32_t tag, int64_t rows,
                               int cols, AdamArgs a, __half* __restrict__ P16) {
  const int c4n = cols >> 2;
  const int64_t n4 = rows * c4n;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = i / c4n;
    const bool hit = tags ? tags[row] == tag : true;
    f4 p = __builtin_nontemporal_load(reinterpret_cast<f4*>(P) + i);
    f4 m = __builtin_nontemporal_load(reinterpret_cast<f4*>(M) + i);
    f4 v = __builtin_nontemporal_load(reinterpret_cast<f4*>(V) + i);
    f4 g = {0.f, 0.f, 0.f, 0.f};
    if (hit) {
      g = reinterpret_cast<f4*>(G)[i];
      reinterpret_cast<f4*>(G)[i] = f4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float pq = p[q], mq = m[q], vq = v[q];
      adam_elem(pq, mq, vq, g[q], a);
      p[q] = pq;
      m[q] = mq;
      v[q] = vq;
    }
    __builtin_nontemporal_store(p, reinterpret_cast<f4*>(P) + i);
    __builtin_nontemporal_store(m, reinterpret_cast<f4*>(M) + i);
    __builtin_nontemporal_store(v, reinterpret_cast<f4*>(V) + i);
    const __half2 lo = __floats2half2_rn(p[0], p[1]), hi = __floats2half2_rn(p[2], p[3]);
    uint2 u;
    u.x = *reinterpret_cast<const uint32_t*>(&lo);
    u.y = *reinterpret_cast<const uint32_t*>(&hi);
    reinterpret_cast<uint2*>(P16)[i] = u;
  }
}

// tags == nullptr: every row takes its gradient (the dense all-reduced table
// of the multi-GPU trunk); the gradient table is cleared either way.
extern "C" int rg_adam_rows_h(float* P, float* M, float* V, float* G, const int32_t* tags, int32_t tag, int64_t rows,
                              int cols, const float* adam6, uint16_t* P16, hipStream_t stream) {
  if (rows <= 0 || cols <= 0 || cols % 4 || !P16) return RG_ERR_ARG;
  const int64_t n = rows * (cols / 4);
  int blocks = (int)((n + 255) / 256);
  if (blocks > 262144) blocks = 262144;   // (as rg_adam_rows)
  hipLaunchKernelGGL(k_adam_rows4_h, dim3(blocks), dim3(256), 0, stream, P, M, V, G, tags, tag, rows, cols,
                     to_args(adam6), reinterpret_cast<__half*>(P16));
  RG_LAUNCH_CHECK();
  return RG_OK;
}

// out = fp16(x), round to nearest even (initial copy / after load_state_dict)
// 8 values per thread-iteration (two 16-B loads, one 16-B store; the
// tables are E-wide rows, E % 8 == 0 — a scalar tail covers any n)
__global__ __launch_bounds__(256) void k_f32_to_f16(const float* __restrict__ x, int64_t n, __half* __restrict__ out) {
  const int64_t n8 = n / 8;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n8; i += stride) {
    const f4 a = reinterpret_cast<const f4*>(x)[2 * i], b = reinterpret_cast<const f4*>(x)[2 * i + 1];
    union {
      __half h[8];
      uint4 u;
    } o;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      o.h[k] = __float2half_rn(a[k]);
      o.h[4 + k] = __float2half_rn(b[k]);
    }
    reinterpret_cast<uint4*>(out)[i] = o.u;
  }
  for (int64_t i = 8 * n8 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += stride)
    out[i] = __float2half_rn(x[i]);
}

extern "C" int rg_f32_to_f16(const float* x, int64_t n, uint16_t* out, hipStream_t stream) {
  if (n <= 0) return RG_ERR_ARG;
  if ((reinterpret_cast<uintptr_t>(x) & 15) || (reinterpret_cast<uintptr_t>(out) & 15)) return RG_ERR_ARG;
  int blocks = (int)((n / 8 + 255) / 256);
  blocks = blocks < 1 ? 1 : (blocks > 8192 ? 8192 : blocks);
  hipLaunchKernelGGL(k_f32_to_f16, dim3(blocks), dim3(256), 0, stream, x, n, reinterpret_cast<__half*>(out));
  RG_LAUNCH_CHECK();
  return RG_OK;
}

// Fused slab reduction (split-K weight gradients) + Adam.  Workgroup = 32
// parameters × 8 slab groups: thread (q, c) sums slabs z ≡ q (mod 8) of
// parameter 32·bx + c in slab order (eight independent load chains per
// parameter instead of one serial chain over all slabs: the GRU's 49 k-
// parameter matrices with 128 token slabs went from ~50 µs to a few), then
// the eight partials are added in q order — a fixed order, so two runs are
// bitwise identical.  g_out: write the gradient instead of stepping.
__global__ __launch_bounds__(256) void k_adam_slabs(float* __restrict__ P, float* __restrict__ M,
                                                    float* __restrict__ V, const float* __restrict__ slabs,
                                                    int nslab, int64_t n, AdamArgs a, float* __restrict__ g_out) {
  rg_main_prio();
  __shared__ float part[8][33];
  const int c = threadIdx.x & 31, q = threadIdx.x >> 5;
  const int64_t i = (int64_t)blockIdx.x * 32 + c;
  float g = 0.f;
  if (i < n) {
    int z = q;
#pragma unroll 4
    for (; z < nslab; z += 8) g += slabs[(int64_t)z * n + i];
  }
  part[q][c] = g;
  __syncthreads();
  if (q != 0 || i >= n) return;
  g = part[0][c];
#pragma unroll
  for (int k = 1; k < 8; ++k) g += part[k][c];
  if (g_out) {
    g_out[i] = g;
    return;
  }
  float p = P[i], m = M[i], v = V[i];
  adam_elem(p, m, v, g, a);
  P[i] = p;
  M[i] = m;
  V[i] = v;
}

extern "C" int rg_adam_slabs(float* P, float* M, float* V, const float* slabs, int nslab, int64_t n,
                             const float* adam6, float* g_out, hipStream_t stream) {
  if (n <= 0 || nslab <= 0) return RG_ERR_ARG;
  AdamArgs a{};
  if (adam6) a = to_args(adam6);
  else if (!g_out) return RG_ERR_ARG;
  if (n > (int64_t)INT32_MAX * 32) return RG_ERR_ARG;
  hipLaunchKernelGGL(k_adam_slabs, dim3((unsigned)((n + 31) / 32)), dim3(256), 0, stream, P, M, V, slabs, nslab, n,
                     a, g_out);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

// ---- catch-up ("lazy") Adam with the dense semantics, bit for bit --------
// torch.optim.Adam moves EVERY row of a table every step (a row without a
// gradient sees g = 0: m ← m + w1·(0 − m), v ← β2·v, p moves by −lr·m̂/(√v̂ + ε)),
// and for a table read only a few rows at a time (the embedding; the sampled
// head's targets and negatives) the eager sweep is 24 B of HBM traffic per
// parameter and step for rows nobody reads.  Here a row's zero-gradient steps
// are replayed only when it is next read: last[r] = the table steps already
// applied to row r; hist row s − 1 = step s's scalars (written by step s's own
// rg_lazy_adam_rows).  A replayed step is adam_zero_step: adam_elem with g = 0
// in fewer operations but the same fp32 results (argued at adam_zero_step),
// so the table after any sequence of reads equals the eager one bitwise
// (tests/test_gpu_lazy_adam.py against k_adam_rows4's untagged rows).
struct LazyTab {
  float* P;
  float* M;
  float* V;
  float* G;        // adam: gradient rows (cleared after use)
  __half* P16;     // optional fp16 copy of P (config C5's gather table)
  float* Pb;       // optional 1-column companion (bias), same rows
  float* Mb;
  float* Vb;
  float* Gb;
  int cols;
};

// hist row s − 1 = step s's scalars, LAZY_HS floats: the six of AdamArgs, then
// RN(1 / bc2_sqrt) (written by the step's own kernel) and a pad to 32 bytes
constexpr int LAZY_HS = 8;
// One replayed step, g = 0: adam_elem(p, m, v, 0, a) bit for bit, in fewer
// operations (h0 = (w1, β2, c2, bc2_sqrt), h1 = (ε, neg_step, RN(1/bc2_sqrt), ·)):
//  * m: w1·(0 − m) + m — 0 − m and −m differ only at m = ±0, where the fma
//    gives +0 either way;
//  * v: β2·v + c2·0·0 = β2·v (v ≥ +0: + (+0) changes nothing);
//  * √v / bc2_sqrt by Markstein's correction with the step's exact reciprocal
//    r: q0 = x·r, q = fma(fma(−q0, d, x), r, q0) = RN(x / d) when r = RN(1/d)
//    and the residual does not underflow (x = √v ≥ 2^-75); checked against the
//    division for 1.5e9 quotients over the first 20000 steps' d at β2 ∈ {0.9 …
//    0.999} (tools/markstein_check.c; every mantissa at six exponents for
//    some d); x = ∞ keeps the division's ∞.
__device__ __forceinline__ void adam_zero_step(float& p, float& m, float& v, const f4 h0, const f4 h1) {
#pragma clang fp contract(off)
  m = __builtin_fmaf(h0.x, -m, m);
  v = v * h0.y;
  const float x = sqrtf(v);
  const float q0 = x * h1.z;
  const float q = __builtin_fmaf(__builtin_fmaf(-q0, h0.w, x), h1.z, q0);
  const float denom = (__builtin_isinf(x) ? x : q) + h1.x;
  p = p + h1.y * (m / denom);
}

// steps lo .. hi (inclusive) of one value (and, with BIAS, of the companion
// value); the step scalars by scalar loads from hist (wave-uniform addresses:
// every workgroup reads the same rows, L2 / scalar-cache hits — staging them
// in LDS measured slower, 2.40 vs 2.43 (256 steps) vs 2.45 ms (1024) per C3
// step at steady state, profiles/r07/ab_lazy_window_prefetch.txt)
template <bool BIAS>
__device__ __forceinline__ void lazy_replay(float& p0, float& m0, float& v0, float& p1, float& m1, float& v1,
                                            const float* __restrict__ h, int lo, int hi) {
#pragma unroll 2
  for (int s = lo; s <= hi; ++s) {
    const f4* r = reinterpret_cast<const f4*>(h + LAZY_HS * (int64_t)s);
    const f4 h0 = r[0], h1 = r[1];
    adam_zero_step(p0, m0, v0, h0, h1);
    if (BIAS) adam_zero_step(p1, m1, v1, h0, h1);
  }
}

// mode 0 (catch-up): rows with sel[r] == selv (sel NULL: every row) replay
// last[r] + 1 .. n; mode 1 (adam step n): rows with sel[r] == selv replay
// last[r] + 1 .. n − 1, then step n with their gradient (cleared); hist row n − 1 = a.
// Workgroup = 256 threads over 64 rows: the selected rows are processed
// 256 / CPR at a time, thread t on value t % CPR of row slot t / CPR (CPR =
// cols rounded up to a power of two, at least 64, so a row slot is whole waves
// and its step loop runs on scalar bounds), so every thread carries ONE
// value's chain of replayed steps and a row's values run in parallel; the
// thread of value 0 also carries the bias (a second, interleaved chain).  (The
// first form — one wave per row, each lane 4–5 values — ran the negatives' k ≈
// 400 step chains at 2 waves per SIMD and cost 1 ms per C3 step at steady
// state, profiles/r07/lazy_long_c3_v1.txt.)
template <int MODE, int CPR>
__global__ __launch_bounds__(256) void k_lazy_rows(LazyTab t, const int32_t* __restrict__ sel, int32_t selv,
                                                   int32_t* __restrict__ last, int64_t rows, int n,
                                                   float* __restrict__ hist, AdamArgs a) {
  if constexpr (MODE == 1) rg_main_prio();   // the step's own update (the replay-only mode stays at 0)
  static_assert(CPR >= 64 && CPR <= 256, "a row slot is whole waves");
  constexpr int RPP = 256 / CPR;   // rows per pass
  __shared__ int32_t rlist[64], rfirst[64];
  __shared__ int nsel;
  const int tid = threadIdx.x;
  const int nr = MODE == 1 ? n - 1 : n;   // newest replayed step
  if (MODE == 1 && blockIdx.x == 0 && tid == 0) {
    float* h = hist + LAZY_HS * (int64_t)(n - 1);
    h[0] = a.w1; h[1] = a.beta2; h[2] = a.c2; h[3] = a.bc2_sqrt; h[4] = a.eps; h[5] = a.neg_step;
    h[6] = 1.0f / a.bc2_sqrt;
    h[7] = 0.f;
  }
  const int64_t r0 = (int64_t)blockIdx.x * 64;
  if (tid < 64) {   // wave 0: this workgroup's selected rows, compacted in row order
    const int64_t rl = r0 + tid;
    const bool hit = rl < rows && (sel == nullptr || sel[rl] == selv);
    const int32_t lst = hit ? last[rl] : 0;
    const bool go = hit && (MODE == 1 || lst < n);
    const uint64_t mask = __ballot(go);
    if (go) {
      const int pos = __builtin_popcountll(mask & ((1ull << tid) - 1));
      rlist[pos] = tid;
      rfirst[pos] = lst + 1;
    }
    if (tid == 0) nsel = __builtin_popcountll(mask);
  }
  __syncthreads();
  const int ns = nsel;
  if (ns == 0) return;   // (uniform)
  const float* hg = hist - LAZY_HS;   // hg + LAZY_HS·s = step s's scalars (hist row s − 1)
  const int slot = tid / CPR, c = tid % CPR;
  for (int q0 = 0; q0 < ns; q0 += RPP) {
    const int q = q0 + slot;   // (wave-uniform)
    if (q >= ns) break;
    const int64_t r = r0 + rlist[q];
    const int s0 = __builtin_amdgcn_readfirstlane(rfirst[q]);
    const bool val = c < t.cols;
    const bool bia = t.Pb != nullptr && c == 0;
    const int64_t i = r * t.cols + (val ? c : 0);
    float p0 = val ? t.P[i] : 0.f, m0 = val ? t.M[i] : 0.f, v0 = val ? t.V[i] : 0.f;
    float p1 = bia ? t.Pb[r] : 0.f, m1 = bia ? t.Mb[r] : 0.f, v1 = bia ? t.Vb[r] : 0.f;
    float g0 = 0.f, g1 = 0.f;
    if (MODE == 1) {
      if (val) {
        g0 = t.G[i];
        t.G[i] = 0.f;
      }
      if (bia) {
        g1 = t.Gb[r];
        t.Gb[r] = 0.f;
      }
    }
    // steps s0 .. nr (idle lanes of a partial row run the chain on zeros: no branch per lane)
    if (__any(bia))   // (wave-uniform: only the wave holding a value-0 thread runs the bias chains)
      lazy_replay<true>(p0, m0, v0, p1, m1, v1, hg, s0, nr);
    else
      lazy_replay<false>(p0, m0, v0, p1, m1, v1, hg, s0, nr);
    if (MODE == 1) {
      adam_elem(p0, m0, v0, g0, a);
      adam_elem(p1, m1, v1, g1, a);
    }
    if (val) {
      t.P[i] = p0;
      t.M[i] = m0;
      t.V[i] = v0;
      if (t.P16) t.P16[i] = __float2half_rn(p0);
    }
    if (bia) {
      t.Pb[r] = p1;
      t.Mb[r] = m1;
      t.Vb[r] = v1;
    }
    if (c == 0) last[r] = n;
  }
}

static inline unsigned lazy_grid(int64_t rows) { return (unsigned)((rows + 63) / 64); }

// need[id] = stamp for the n ids (int64) in [0, rows) and, with S > 0, the S
// negatives of draw `counter` (draw_id over [0, rows), csrc/common.h)
__global__ void k_lazy_mark(const int64_t* __restrict__ ids, int64_t n, int64_t rows, uint64_t seed,
                            uint64_t counter, int S, int32_t* __restrict__ need, int32_t stamp) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const int64_t id = ids[i];
    if (id >= 0 && id < rows) need[id] = stamp;
  } else if (i < n + S) {
    need[draw_id(seed, counter, S, (int)(i - n), (uint64_t)rows)] = stamp;
  }
}

// need[id − lo] = stamp for the n int32 global ids in [lo, lo + rows) (the
// row-sharded table: the ids the other ranks requested from this shard)
__global__ void k_lazy_mark32(const int32_t* __restrict__ ids, int n, int64_t lo, int64_t rows,
                              int32_t* __restrict__ need, int32_t stamp) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t l = (int64_t)ids[i] - lo;
  if (l >= 0 && l < rows) need[l] = stamp;
}

static inline bool lazy_tab_ok(const LazyTab& t) {
  return t.P && t.M && t.V && t.cols > 0 && (!t.Pb || (t.Mb && t.Vb));
}


extern "C" int rg_lazy_mark_rows(const int64_t* ids, int64_t n, int64_t rows, uint64_t seed, uint64_t counter, int S,
                                 int32_t* need, int32_t stamp, hipStream_t stream) {
  if (n < 0 || S < 0 || rows <= 0 || !need || (n > 0 && !ids) || n + S == 0) return RG_ERR_ARG;
  hipLaunchKernelGGL(k_lazy_mark, dim3((unsigned)((n + S + 255) / 256)), dim3(256), 0, stream, ids, n, rows, seed,
                     counter, S, need, stamp);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_lazy_mark_rows32(const int32_t* ids, int n, int64_t lo, int64_t rows, int32_t* need, int32_t stamp,
                                   hipStream_t stream) {
  if (n < 0 || rows <= 0 || !need || (n > 0 && !ids)) return RG_ERR_ARG;
  if (n == 0) return RG_OK;
  hipLaunchKernelGGL(k_lazy_mark32, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, ids, n, lo, rows, need,
                     stamp);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_lazy_catch_up(float* P, float* M, float* V, int cols, uint16_t* P16, float* Pb, float* Mb, float* Vb,
                                int64_t rows, int32_t* last, const int32_t* need, int32_t stamp, int32_t n_steps,
                                float* hist, hipStream_t stream) {
  const LazyTab t{P, M, V, nullptr, reinterpret_cast<__half*>(P16), Pb, Mb, Vb, nullptr, cols};
  if (!lazy_tab_ok(t) || rows <= 0 || !last || n_steps < 0 || (n_steps > 0 && !hist)) return RG_ERR_ARG;
  if (n_steps == 0) return RG_OK;
#define LZ(CPR) hipLaunchKernelGGL((k_lazy_rows<0, CPR>), dim3(lazy_grid(rows)), dim3(256), 0, stream, t, need, stamp, \
                                 last, rows, n_steps, hist, AdamArgs{})
  if (cols <= 64) LZ(64);
  else if (cols <= 128) LZ(128);
  else if (cols <= 256) LZ(256);
  else return RG_ERR_SHAPE;
#undef LZ
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_lazy_adam_rows(float* P, float* M, float* V, float* G, int cols, uint16_t* P16, float* Pb, float* Mb,
                                 float* Vb, float* Gb, int64_t rows, int32_t* last, const int32_t* tags, int32_t tag,
                                 int32_t step, float* hist, const float* adam6, hipStream_t stream) {
  const LazyTab t{P, M, V, G, reinterpret_cast<__half*>(P16), Pb, Mb, Vb, Gb, cols};
  if (!lazy_tab_ok(t) || !G || (Pb && !Gb) || rows <= 0 || !last || !tags || step < 1 || !hist || !adam6)
    return RG_ERR_ARG;
#define LZ(CPR) hipLaunchKernelGGL((k_lazy_rows<1, CPR>), dim3(lazy_grid(rows)), dim3(256), 0, stream, t, tags, tag, last, \
                                 rows, step, hist, to_args(adam6))
  if (cols <= 64) LZ(64);
  else if (cols <= 128) LZ(128);
  else if (cols <= 256) LZ(256);
  else return RG_ERR_SHAPE;
#undef LZ
  RG_LAUNCH_CHECK();
  return RG_OK;
}
