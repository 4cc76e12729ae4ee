// Generic exact-f32 MFMA GEMM for the GRU's dense contractions:
//   input projection  Gi  = X · W_ihᵀ + b_ih      (T × 3H, K = E)
//   input gradient    dX  = dGi · W_ih             (T × E,  K = 3H)
//   weight gradients  dW  = dGᵀ · X / Hprev        (3H × E, K = T, split-K)
// C(m,n) = Σ_k A(m,k)·B(k,n) with A(m,k) = A[m*sam + k*sak], B(k,n) =
// B[k*sbk + n*sbn]; M and K may be read from device memory (T is only known
// on the device after packing).  64×64 block tile, BK = 16, four waves each
// owning one 32×32 v_mfma_f32_32x32x2_f32 accumulator.  Split-K writes one
// slab per grid.z; rg_reduce_slabs sums them in slab order (deterministic).
#include "common.h"

#define GB_M 64
#define GB_N 64
#define GB_K 16
#define GB_PAD 4

template <bool A_KCONTIG, bool B_NCONTIG>
__global__ __launch_bounds__(256) void k_gemm_f32(const float* __restrict__ A, int64_t sam, int64_t sak,
                                                  const float* __restrict__ Bm, int64_t sbk,
                                                  int64_t sbn, float* __restrict__ C, int64_t ldc,
                                                  int64_t slab, const float* __restrict__ bias, int M_,
                                                  const int32_t* __restrict__ Mptr, int N, int K_,
                                                  const int32_t* __restrict__ Kptr, int kchunk) {
  __shared__ float As[GB_K][GB_M + GB_PAD];
  __shared__ float Bs[GB_K][GB_N + GB_PAD];
  const int M = Mptr ? *Mptr : M_;
  const int K = Kptr ? *Kptr : K_;
  const int m0 = blockIdx.y * GB_M;
  const int n0 = blockIdx.x * GB_N;
  const int kbeg = blockIdx.z * kchunk;
  const int kend = min(K, kbeg + kchunk);
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = tid >> 6;
  const int wm = w >> 1, wn = w & 1;
  float* Cz = C + (int64_t)blockIdx.z * slab;
  if (m0 >= M) return;  // whole tile beyond the device-side row count
  f16v acc = {};
  for (int k0 = kbeg; k0 < kend; k0 += GB_K) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int e = tid + 256 * i;
      int kk, mm;
      if (A_KCONTIG) {
        kk = e & 15;
        mm = e >> 4;
      } else {
        mm = e & 63;
        kk = e >> 6;
      }
      int m = m0 + mm, k = k0 + kk;
      As[kk][mm] = (m < M && k < kend) ? A[(int64_t)m * sam + (int64_t)k * sak] : 0.0f;
      int nn;
      if (B_NCONTIG) {
        nn = e & 63;
        kk = e >> 6;
      } else {
        kk = e & 15;
        nn = e >> 4;
      }
      int n = n0 + nn;
      k = k0 + kk;
      Bs[kk][nn] = (n < N && k < kend) ? Bm[(int64_t)k * sbk + (int64_t)n * sbn] : 0.0f;
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < GB_K / 2; ++s) {
      float a = As[2 * s + (lane >> 5)][wm * 32 + (lane & 31)];
      float b = Bs[2 * s + (lane >> 5)][wn * 32 + (lane & 31)];
      acc = mfma32(a, b, acc);
    }
    __syncthreads();
  }
  const int col = n0 + wn * 32 + (lane & 31);
  if (col >= N) return;
  const float bv = bias ? bias[col] : 0.0f;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    int row = m0 + wm * 32 + acc32_row(r, lane >> 5);
    if (row < M) Cz[(int64_t)row * ldc + col] = acc[r] + bv;
  }
}

// Large-tile form for the trunk's token-major GEMMs (Gi = X·W_ihᵀ + b: A k-
// contiguous, B = W_ih with k contiguous per output column; dX = dGi·W_ih: B
// n-contiguous), no split-K, K % 32 == 0.  128 × 128 tile, BK = 32, double-
// buffered LDS filled by 16-B loads of whole 128-B row pieces (register
// prefetch of stage s+1 under stage s's MFMAs), two workgroups per CU; four
// waves each own a 64 × 64 block = 2 × 2 v_mfma_f32_32x32x2_f32 chains.  The
// k order inside a 4-deep quad is permuted (lane half h, MFMA j ↔ k = 2h + j)
// so one ds_read_b64 of a k-contiguous LDS row yields a lane's operands of
// both MFMAs of the quad.  Replaces the 64 × 64 / BK 16 / scalar-load tile at
// these shapes (C3: Gi 146 µs, dX 198 µs at T ≈ 85 k, 3H = 384, E = 128).
constexpr int GT_M = 128, GT_N = 128, GT_K = 32, GT_PA = GT_K + 4, GT_PB = GT_N + 4;

template <bool B_KCONTIG>
__global__ __launch_bounds__(256, 2) void k_gemm_nt(const float* __restrict__ A, int64_t lda,
                                                    const float* __restrict__ Bm, int64_t ldb,
                                                    float* __restrict__ C, int64_t ldc,
                                                    const float* __restrict__ bias, int M_,
                                                    const int32_t* __restrict__ Mptr, int N, int K) {
  constexpr int BSZ = B_KCONTIG ? GT_N * GT_PA : GT_K * GT_PB;
  __shared__ __attribute__((aligned(16))) float As[2][GT_M * GT_PA];
  __shared__ __attribute__((aligned(16))) float Bs[2][BSZ];
  const int M = Mptr ? *Mptr : M_;
  const int m0 = blockIdx.y * GT_M, n0 = blockIdx.x * GT_N;
  if (m0 >= M) return;  // whole tile beyond the device-side row count
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, l32 = lane & 31;
  const int wm = w >> 1, wn = w & 1;
  // this thread's four 16-B pieces of each stage (addresses clamped into the
  // matrices: rows past M / columns past N compute garbage that is never stored)
  const float* ap[4];
  const float* bp[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int e = tid + 256 * q;
    const int r = e >> 3, kq = e & 7;
    ap[q] = A + (int64_t)min(m0 + r, M - 1) * lda + 4 * kq;
    if (B_KCONTIG) bp[q] = Bm + (int64_t)min(n0 + r, N - 1) * ldb + 4 * kq;
    else bp[q] = Bm + (int64_t)(e >> 5) * ldb + min(n0 + 4 * (e & 31), N - 4);
  }
  f4 ra[4], rb[4];
  auto load = [&](int k0) __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      ra[q] = *reinterpret_cast<const f4*>(ap[q] + k0);
      rb[q] = *reinterpret_cast<const f4*>(bp[q] + (B_KCONTIG ? (int64_t)k0 : (int64_t)k0 * ldb));
    }
  };
  auto store = [&](int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int e = tid + 256 * q;
      *reinterpret_cast<f4*>(&As[buf][(e >> 3) * GT_PA + 4 * (e & 7)]) = ra[q];
      if (B_KCONTIG) *reinterpret_cast<f4*>(&Bs[buf][(e >> 3) * GT_PA + 4 * (e & 7)]) = rb[q];
      else *reinterpret_cast<f4*>(&Bs[buf][(e >> 5) * GT_PB + 4 * (e & 31)]) = rb[q];
    }
  };
  f16v acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i) acc[i][0] = acc[i][1] = f16v{};
  load(0);
  store(0);
  __syncthreads();
  int cur = 0;
  for (int k0 = 0; k0 < K; k0 += GT_K) {
    const bool more = k0 + GT_K < K;
    if (more) load(k0 + GT_K);
    const float* as = As[cur];
    const float* bs = Bs[cur];
#pragma unroll
    for (int kk = 0; kk < GT_K; kk += 4) {
      float2 a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        a[i] = *reinterpret_cast<const float2*>(&as[(wm * 64 + 32 * i + l32) * GT_PA + kk + 2 * h]);
        const int n = wn * 64 + 32 * i + l32;
        if (B_KCONTIG) {
          b[i] = *reinterpret_cast<const float2*>(&bs[n * GT_PA + kk + 2 * h]);
        } else {
          b[i].x = bs[(kk + 2 * h) * GT_PB + n];
          b[i].y = bs[(kk + 2 * h + 1) * GT_PB + n];
        }
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          acc[i][j] = mfma32(a[i].x, b[j].x, acc[i][j]);
          acc[i][j] = mfma32(a[i].y, b[j].y, acc[i][j]);
        }
    }
    if (more) store(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = n0 + wn * 64 + 32 * j + l32;
    if (col >= N) continue;
    const float bv = bias ? bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * 64 + 32 * i + acc32_row(r, h);
        if (row < M) C[(int64_t)row * ldc + col] = acc[i][j][r] + bv;
      }
  }
}

extern "C" int rg_gemm_f32(const float* A, int64_t sam, int64_t sak, const float* B, int64_t sbk,
                           int64_t sbn, float* C, int64_t ldc, const float* bias, int M, const int32_t* Mptr,
                           int N, int K, const int32_t* Kptr, int splits, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0 || splits <= 0) return RG_ERR_ARG;
  if (!(sak == 1 || sam == 1) || !(sbn == 1 || sbk == 1)) return RG_ERR_ARG;
  // large-tile path: A k-contiguous, no split-K, K % 32 == 0, N % 4 == 0 (≥ 4),
  // 16-B aligned rows (B either k- or n-contiguous)
  const bool b_kc = (sbk == 1), b_nc = (sbn == 1);
  if (splits == 1 && sak == 1 && K % GT_K == 0 && N % 4 == 0 && sam % 4 == 0 && ldc >= N &&
      ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(B)) & 15) == 0 &&
      ((b_kc && sbn % 4 == 0) || (b_nc && sbk % 4 == 0))) {
    dim3 gt((N + GT_N - 1) / GT_N, (M + GT_M - 1) / GT_M);
    if (b_kc)
      hipLaunchKernelGGL(k_gemm_nt<true>, gt, dim3(256), 0, stream, A, sam, B, sbn, C, ldc, bias, M, Mptr, N, K);
    else
      hipLaunchKernelGGL(k_gemm_nt<false>, gt, dim3(256), 0, stream, A, sam, B, sbk, C, ldc, bias, M, Mptr, N, K);
    RG_LAUNCH_CHECK();
    return RG_OK;
  }
  int kchunk = (K + splits - 1) / splits;
  kchunk = (kchunk + GB_K - 1) / GB_K * GB_K;
  int64_t slab = (int64_t)M * ldc;
  if (splits > 1 && bias) return RG_ERR_ARG;  // bias is added by the slab reduction
  dim3 grid((N + GB_N - 1) / GB_N, (M + GB_M - 1) / GB_M, splits);
  bool ak = (sak == 1), bn = (sbn == 1);
#define GL(AK, BN)                                                                                     \
  hipLaunchKernelGGL((k_gemm_f32<AK, BN>), grid, dim3(256), 0, stream, A, sam, sak, B, sbk, sbn, C, ldc, \
                     slab, bias, M, Mptr, N, K, Kptr, kchunk)
  if (ak && bn) GL(true, true);
  else if (ak && !bn) GL(true, false);
  else if (!ak && bn) GL(false, true);
  else GL(false, false);
#undef GL
  RG_LAUNCH_CHECK();
  return RG_OK;
}

// out[i] = Σ_z slabs[z*n + i] (+ bias[i % ncol]), z in order.
__global__ void k_reduce_slabs(const float* __restrict__ slabs, int nslab, int64_t n, float* __restrict__ out,
                               const float* __restrict__ bias, int ncol, int accumulate) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float s = 0.0f;
    for (int z = 0; z < nslab; ++z) s += slabs[(int64_t)z * n + i];
    if (bias) s += bias[i % ncol];
    out[i] = accumulate ? out[i] + s : s;
  }
}

extern "C" int rg_reduce_slabs(const float* slabs, int nslab, int64_t n, float* out, const float* bias, int ncol,
                               int accumulate, hipStream_t stream) {
  if (n <= 0 || nslab <= 0) return RG_ERR_ARG;
  int blocks = (int)((n + 255) / 256);
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(k_reduce_slabs, dim3(blocks), dim3(256), 0, stream, slabs, nslab, n, out, bias, ncol,
                     accumulate);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

// Column sums of a row-major (rows × ncol) matrix, split over rows into
// slabs: slabs[z*ncol + c] = Σ_{rows in split z} X[r*ncol + c].
__global__ void k_colsum(const float* __restrict__ X, int ncol, int rows_, const int32_t* __restrict__ rows_ptr,
                         int rchunk, float* __restrict__ slabs) {
  const int rows = rows_ptr ? *rows_ptr : rows_;
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= ncol) return;
  const int r0 = blockIdx.y * rchunk;
  const int r1 = min(rows, r0 + rchunk);
  float s = 0.0f;
  for (int r = r0; r < r1; ++r) s += X[(int64_t)r * ncol + c];
  slabs[(int64_t)blockIdx.y * ncol + c] = s;
}

extern "C" int rg_colsum(const float* X, int ncol, int rows, const int32_t* rows_ptr, int splits, float* slabs,
                         hipStream_t stream) {
  if (ncol <= 0 || splits <= 0 || rows <= 0) return RG_ERR_ARG;
  int rchunk = (rows + splits - 1) / splits;
  dim3 grid((ncol + 255) / 256, splits);
  hipLaunchKernelGGL(k_colsum, grid, dim3(256), 0, stream, X, ncol, rows, rows_ptr, rchunk, slabs);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

// ---------------------------------------------------------------------------
// Weight gradient of a dense layer over packed tokens, fused with the bias
// gradient:  dW[m][n] = Σ_t G[t][m]·X[t][n],  db[m] = Σ_t G[t][m]
// (nn.GRU backward: dW_ih = dGiᵀ·X, dW_hh = dGhᵀ·H_prev, b_ih/b_hh sums).
// G is (T × M) row-major, X is (T × N); T is read from the device.  One
// workgroup = a 128-row M tile × all N columns (N ≤ 128) over one token split;
// per 32-token step the G and X tiles go through LDS once and feed
// 16 k-steps × N/32 v_mfma_f32_32x32x2_f32 per wave; the bias column sums come
// from the same staged G values.  Slab z of dW / db holds split z.
template <int N>
__global__ __launch_bounds__(256) void k_wgrad(const float* __restrict__ G, int M, const float* __restrict__ X,
                                               const int32_t* __restrict__ Tptr, int tchunk,
                                               float* __restrict__ dw_slabs, float* __restrict__ db_slabs) {
  constexpr int NP = N < 32 ? 32 : N;
  constexpr int NCT = NP / 32;
  constexpr int TB = 32;
  constexpr int NX4 = TB * N / 4;
  constexpr int NXL = (NX4 + 255) / 256;
  __shared__ __attribute__((aligned(16))) float gs[2][TB][128 + 4];
  __shared__ __attribute__((aligned(16))) float xs[2][TB][NP + 4];
  __shared__ float csum[8][128];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, half = lane >> 5, l32 = lane & 31;
  const int T = *Tptr;
  // split the tokens actually present (T is only known on the device) evenly
  if (tchunk <= 0) tchunk = ((T + (int)gridDim.y - 1) / (int)gridDim.y + 31) / 32 * 32;
  const int m0 = blockIdx.x * 128;
  const int t0 = blockIdx.y * tchunk;
  const int t1 = min(T, t0 + tchunk);
  const int c4 = tid & 31;  // this thread's 4 G columns
  const int tr = tid >> 5;  // rows tr + 8i
  const int m = m0 + 4 * c4;
  const bool mv = m < M;
  const int mc = mv ? m : 0;
  f4 cs = {0.f, 0.f, 0.f, 0.f};
  f16v acc[NCT];
#pragma unroll
  for (int ct = 0; ct < NCT; ++ct) acc[ct] = f16v{};
  // register prefetch of one 32-token chunk; addresses clamped so every load
  // is issued unconditionally and stays in flight across the MFMA phase
  f4 gp[4], xp[NXL];
  float gk[4], xk[NXL];
  const int tlast = t1 > 0 ? t1 - 1 : 0;
  auto load = [&](int tb) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int t = tb + tr + 8 * i;
      gp[i] = *reinterpret_cast<const f4*>(G + (int64_t)(t < t1 ? t : tlast) * M + mc);
      gk[i] = (t < t1 && mv) ? 1.f : 0.f;
    }
#pragma unroll
    for (int i = 0; i < NXL; ++i) {
      const int e = tid + 256 * i;
      const int rr = (e < NX4 ? e : 0) / (N / 4), cc = (e < NX4 ? e : 0) % (N / 4);
      const int t = tb + rr;
      xp[i] = *reinterpret_cast<const f4*>(X + (int64_t)(t < t1 ? t : tlast) * N + 4 * cc);
      xk[i] = (e < NX4 && t < t1) ? 1.f : 0.f;
    }
  };
  auto commit = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const f4 v = gp[i] * gk[i];
      cs += v;
      *reinterpret_cast<f4*>(&gs[buf][tr + 8 * i][4 * c4]) = v;
    }
#pragma unroll
    for (int i = 0; i < NXL; ++i) {
      const int e = tid + 256 * i;
      if (e < NX4) {
        const int rr = e / (N / 4), cc = e % (N / 4);
        *reinterpret_cast<f4*>(&xs[buf][rr][4 * cc]) = xp[i] * xk[i];
      }
    }
  };
  int cur = 0;
  if (t0 < t1) {
    load(t0);
    commit(0);
  }
  __syncthreads();
  for (int tb = t0; tb < t1; tb += TB) {
    const bool more = tb + TB < t1;
    if (more) load(tb + TB);
#pragma unroll
    for (int s = 0; s < TB / 2; ++s) {
      const int t = half * (TB / 2) + s;
      const float a = gs[cur][t][32 * w + l32];
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) {
        const float b = (N >= 32 || l32 < N) ? xs[cur][t][ct * 32 + l32] : 0.f;
        acc[ct] = mfma32(a, b, acc[ct]);
      }
    }
    if (more) commit(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }
  float* dw = dw_slabs + (int64_t)blockIdx.y * M * N;
#pragma unroll
  for (int ct = 0; ct < NCT; ++ct) {
    const int n = ct * 32 + l32;
    if (n >= N) continue;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int mm = m0 + 32 * w + acc32_row(r, half);
      if (mm < M) dw[(int64_t)mm * N + n] = acc[ct][r];
    }
  }
  *reinterpret_cast<f4*>(&csum[tr][4 * c4]) = cs;
  __syncthreads();
  if (tid < 128) {
    float sm = 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q) sm += csum[q][tid];
    const int mm = m0 + tid;
    if (mm < M) db_slabs[(int64_t)blockIdx.y * M + mm] = sm;
  }
}

extern "C" int rg_wgrad(const float* G, int M, const float* X, int N, int T_max, const int32_t* Tptr, int splits,
                        float* dw_slabs, float* db_slabs, hipStream_t stream) {
  if (M <= 0 || M % 4 || T_max <= 0 || splits <= 0 || !Tptr) return RG_ERR_ARG;
  const int tchunk = 0;  // derived from the device-side token count
  dim3 grid((M + 127) / 128, splits);
#define WG(NV) hipLaunchKernelGGL(k_wgrad<NV>, grid, dim3(256), 0, stream, G, M, X, Tptr, tchunk, dw_slabs, db_slabs)
  switch (N) {
    case 16: WG(16); break;
    case 32: WG(32); break;
    case 64: WG(64); break;
    case 128: WG(128); break;
    case 256: WG(256); break;
    default: return RG_ERR_SHAPE;
  }
#undef WG
  RG_LAUNCH_CHECK();
  return RG_OK;
}

// ---------------------------------------------------------------------------
// Split-bf16 forms of the trunk's GEMMs (precision f32x6 / f32x6d3 / f32x9:
// the trainers' matmul_precision; "f32" keeps the fp32 MFMA kernels above).
// Every fp32 operand is split exactly into three bf16 planes while it is
// staged into LDS (common.h split3x8's RNE split), and each 16 × 16 output
// tile takes the plane products a_p·b_q with p + q <= 2 (NT = 6) or all nine
// (NT = 9) on v_mfma_f32_16x16x32_bf16 with fp32 accumulation — the fused
// head's arithmetic (the dropped products are below fp32's unit
// roundoff), at 1024 bf16 FLOP per SIMD-cycle instead of the fp32 MFMA's 64.
//
// LDS planes: [plane][row][32 k + 8 pad] bf16 (80-B rows: the sixteen rows
// one 16-lane group reads with ds_read_b128 fall on 16 distinct 4-bank groups).
constexpr int GX_T = 128, GX_K = 32, GX_RS = GX_K + 8;   // tile rows, k per stage, bf16 per LDS row

typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void split3x4(const f4& x, bf16x4& p0, bf16x4& p1, bf16x4& p2) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const __bf16 b0 = (__bf16)x[i];
    const float r1 = x[i] - (float)b0;
    const __bf16 b1 = (__bf16)r1;
    p0[i] = b0;
    p1[i] = b1;
    p2[i] = (__bf16)(r1 - (float)b1);
  }
}

// acc (16 × 16 tiles of a wave's 64 × 64 block) += A_tile · B_tileᵀ over one
// 32-deep stage: fragments straight from the LDS planes
template <int NT>
__device__ __forceinline__ void gx_stage_mfma(const __bf16* __restrict__ ap, const __bf16* __restrict__ bp, int wm,
                                              int wn, int lane, f4 (&acc)[4][4]) {
  constexpr int PL = GX_T * GX_RS;   // bf16 per plane
  const int r = lane & 15, kg = lane >> 4;
  bf16x8 b[4][3];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int p = 0; p < 3; ++p)
      b[j][p] = *reinterpret_cast<const bf16x8*>(bp + p * PL + (wn * 64 + 16 * j + r) * GX_RS + 8 * kg);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    bf16x8 a[3];
#pragma unroll
    for (int p = 0; p < 3; ++p)
      a[p] = *reinterpret_cast<const bf16x8*>(ap + p * PL + (wm * 64 + 16 * i + r) * GX_RS + 8 * kg);
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = mfma16_split<NT>(a[0], a[1], a[2], b[j][0], b[j][1], b[j][2], acc[i][j]);
  }
}

// C = A · Bᵀ (+ bias): A (M × K) k-contiguous (A_KCONTIG) or (K × M)
// m-contiguous, B (N × K) k-contiguous (B_KCONTIG) or (K × N) n-contiguous;
// K % 32 == 0; M may come from the device.  128 × 128 tile per 256-thread
// workgroup, two per CU (one 60 KB plane stage each; the next stage's fp32
// pieces are prefetched into registers under this stage's MFMAs).  Split-K:
// workgroup z takes k in [z·kchunk, (z+1)·kchunk) and writes slab z of C
// (C + z·slab; rg_reduce_slabs sums them in slab order).
template <int NT, bool A_KCONTIG, bool B_KCONTIG>
__global__ __launch_bounds__(256, 2) void k_gemm_x6(const float* __restrict__ A, int64_t lda,
                                                    const float* __restrict__ Bm, int64_t ldb,
                                                    float* __restrict__ C, int64_t ldc, const float* __restrict__ bias,
                                                    int M_, const int32_t* __restrict__ Mptr, int N, int K,
                                                    int kchunk, int64_t slab) {
  constexpr int PL = GX_T * GX_RS;
  __shared__ __attribute__((aligned(16))) __bf16 As[3 * PL];
  __shared__ __attribute__((aligned(16))) __bf16 Bs[3 * PL];
  // raised wave priority over the side streams' VALU work (the catch-up replay,
  // the head's pass 2): C2 +0.5 %, C3 +1.3 %, C4 −0.5 % (noise), same box,
  // profiles/r07/ab_x6_setprio.txt
  __builtin_amdgcn_s_setprio(2);
  const int M = Mptr ? *Mptr : M_;
  const int m0 = blockIdx.y * GX_T, n0 = blockIdx.x * GX_T;
  if (m0 >= M) return;
  const int kb = blockIdx.z * kchunk, ke = min(K, kb + kchunk);
  C += (int64_t)blockIdx.z * slab;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wm = w >> 1, wn = w & 1;
  // this thread's four 16-B pieces of each stage (rows clamped: rows past M /
  // columns past N compute values that are never stored)
  // (an m- / n-contiguous operand: thread = column c0 + (tid & 127), k =
  // 16·(tid >> 7) .. +15 of the stage, one coalesced 4-B load per k, written
  // as whole 16-B k-runs)
  const float* ap[4];
  const float* bq[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int e = tid + 256 * q;
    if (A_KCONTIG) ap[q] = A + (int64_t)min(m0 + (e >> 3), M - 1) * lda + 4 * (e & 7);
    if (B_KCONTIG) bq[q] = Bm + (int64_t)min(n0 + (e >> 3), N - 1) * ldb + 4 * (e & 7);
  }
  const float* acol = A + min(m0 + (tid & 127), M - 1) + (int64_t)(16 * (tid >> 7)) * lda;
  const float* bcol = Bm + min(n0 + (tid & 127), N - 1) + (int64_t)(16 * (tid >> 7)) * ldb;
  f4 ra[4], rb[4];
  auto load = [&](int k0) __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (A_KCONTIG) {
        ra[q] = *reinterpret_cast<const f4*>(ap[q] + k0);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) ra[q][i] = acol[(int64_t)(k0 + 4 * q + i) * lda];
      }
      if (B_KCONTIG) {
        rb[q] = *reinterpret_cast<const f4*>(bq[q] + k0);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) rb[q][i] = bcol[(int64_t)(k0 + 4 * q + i) * ldb];
      }
    }
  };
  auto store = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int e = tid + 256 * q;
      bf16x4 p0, p1, p2;
      split3x4(ra[q], p0, p1, p2);
      const int ko = (e >> 3) * GX_RS + 4 * (e & 7);
      const int co = (tid & 127) * GX_RS + 16 * (tid >> 7) + 4 * q;   // (this thread's k-run of column tid & 127)
      const int ao = A_KCONTIG ? ko : co;
      *reinterpret_cast<bf16x4*>(&As[ao]) = p0;
      *reinterpret_cast<bf16x4*>(&As[PL + ao]) = p1;
      *reinterpret_cast<bf16x4*>(&As[2 * PL + ao]) = p2;
      split3x4(rb[q], p0, p1, p2);
      const int bo = B_KCONTIG ? ko : co;
      *reinterpret_cast<bf16x4*>(&Bs[bo]) = p0;
      *reinterpret_cast<bf16x4*>(&Bs[PL + bo]) = p1;
      *reinterpret_cast<bf16x4*>(&Bs[2 * PL + bo]) = p2;
    }
  };
  f4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  if (kb < ke) load(kb);
  for (int k0 = kb; k0 < ke; k0 += GX_K) {
    store();
    __syncthreads();
    if (k0 + GX_K < ke) load(k0 + GX_K);
    gx_stage_mfma<NT>(As, Bs, wm, wn, lane, acc);
    __syncthreads();
  }
  const int r = lane & 15, kg = lane >> 4;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = n0 + wn * 64 + 16 * j + r;
    if (col >= N) continue;
    const float bv = bias ? bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int row = m0 + wm * 64 + 16 * i + 4 * kg + u;
        if (row < M) C[(int64_t)row * ldc + col] = acc[i][j][u] + bv;
      }
  }
}

static int gemm_x6_launch(const float* A, int64_t lda, int a_kcontig, const float* B, int64_t ldb, int b_kcontig,
                          float* C, int64_t ldc, int64_t slab, const float* bias, int M, const int32_t* Mptr, int N,
                          int K, int splits, int terms, hipStream_t stream) {
  // (16-B loads along k need k-contiguous rows at 4-float strides; the other layouts load 4 B per element)
  if (M <= 0 || N < 4 || K <= 0 || K % GX_K || N % 4 || (a_kcontig && lda % 4) || (b_kcontig && ldb % 4) ||
      ldc < N || splits < 1 || (terms != 6 && terms != 9))
    return RG_ERR_ARG;
  if (((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(B)) & 15) != 0) return RG_ERR_ARG;
  const int kchunk = (K / GX_K + splits - 1) / splits * GX_K;   // (a multiple of the 32-deep stage)
  const dim3 grid((N + GX_T - 1) / GX_T, (M + GX_T - 1) / GX_T, splits);
#define GX(NTV, AK, BK)                                                                                             \
  hipLaunchKernelGGL((k_gemm_x6<NTV, AK, BK>), grid, dim3(256), 0, stream, A, lda, B, ldb, C, ldc, bias, M, Mptr, N, \
                     K, kchunk, slab)
#define GXB(NTV, AK) \
  do {               \
    if (b_kcontig)   \
      GX(NTV, AK, true); \
    else             \
      GX(NTV, AK, false); \
  } while (0)
  if (terms == 6) {
    if (a_kcontig) GXB(6, true);
    else GXB(6, false);
  } else {
    if (a_kcontig) GXB(9, true);
    else GXB(9, false);
  }
#undef GXB
#undef GX
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_gemm_x6(const float* A, int64_t lda, const float* B, int64_t ldb, int b_kcontig, float* C,
                          int64_t ldc, const float* bias, int M, const int32_t* Mptr, int N, int K, int terms,
                          hipStream_t stream) {
  return gemm_x6_launch(A, lda, 1, B, ldb, b_kcontig, C, ldc, 0, bias, M, Mptr, N, K, 1, terms, stream);
}

extern "C" int rg_gemm_x6_sk(const float* A, int64_t lda, int a_kcontig, const float* B, int64_t ldb, int b_kcontig,
                             float* C, int64_t ldc, int64_t slab, int M, int N, int K, int splits, int terms,
                             hipStream_t stream) {
  if (splits > 1 && slab < (int64_t)M * ldc) return RG_ERR_ARG;
  return gemm_x6_launch(A, lda, a_kcontig, B, ldb, b_kcontig, C, ldc, slab, nullptr, M, nullptr, N, K, splits, terms,
                        stream);
}

// Split-bf16 weight gradient over packed tokens (rg_wgrad's contract):
// dW[m][n] = Σ_t G[t][m]·X[t][n] and db[m] = Σ_t G[t][m] into token-split
// slabs.  Workgroup = 128 m × 128 n (N = 256: two column tiles, grid.x) over
// one token split; k = tokens, 32 per stage: G's and X's fp32 rows are read
// coalesced and written transposed into the [m][t] / [n][t] planes.
template <int NT>
__global__ __launch_bounds__(256, 2) void k_wgrad_x6(const float* __restrict__ G, int M, const float* __restrict__ X,
                                                     int N, const int32_t* __restrict__ Tptr,
                                                     float* __restrict__ dw_slabs, float* __restrict__ db_slabs) {
  constexpr int PL = GX_T * GX_RS;
  __shared__ __attribute__((aligned(16))) __bf16 As[3 * PL];
  __shared__ __attribute__((aligned(16))) __bf16 Bs[3 * PL];
  __shared__ float csum[2][GX_T];
  __builtin_amdgcn_s_setprio(2);   // as in k_gemm_x6
  const int T = *Tptr;
  const int ntile_m = (M + GX_T - 1) / GX_T;
  const int mt = blockIdx.x % ntile_m, nt = blockIdx.x / ntile_m;
  const int m0 = mt * GX_T, n0 = nt * GX_T;
  const int tchunk = ((T + (int)gridDim.y - 1) / (int)gridDim.y + GX_K - 1) / GX_K * GX_K;
  const int t0 = blockIdx.y * tchunk, t1 = min(T, t0 + tchunk);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wm = w >> 1, wn = w & 1;
  // staging: thread = column c = tid & 127 of the G tile (m0 + c) and of the X
  // tile (n0 + c), tokens 16·(tid >> 7) .. +15 of the stage: one coalesced 4-B
  // load per token and operand, the 16 values written as whole 16-B runs of k
  const int c = tid & 127, tg = 16 * (tid >> 7);
  const float* gcol = G + min(m0 + c, M - 1);
  const float* xcol = X + min(n0 + c, N - 1);
  float cs = 0.f;
  f4 rg[4], rx[4];
  auto load = [&](int tb) __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int t = tb + tg + 4 * q + i;
        const bool ok = t < t1;
        const int64_t tc = ok ? t : t0;
        rg[q][i] = ok ? gcol[tc * M] : 0.f;
        rx[q][i] = ok ? xcol[tc * N] : 0.f;
      }
  };
  auto store = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      cs += (rg[q][0] + rg[q][1]) + (rg[q][2] + rg[q][3]);
      const int o = c * GX_RS + tg + 4 * q;
      bf16x4 p0, p1, p2;
      split3x4(rg[q], p0, p1, p2);
      *reinterpret_cast<bf16x4*>(&As[o]) = p0;
      *reinterpret_cast<bf16x4*>(&As[PL + o]) = p1;
      *reinterpret_cast<bf16x4*>(&As[2 * PL + o]) = p2;
      split3x4(rx[q], p0, p1, p2);
      *reinterpret_cast<bf16x4*>(&Bs[o]) = p0;
      *reinterpret_cast<bf16x4*>(&Bs[PL + o]) = p1;
      *reinterpret_cast<bf16x4*>(&Bs[2 * PL + o]) = p2;
    }
  };
  f4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  if (t0 < t1) load(t0);
  for (int tb = t0; tb < t1; tb += GX_K) {
    store();
    __syncthreads();
    if (tb + GX_K < t1) load(tb + GX_K);
    gx_stage_mfma<NT>(As, Bs, wm, wn, lane, acc);
    __syncthreads();
  }
  float* dw = dw_slabs + (int64_t)blockIdx.y * M * N;
  const int r = lane & 15, kg = lane >> 4;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = n0 + wn * 64 + 16 * j + r;
    if (n >= N) continue;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int m = m0 + wm * 64 + 16 * i + 4 * kg + u;
        if (m < M) dw[(int64_t)m * N + n] = acc[i][j][u];
      }
  }
  if (nt != 0) return;   // (one column tile writes the bias sums: column c's two token halves)
  csum[tid >> 7][c] = cs;
  __syncthreads();
  if (tid < GX_T && m0 + tid < M) db_slabs[(int64_t)blockIdx.y * M + m0 + tid] = csum[0][tid] + csum[1][tid];
}

extern "C" int rg_wgrad_x6(const float* G, int M, const float* X, int N, int T_max, const int32_t* Tptr, int splits,
                           float* dw_slabs, float* db_slabs, int terms, hipStream_t stream) {
  if (M <= 0 || M % 4 || N < 4 || N % 4 || T_max <= 0 || splits <= 0 || !Tptr || (terms != 6 && terms != 9))
    return RG_ERR_ARG;
  if (((reinterpret_cast<uintptr_t>(G) | reinterpret_cast<uintptr_t>(X)) & 15) != 0) return RG_ERR_ARG;
  const int ntm = (M + GX_T - 1) / GX_T, ntn = (N + GX_T - 1) / GX_T;
  const dim3 grid((unsigned)(ntm * ntn), (unsigned)splits);
  if (terms == 6)
    hipLaunchKernelGGL(k_wgrad_x6<6>, grid, dim3(256), 0, stream, G, M, X, N, Tptr, dw_slabs, db_slabs);
  else
    hipLaunchKernelGGL(k_wgrad_x6<9>, grid, dim3(256), 0, stream, G, M, X, N, Tptr, dw_slabs, db_slabs);
  RG_LAUNCH_CHECK();
  return RG_OK;
}
