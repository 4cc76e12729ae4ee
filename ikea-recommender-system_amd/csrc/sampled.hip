// Sampled-softmax output head (SURVEY §8 A7 "sampled/BPR ext.", config C3, and
// the north-star "embedding gather + sampled logits" step).
//
// Not in the reference (its loss is the full-softmax CrossEntropyLoss of
// GRU4Rec/model.py:121,146); the build defines it (parity pinned
// by the build's own CPU restatement, oracle/models.py:sampled_ce):
//   z_b,pos = h_b·W[a_b] + bias[a_b]
//   z_b,s   = h_b·W[neg_s] + bias[neg_s]            s < S, shared by the batch
//   loss    = mean_b [ logsumexp(z_b,pos, z_b,0..S-1) − z_b,pos ]
// Negatives are drawn uniformly on [0, A) with replacement; collisions with
// the target or with each other are kept and no logQ correction is applied
// (a uniform proposal shifts every logit by the same constant).
//
//  k_sample_uniform: counter-based draw (splitmix64 of seed/step/slot, then
//                    the high 64 bits of x·A) — reproducible bit-for-bit on
//                    the host without any RNG state.
//  k_sampled_fwd   : 128-negative × 128-row logit tile per workgroup.  The
//                    negatives' W rows are gathered straight from the table
//                    and staged with the h rows through LDS in 32-wide k
//                    chunks (double-buffered, register prefetch); four waves
//                    each own a 64×64 block = 2×2 v_mfma_f32_32x32x2_f32.
//                    Epilogue: + bias, Zᵀ[s][b] stores (consecutive b per
//                    half-wave) and per-(tile, row) online (max, Σexp)
//                    partials.  Row-tile 0 also writes the gathered W/bias
//                    rows (Wg, bg) that both backward GEMMs consume.
//  k_sampled_lse   : one wave per row: the positive logit as a wave-shuffle
//                    dot product, the tile partials merged by shuffles, lse,
//                    loss_b, and the positive's gradient rows.
//  k_sampled_dz    : dZᵀ = exp(Zᵀ − lse)·g in place, one workgroup per
//                    negative, with the bias gradient as its row sum.
#include "common.h"

#define SF_T 128
#define SF_KC 32
#define SF_LD (SF_KC + 4)

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ void k_sample_uniform(uint64_t seed, uint64_t counter, int S, uint64_t A, int32_t* __restrict__ out) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= S) return;
  const uint64_t x = mix64(seed + 0x9E3779B97F4A7C15ull * (counter * (uint64_t)S + (uint64_t)s + 1ull));
  out[s] = (int32_t)__umul64hi(x, A);
}

extern "C" int rg_sample_uniform(uint64_t seed, uint64_t counter, int S, int64_t A, int32_t* out,
                                 hipStream_t stream) {
  if (S <= 0 || A <= 0 || A > INT32_MAX) return RG_ERR_ARG;
  hipLaunchKernelGGL(k_sample_uniform, dim3((S + 255) / 256), dim3(256), 0, stream, seed, counter, S, (uint64_t)A,
                     out);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

__device__ __forceinline__ void lse_merge(float& m, float& s, float m2, float s2) {
  const float M = fmaxf(m, m2);
  if (M == -__builtin_inff()) return;  // both empty
  s = s * __expf(m - M) + s2 * __expf(m2 - M);
  m = M;
}

// ------------------------------------------------------------------ fwd ----
template <int HF>
__global__ __launch_bounds__(256) void k_sampled_fwd(const float* __restrict__ h, const float* __restrict__ W,
                                                     const float* __restrict__ bias,
                                                     const int32_t* __restrict__ neg, int B, int S,
                                                     float* __restrict__ ZT, int64_t ldz,
                                                     float* __restrict__ pmax, float* __restrict__ psum,
                                                     float* __restrict__ Wg, float* __restrict__ bg) {
  constexpr int NK = HF / SF_KC;
  __shared__ __attribute__((aligned(16))) float Ws[2][SF_T][SF_LD];
  __shared__ __attribute__((aligned(16))) float Hs[2][SF_T][SF_LD];
  __shared__ float sb[SF_T];
  __shared__ float rm[2][SF_T], rs[2][SF_T];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, half = lane >> 5, l32 = lane & 31;
  const int wm = w >> 1, wn = w & 1;
  const int s0 = blockIdx.x * SF_T, b0 = blockIdx.y * SF_T;
  const bool emit = Wg != nullptr && blockIdx.y == 0;
  // staging: this thread moves float4 column c4 of rows (tid >> 3) + 32 i
  const int c4 = tid & 7;
  const float* wrow[4];
  const float* hrow[4];
  float wk[4], hk[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = (tid >> 3) + 32 * i;
    const int s = s0 + r, b = b0 + r;
    const int id = s < S ? neg[s] : 0;
    wrow[i] = W + (int64_t)id * HF + 4 * c4;
    wk[i] = s < S ? 1.f : 0.f;
    hrow[i] = h + (int64_t)(b < B ? b : B - 1) * HF + 4 * c4;
    hk[i] = b < B ? 1.f : 0.f;
  }
  if (tid < SF_T) {
    const int s = s0 + tid;
    const float bv = s < S ? bias[neg[s]] : 0.f;
    sb[tid] = bv;
    if (emit && s < S) bg[s] = bv;
  }
  f4 pw[4], ph[4];
  auto load = [&](int k0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      pw[i] = *reinterpret_cast<const f4*>(wrow[i] + k0);
      ph[i] = *reinterpret_cast<const f4*>(hrow[i] + k0);
    }
  };
  auto commit = [&](int buf, int k0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = (tid >> 3) + 32 * i;
      const f4 x = pw[i] * wk[i];
      *reinterpret_cast<f4*>(&Ws[buf][r][4 * c4]) = x;
      *reinterpret_cast<f4*>(&Hs[buf][r][4 * c4]) = ph[i] * hk[i];
      if (emit && s0 + r < S) *reinterpret_cast<f4*>(Wg + (int64_t)(s0 + r) * HF + k0 + 4 * c4) = x;
    }
  };
  f16v acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f16v{};
  load(0);
  commit(0, 0);
  __syncthreads();
  int cur = 0;
#pragma unroll 1
  for (int kc = 0; kc < NK; ++kc) {
    const bool more = kc + 1 < NK;
    if (more) load((kc + 1) * SF_KC);
    const float* wa = &Ws[cur][64 * wm + l32][half * (SF_KC / 2)];
    const float* hb = &Hs[cur][64 * wn + l32][half * (SF_KC / 2)];
#pragma unroll
    for (int k = 0; k < SF_KC / 2; k += 4) {
      const f4 a0 = *reinterpret_cast<const f4*>(wa + k);
      const f4 a1 = *reinterpret_cast<const f4*>(wa + 32 * SF_LD + k);
      const f4 x0 = *reinterpret_cast<const f4*>(hb + k);
      const f4 x1 = *reinterpret_cast<const f4*>(hb + 32 * SF_LD + k);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        acc[0][0] = mfma32(a0[q], x0[q], acc[0][0]);
        acc[0][1] = mfma32(a0[q], x1[q], acc[0][1]);
        acc[1][0] = mfma32(a1[q], x0[q], acc[1][0]);
        acc[1][1] = mfma32(a1[q], x1[q], acc[1][1]);
      }
    }
    if (more) commit(cur ^ 1, (kc + 1) * SF_KC);
    __syncthreads();
    cur ^= 1;
  }
  // epilogue: bias, Zᵀ stores, online (max, Σexp) over this tile's negatives
#pragma unroll
  for (int nb = 0; nb < 2; ++nb) {
    const int bl = 64 * wn + 32 * nb + l32;
    const int b = b0 + bl;
    const bool bv = b < B;
    float m = -__builtin_inff(), sum = 0.f;
#pragma unroll
    for (int mb = 0; mb < 2; ++mb) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int sl = 64 * wm + 32 * mb + acc32_row(r, half);
        const float z = acc[mb][nb][r] + sb[sl];
        acc[mb][nb][r] = z;
        if (s0 + sl < S) {
          if (bv && ZT) ZT[(int64_t)(s0 + sl) * ldz + b] = z;
          m = fmaxf(m, z);
        }
      }
    }
    if (m != -__builtin_inff()) {
      const float m2 = m * 1.4426950408889634f;
#pragma unroll
      for (int mb = 0; mb < 2; ++mb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int sl = 64 * wm + 32 * mb + acc32_row(r, half);
          if (s0 + sl < S) sum += __builtin_amdgcn_exp2f(fmaf(acc[mb][nb][r], 1.4426950408889634f, -m2));
        }
    }
    lse_merge(m, sum, __shfl_xor(m, 32), __shfl_xor(sum, 32));
    if (half == 0) {
      rm[wm][bl] = m;
      rs[wm][bl] = sum;
    }
  }
  __syncthreads();
  if (tid < SF_T && b0 + tid < B) {
    float m = rm[0][tid], s = rs[0][tid];
    lse_merge(m, s, rm[1][tid], rs[1][tid]);
    const int64_t o = (int64_t)blockIdx.x * B + b0 + tid;
    pmax[o] = m;
    psum[o] = s;
  }
}

// ------------------------------------------------- split-bf16 forward ----
// Precision f32x9 / f32x6 (common.h): the same logits and (max, Σexp)
// partials as k_sampled_fwd (in 32-negative blocks), every fp32 product carried by bf16 MFMAs
// (v_mfma_f32_32x32x16_bf16, 16× the f32 MFMA rate).  Two launches:
//
//  k_sampled_prep: one thread per (row, 8-value k group) of the S negative
//    rows and of the B rows of h.  Negatives: optionally draws the id (the
//    k_sample_uniform stream), gathers the W row piece (coalesced: consecutive
//    threads read consecutive 32 B of a row) and writes Wg/bg (the logits
//    kernel and both backward GEMMs consume them); h rows: the three bf16
//    planes in MFMA fragment order, [32-row block][k slice][plane][lane] ×
//    16 B (whole 1 KB wave-instructions, nothing converted in the GEMM).
//  logits: rg_head_fwd_xp (csrc/head_split.hip) with the gathered negatives
//    as the item rows — each wave splits its 32 negatives' rows into VGPR
//    planes once and streams h's planes through an LDS ring, with Zᵀ stores
//    and the (max, Σexp) partials in the epilogue; the rows are split over
//    grid.y so S/(32·waves) negative groups still fill the chip.

// fragment-order plane buffer: entry (block, slice j, plane p, lane)
__device__ __forceinline__ int64_t plane_idx(int blk, int j, int p, int lane, int NS) {
  return (((int64_t)blk * NS + j) * 3 + p) * 64 + lane;
}

template <int HF>
__global__ __launch_bounds__(256) void k_sampled_prep(const float* __restrict__ h, const float* __restrict__ W,
                                                      const float* __restrict__ bias, int32_t* __restrict__ neg,
                                                      int draw, uint64_t seed, uint64_t counter, uint64_t A, int B,
                                                      int S, float* __restrict__ Wg, float* __restrict__ bg,
                                                      bf16x8* __restrict__ Wp, bf16x8* __restrict__ Hp) {
  constexpr int G = HF / 8;  // 8-value groups per row
  constexpr int NS = HF / 16;
  // thread order (32-row block, group g, row in block): a wave covers 32 rows
  // × 2 groups = one k slice, so each of its three plane stores is one
  // contiguous 1 KB fragment (S and B are multiples of 32)
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t blk = i / (32 * G);
  const int rem = (int)(i - blk * (32 * G));
  const int64_t nblk_neg = S / 32;
  if (blk >= nblk_neg + B / 32) return;
  const bool isneg = blk < nblk_neg;
  const int x = (int)((isneg ? blk : blk - nblk_neg) * 32) + (rem & 31), g = rem >> 5;
  const int j = g >> 1, hh = g & 1;
  const float* src;
  if (isneg) {
    int id;
    if (draw) {
      const uint64_t z = mix64(seed + 0x9E3779B97F4A7C15ull * (counter * (uint64_t)S + (uint64_t)x + 1ull));
      id = (int32_t)__umul64hi(z, A);
    } else {
      id = neg[x];
    }
    src = W + (int64_t)id * HF + 8 * g;
    if (g == 0) {
      if (draw) neg[x] = id;
      if (bg) bg[x] = bias[id];
    }
  } else {
    src = h + (int64_t)x * HF + 8 * g;
  }
  const f4 lo = *reinterpret_cast<const f4*>(src);
  const f4 hi = *reinterpret_cast<const f4*>(src + 4);
  if (isneg && Wg) {
    float* dst = Wg + (int64_t)x * HF + 8 * g;
    *reinterpret_cast<f4*>(dst) = lo;
    *reinterpret_cast<f4*>(dst + 4) = hi;
  }
  if (isneg && Wp == nullptr) return;  // only h's planes are needed
  bf16x8 p0, p1, p2;
  split3x8(lo, hi, p0, p1, p2);
  bf16x8* dst = isneg ? Wp : Hp;
  const int lane = hh * 32 + (x & 31);
  dst[plane_idx(x >> 5, j, 0, lane, NS)] = p0;
  dst[plane_idx(x >> 5, j, 1, lane, NS)] = p1;
  dst[plane_idx(x >> 5, j, 2, lane, NS)] = p2;
}

// split-bf16 logits kernel shared with the full-softmax head (csrc/head_split.hip)
extern "C" int rg_head_fwd_xp(const void* hplanes, const float* W, const float* bias, int B, int A, int HF,
                              int terms, int rpb, float* ZT, int64_t ldz, float* pmax, float* psum, int32_t* parg,
                              int want_sum, hipStream_t stream);

// --------------------------------------------- split-bf16 logits GEMM ----
// Zᵀ = Wneg·hᵀ + b from operand planes already in MFMA fragment order
// ([32-row block][16-deep slice j][plane p][lane] × 16 B, lane (hh, n) holding
// row n, k = 16j + 8hh .. +8): the negatives' planes Wk (k_sampled_prep, or
// the trunk gather's fused negative prep rg_gather_neg) and h's planes Hk
// (k_sampled_prep, or the GRU forward's epilogue).  No VALU besides the
// epilogue.
//
// Workgroup = 512 threads = 8 waves over 256 negatives × 128 rows; grid.x =
// negative tiles, so the dispatch's XCD round-robin keeps a tile's 32 row
// tiles on one XCD (its A planes are fetched into one L2).  Wave w holds the
// planes of negatives 256·bx + 32w in VGPRs (3·HF/16 coalesced 1 KB loads);
// the four 32-row chunks of h's planes go global → LDS by DMA into four
// separate arrays (the compiler then orders each chunk's reads after that
// chunk's DMA only).  Issue order: chunk 0's DMA, the A loads, chunks 1-3's
// DMA; chunk c is waited for with vmcnt(#younger DMA) + s_barrier, and slice
// j's MFMAs wait only for slice j's A loads, so the MFMAs start before the A
// planes have all landed.  Accumulators alternate: chunk c's epilogue (+
// bias, Zᵀ buffer stores with scalar offsets, max / Σexp per (32-negative
// block, row)) issues under chunk c+1's MFMAs.
constexpr int SG_NEG = 256;   // negatives per workgroup (8 waves × 32)
constexpr int SG_ROWS = 128;  // rows per workgroup (4 chunks of 32)

__device__ __forceinline__ void sg_lds_dma(const void* src, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)const_cast<void*>(src),
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

// s_waitcnt vmcnt(N) with lgkmcnt / expcnt left free (gfx9 encoding)
#define SG_VMCNT(N) __builtin_amdgcn_s_waitcnt(((N) & 0xF) | (((N) >> 4) << 14) | (0x7 << 4) | (0xF << 8))

template <int HF, int NT>
__global__ __launch_bounds__(512) void k_sampled_gemm(const bf16x8* __restrict__ Wk, const float* __restrict__ bg,
                                                      const bf16x8* __restrict__ Hk, int B, int S,
                                                      float* __restrict__ ZT, int64_t ldz,
                                                      float* __restrict__ pmax, float* __restrict__ psum) {
  constexpr int NS = HF / 16;
  constexpr int CH = NS * 192;              // 16-B fragments of one 32-row chunk's planes
  constexpr int NPC = CH / 64;              // 1 KB DMA pieces per chunk
  constexpr int PPW = (NPC + 7) / 8;        // pieces per wave per chunk (duplicates pad the last round)
  constexpr float L2E = 1.4426950408889634f;
  __shared__ bf16x8 hc0[CH], hc1[CH], hc2[CH], hc3[CH];
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, hh = lane >> 5, l32 = lane & 31;
  const int s0 = blockIdx.x * SG_NEG + 32 * w;
  const bool nact = s0 < S;                 // S % 32 == 0
  const int rbase = blockIdx.y * SG_ROWS;
  const int nch = min(SG_ROWS, B - rbase) / 32;   // B % 32 == 0
#ifdef SG_STAMP
  const uint64_t t_start = __builtin_amdgcn_s_memtime();
#endif
  const bf16x8* __restrict__ hsrc = Hk + (int64_t)(rbase / 32) * CH;
  // chunks past nch re-fetch chunk 0 (keeps the per-wave DMA count uniform;
  // never read).  A macro: the DMA's LDS operand must name its array.
#define SG_DMA(C, DST)                                                                                     \
  do {                                                                                                      \
    const int cs_ = (C) < nch ? (C) : 0;                                                                    \
    _Pragma("unroll") for (int i = 0; i < PPW; ++i) {                                                       \
      const int q = (w + 8 * i) % NPC;                                                                      \
      sg_lds_dma(hsrc + (int64_t)cs_ * CH + 64 * q + lane, &DST[64 * q]);                                   \
    }                                                                                                       \
  } while (0)
  // bias of accumulator row acc32_row(r, hh): four runs of 4 negatives (no
  // lane shuffles here: an LDS-class instruction would make the compiler wait
  // for every outstanding DMA)
  f4 bq[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) bq[q] = *reinterpret_cast<const f4*>(bg + (nact ? s0 : 0) + 8 * q + 4 * hh);
  // the scheduling barriers pin the vector-memory issue order the vmcnt
  // waits below count on: bias, chunk 0's DMA, A planes, chunks 1-3's DMA
  __builtin_amdgcn_sched_barrier(0);
  SG_DMA(0, hc0);
  __builtin_amdgcn_sched_barrier(0);
  bf16x8 a[NS][3];
  const bf16x8* __restrict__ asrc = Wk + (int64_t)(nact ? s0 / 32 : 0) * CH + lane;
#pragma unroll
  for (int j = 0; j < NS; ++j)
#pragma unroll
    for (int p = 0; p < 3; ++p) a[j][p] = asrc[j * 192 + p * 64];
  __builtin_amdgcn_sched_barrier(0);
  SG_DMA(1, hc1);
  SG_DMA(2, hc2);
  SG_DMA(3, hc3);
  __builtin_amdgcn_sched_barrier(0);
  float bj[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) bj[r] = bq[r >> 2][r & 3];
  // Zᵀ stores through a buffer descriptor over this wave's 32 negative rows
  const uint64_t zb = (uint64_t)(ZT + (int64_t)(nact ? s0 : 0) * ldz);
  const uint32_t zlo = __builtin_amdgcn_readfirstlane((uint32_t)zb);
  const uint32_t zhi = __builtin_amdgcn_readfirstlane((uint32_t)(zb >> 32));
  const uint32_t znb = __builtin_amdgcn_readfirstlane(nact ? (uint32_t)(32 * ldz * 4) : 0u);
  const __amdgpu_buffer_rsrc_t zrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)zhi << 32) | zlo), 0, znb, 0x00020000);
  const int zlane = (4 * hh * (int)ldz + l32) * 4;
  const int zrow4 = __builtin_amdgcn_readfirstlane((int)ldz * 4);
  float* __restrict__ pm = pmax + (int64_t)(s0 / 32) * B + rbase + l32;
  float* __restrict__ ps = psum + (int64_t)(s0 / 32) * B + rbase + l32;
  // (a macro, not a pointer-taking helper: indexing each chunk's own LDS array
  // keeps the compiler's per-array DMA ordering)
#define SG_MMA(HC, ACC)                                                                                  \
  do {                                                                                                    \
    ACC = f16v{};                                                                                         \
    _Pragma("unroll") for (int j = 0; j < NS; ++j) ACC =                                                  \
        mfma_split<NT>(a[j][0], a[j][1], a[j][2], HC[j * 192 + lane], HC[j * 192 + 64 + lane],            \
                       HC[j * 192 + 128 + lane], ACC);                                                    \
  } while (0)
  auto epi = [&](f16v& acc, int c) __attribute__((always_inline)) {
    float m = -__builtin_inff();
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float z = acc[r] + bj[r];
      acc[r] = z;
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(z), zrs, zlane,
                                            ((r & 3) + 8 * (r >> 2)) * zrow4 + (rbase + 32 * c) * 4, 0);
      m = fmaxf(m, z);
    }
    m = fmaxf(m, __shfl_xor(m, 32));
    const float m2 = m * L2E;
    float sum = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) sum += __builtin_amdgcn_exp2f(fmaf(acc[r], L2E, -m2));
    sum += __shfl_xor(sum, 32);
    if (nact && hh == 0) {
      pm[32 * c] = m;
      ps[32 * c] = sum;
    }
  };
  auto sync = [&]() __attribute__((always_inline)) {
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  // chunk 0: wait for its DMA only (the A loads and chunks 1-3 may still fly)
  SG_VMCNT(3 * NS + 3 * PPW);
  sync();
  // Waves without negatives (s0 >= S) run the MFMAs on zero planes and write
  // nothing (their Zᵀ descriptor has no records, their partials are skipped):
  // no branch around the MFMA chains, whose operand waits stay per-slice.
  f16v accA, accB;
  SG_MMA(hc0, accA);
#ifdef SG_STAMP
  const uint64_t t_c0 = __builtin_amdgcn_s_memtime();
#endif
  if (nch > 1) {
    SG_VMCNT(2 * PPW);
    sync();
    SG_MMA(hc1, accB);
    epi(accA, 0);
  }
  if (nch > 2) {
    SG_VMCNT(PPW);
    sync();
    SG_MMA(hc2, accA);
    epi(accB, 1);
  }
  if (nch > 3) {
    SG_VMCNT(0);
    sync();
    SG_MMA(hc3, accB);
    epi(accA, 2);
    epi(accB, 3);
  } else {
    if (nch == 1) epi(accA, 0);
    if (nch == 2) epi(accB, 1);
    if (nch == 3) epi(accA, 2);
  }
  SG_VMCNT(0);  // no DMA may still target this workgroup's LDS when it retires
#ifdef SG_STAMP
  const uint64_t t_end = __builtin_amdgcn_s_memtime();
  if (lane == 0) {  // diagnostic build only: stamps overwrite pmax (the microbench reads them back)
    int64_t* out = reinterpret_cast<int64_t*>(pmax) + ((int64_t)(blockIdx.y * gridDim.x + blockIdx.x) * 8 + w) * 4;
    out[0] = (int64_t)t_start;
    out[1] = (int64_t)t_c0;
    out[2] = (int64_t)t_end;
    out[3] = 0;
  }
#endif
#undef SG_MMA
#undef SG_DMA
}

// bytes of scratch rg_sampled_fwd_x needs (the negatives' and h's operand planes)
extern "C" int64_t rg_sampled_work_bytes(int B, int S, int HF) {
  if (B <= 0 || S <= 0 || HF <= 0) return RG_ERR_ARG;
  return ((int64_t)S + B) * HF * 6;
}

// The logits GEMM alone, from operand planes (k_sampled_gemm above).
extern "C" int rg_sampled_gemm(const void* Wk, const float* bg, const void* Hk, int B, int S, int HF, int terms,
                               float* ZT, int64_t ldz, float* pmax, float* psum, hipStream_t stream) {
  if (B <= 0 || S <= 0 || (B % 32) || (S % 32) || !Wk || !bg || !Hk || !ZT || !pmax || !psum) return RG_ERR_ARG;
  if (ldz < B) return RG_ERR_ARG;
  if (terms != 6 && terms != 9) return RG_ERR_ARG;
  const dim3 grid((unsigned)((S + SG_NEG - 1) / SG_NEG), (unsigned)((B + SG_ROWS - 1) / SG_ROWS));
#define SGG(HFV, NTV)                                                                                          \
  hipLaunchKernelGGL((k_sampled_gemm<HFV, NTV>), grid, dim3(512), 0, stream, (const bf16x8*)Wk, bg,          \
                     (const bf16x8*)Hk, B, S, ZT, ldz, pmax, psum)
#define SGT(HFV)  \
  if (terms == 9) \
    SGG(HFV, 9);  \
  else            \
    SGG(HFV, 6);
  switch (HF) {
    case 32: SGT(32); break;
    case 64: SGT(64); break;
    case 128: SGT(128); break;
    default: return RG_ERR_SHAPE;
  }
#undef SGT
#undef SGG
  RG_LAUNCH_CHECK();
  return RG_OK;
}

// Split-bf16 forward (terms = 9: exact products, fp32 accumulation; 6: the
// three sub-ulp terms dropped).  Same outputs and partial blocking as the fast
// path of rg_sampled_fwd; needs S % 32 == 0 and B % 32 == 0.  draw = 1: neg
// is an output, filled with the rg_sample_uniform(seed, counter) draw.
// Operand prep (draw, negatives' row gather → Wg/bg and planes, h's planes;
// one launch), then the logits: HF <= 128 on rg_sampled_gemm, HF = 256 on
// rg_head_fwd_xp (a 32-negative HF-256 plane set, 192 VGPRs, does not fit
// beside the accumulators at two waves per SIMD).
extern "C" int rg_sampled_fwd_x(const float* h, const float* W, const float* bias, int32_t* neg, int draw,
                                uint64_t seed, uint64_t counter, int64_t A, int B, int S, int HF, int terms,
                                float* ZT, int64_t ldz, float* pmax, float* psum, float* Wg, float* bg, void* work,
                                hipStream_t stream) {
  if (B <= 0 || S <= 0 || (B % 32) || (S % 32) || work == nullptr || bg == nullptr || Wg == nullptr ||
      ZT == nullptr)
    return RG_ERR_ARG;
  if (ldz < B) return RG_ERR_ARG;
  if (draw && (A <= 0 || A > INT32_MAX)) return RG_ERR_ARG;
  if (terms != 6 && terms != 9) return RG_ERR_ARG;
  const bool gemm = HF <= 128;
  bf16x8* Wp = reinterpret_cast<bf16x8*>(work);
  bf16x8* Hp = Wp + (int64_t)S * HF / 8 * 3;
  const int64_t items = ((int64_t)S + B) * (HF / 8);
  const dim3 gp((unsigned)((items + 255) / 256));
#define SXP(HFV)                                                                                            \
  hipLaunchKernelGGL(k_sampled_prep<HFV>, gp, dim3(256), 0, stream, h, W, bias, neg, draw, seed, counter, \
                     (uint64_t)A, B, S, Wg, bg, gemm ? Wp : (bf16x8*)nullptr, Hp)
  switch (HF) {
    case 32: SXP(32); break;
    case 64: SXP(64); break;
    case 128: SXP(128); break;
    case 256: SXP(256); break;
    default: return RG_ERR_SHAPE;
  }
#undef SXP
  RG_LAUNCH_CHECK();
  if (gemm) return rg_sampled_gemm(Wp, bg, Hp, B, S, HF, terms, ZT, ldz, pmax, psum, stream);
  // negatives × rows on k_head_fwd_x (csrc/head_split.hip): each wave holds
  // 32 gathered negatives' planes in VGPRs, h's planes stream through LDS; the
  // rows are split over grid.y so the S/(32·waves) negative groups fill the chip
  const int nw = 4;
  const int ngx = (S + 32 * nw - 1) / (32 * nw);
  const int ny = max(1, 256 / ngx);
  // rows per workgroup (rows·negatives workgroups ≈ one per CU; the best of
  // 32..512 swept at B 4096, S 2048: 256 at HF 256)
  const int rpb = ((B + ny - 1) / ny + 31) / 32 * 32;
  return rg_head_fwd_xp(Hp, Wg, bg, B, S, HF, terms, rpb, ZT, ldz, pmax, psum, nullptr, 1, stream);
}

// Number of (max, Σexp) partials per row the forward writes: 128-negative
// tiles for rg_sampled_fwd (terms = 0), 32-negative blocks for
// rg_sampled_fwd_x (terms = 6 / 9, S and B multiples of 32).
extern "C" int rg_sampled_nparts(int B, int S, int terms) {
  if (B <= 0 || S <= 0) return RG_ERR_ARG;
  if (terms == 0) return (S + SF_T - 1) / SF_T;
  if ((terms != 6 && terms != 9) || S % 32 || B % 32) return RG_ERR_ARG;
  return S / 32;
}

extern "C" int rg_sampled_fwd(const float* h, const float* W, const float* bias, const int32_t* neg, int B, int S,
                              int HF, float* ZT, int64_t ldz, float* pmax, float* psum, float* Wg, float* bg,
                              hipStream_t stream) {
  if (B <= 0 || S <= 0) return RG_ERR_ARG;
  if (ZT && ldz < B) return RG_ERR_ARG;
  if ((Wg == nullptr) != (bg == nullptr)) return RG_ERR_ARG;
  dim3 grid((S + SF_T - 1) / SF_T, (B + SF_T - 1) / SF_T);
#define SFL(HFV)                                                                                            \
  hipLaunchKernelGGL(k_sampled_fwd<HFV>, grid, dim3(256), 0, stream, h, W, bias, neg, B, S, ZT, ldz, pmax, \
                     psum, Wg, bg)
  switch (HF) {
    case 32: SFL(32); break;
    case 64: SFL(64); break;
    case 128: SFL(128); break;
    case 256: SFL(256); break;
    default: return RG_ERR_SHAPE;
  }
#undef SFL
  RG_LAUNCH_CHECK();
  return RG_OK;
}

// ------------------------------------------------------------------ lse ----
// One wave per row b.  Outputs: lse[b]; loss_row[b] = lse − z_pos (NaN for an
// out-of-range target, as CrossEntropyLoss raises); ids[b] = a_b (int32, −1
// if invalid) for the gradient scatter; dzpos[b] = (p_pos − 1)·g; gpos[b] =
// dzpos·h_b (∂/∂W[a_b]); dhpos[b] = dzpos·W[a_b] (∂/∂h_b, positive part).
template <int HF>
__global__ __launch_bounds__(256) void k_sampled_lse(const float* __restrict__ h, const float* __restrict__ W,
                                                     const float* __restrict__ bias,
                                                     const int64_t* __restrict__ tgt, int B, int64_t A,
                                                     const float* __restrict__ pmax,
                                                     const float* __restrict__ psum, int nT, float gscale,
                                                     float* __restrict__ lse, float* __restrict__ loss_row,
                                                     int32_t* __restrict__ ids, float* __restrict__ dzpos,
                                                     float* __restrict__ gpos, float* __restrict__ dhpos) {
  constexpr int PER = HF >= 64 ? HF / 64 : 1;
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;  // whole wave
  const int64_t t = tgt[b];
  const bool ok = t >= 0 && t < A;
  const int64_t tt = ok ? t : 0;
  float hv[PER], wv[PER];
  float dot = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = lane + 64 * i;
    const bool cv = c < HF;
    hv[i] = cv ? h[(int64_t)b * HF + c] : 0.f;
    wv[i] = cv ? W[tt * HF + c] : 0.f;
    dot = fmaf(hv[i], wv[i], dot);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) dot += __shfl_xor(dot, o);
  const float zp = dot + bias[tt];
  float m = -__builtin_inff(), s = 0.f;
  for (int j = lane; j < nT; j += 64) lse_merge(m, s, pmax[(int64_t)j * B + b], psum[(int64_t)j * B + b]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) lse_merge(m, s, __shfl_xor(m, o), __shfl_xor(s, o));
  lse_merge(m, s, zp, 1.f);
  const float l = m + logf(s);
  const float dp = (expf(zp - l) - 1.f) * gscale;
  if (lane == 0) {
    lse[b] = l;
    loss_row[b] = ok ? l - zp : __builtin_nanf("");
    ids[b] = ok ? (int32_t)t : -1;
    dzpos[b] = ok ? dp : 0.f;
  }
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = lane + 64 * i;
    if (c < HF) {
      gpos[(int64_t)b * HF + c] = ok ? dp * hv[i] : 0.f;
      dhpos[(int64_t)b * HF + c] = ok ? dp * wv[i] : 0.f;
    }
  }
}

extern "C" int rg_sampled_lse(const float* h, const float* W, const float* bias, const int64_t* tgt, int B,
                              int64_t A, int HF, const float* pmax, const float* psum, int nT, float gscale,
                              float* lse, float* loss_row, int32_t* ids, float* dzpos, float* gpos, float* dhpos,
                              hipStream_t stream) {
  if (B <= 0 || A <= 0 || nT <= 0) return RG_ERR_ARG;
  dim3 grid((B + 3) / 4);
#define SLL(HFV)                                                                                              \
  hipLaunchKernelGGL(k_sampled_lse<HFV>, grid, dim3(256), 0, stream, h, W, bias, tgt, B, A, pmax, psum, nT, \
                     gscale, lse, loss_row, ids, dzpos, gpos, dhpos)
  switch (HF) {
    case 32: SLL(32); break;
    case 64: SLL(64); break;
    case 128: SLL(128); break;
    case 256: SLL(256); break;
    default: return RG_ERR_SHAPE;
  }
#undef SLL
  RG_LAUNCH_CHECK();
  return RG_OK;
}

// ------------------------------------------------------------------- dZ ----
// dZᵀ[s][b] = exp(Zᵀ[s][b] − lse[b])·g for b < B (in place); dbg[s] = Σ_b dZᵀ[s][b]
// in a fixed order (deterministic).  One workgroup per negative s.
__global__ __launch_bounds__(256) void k_sampled_dz(float* __restrict__ ZT, int64_t ldz,
                                                    const float* __restrict__ lse, int B, float gscale,
                                                    float* __restrict__ dbg) {
  __shared__ float red[4];
  const int s = blockIdx.x;
  float* row = ZT + (int64_t)s * ldz;
  float acc = 0.f;
  const int nb4 = B >> 2;
  for (int i = threadIdx.x; i < nb4; i += 256) {
    f4 z = reinterpret_cast<f4*>(row)[i];
    const f4 l = reinterpret_cast<const f4*>(lse)[i];
    f4 d;
#pragma unroll
    for (int q = 0; q < 4; ++q) d[q] = __expf(z[q] - l[q]) * gscale;
    reinterpret_cast<f4*>(row)[i] = d;
    acc += (d[0] + d[1]) + (d[2] + d[3]);
  }
  for (int b = 4 * nb4 + threadIdx.x; b < B; b += 256) {
    const float d = __expf(row[b] - lse[b]) * gscale;
    row[b] = d;
    acc += d;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) dbg[s] = (red[0] + red[1]) + (red[2] + red[3]);
}

extern "C" int rg_sampled_dz(float* ZT, int64_t ldz, const float* lse, int B, int S, float gscale, float* dbg,
                             hipStream_t stream) {
  if (B <= 0 || S <= 0 || ldz < B || (ldz & 3)) return RG_ERR_ARG;
  hipLaunchKernelGGL(k_sampled_dz, dim3(S), dim3(256), 0, stream, ZT, ldz, lse, B, gscale, dbg);
  RG_LAUNCH_CHECK();
  return RG_OK;
}
