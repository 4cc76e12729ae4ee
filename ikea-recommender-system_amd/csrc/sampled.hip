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

// fragment-order plane buffer: common.h plane_idx

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

extern "C" int rg_reduce_slabs(const float* slabs, int nslab, int64_t n, float* out, const float* bias, int ncol,
                               int accumulate, hipStream_t stream);

// split-bf16 logits kernel shared with the full-softmax head (csrc/head_split.hip)
extern "C" int rg_head_fwd_xp(const void* hplanes, const float* W, const float* bias, int B, int A, int HF,
                              int terms, int rpb, float* ZT, int64_t ldz, float* pmax, float* psum, int32_t* parg,
                              int want_sum, hipStream_t stream);

// ------------------------------------- fused split-bf16 logits (HF <= 128) ----
// The north-star step's logits (GRU4Rec at C2 shapes) in ONE
// launch: draw, the negatives' row gather, both operands' exact bf16 split,
// the split-bf16 MFMAs, Z and the (max, Σexp) partials.  Z is stored ROW-major
// (B × ldz, negatives contiguous), so every lane writes its accumulator as
// four 16-B runs of 4 negatives (a quarter of the store instructions of the
// Zᵀ layout).
//
// Workgroup = 512 threads = 8 waves over 256 negatives × 128 rows (grid.x
// negative tiles, grid.y row tiles; an XCD takes whole row tiles with every
// negative tile, so h and the negatives' rows are re-read from its L2).  Wave
// w owns negatives 256·bx + 32w: its 32 fp32 rows are loaded straight into
// the MFMA A-fragment layout (lane (hh, n): row n, k = 16j + 8hh .. +8) and
// split slice by slice right before chunk 0's MFMAs of that slice, so the
// MFMAs start while the rest of the rows are in flight (only plain loads are
// in flight there, so the compiler's vmcnt waits stay per slice).  The 128
// rows of h arrive as four 32-row chunks: fp32 loads into registers one chunk
// ahead, split once by the workgroup into a two-buffer LDS ring in B-fragment
// order (lane-linear 16-B writes), one barrier (LDS only, no memory fence) per
// chunk.  Accumulators alternate, so chunk c's epilogue (+ bias, Z stores,
// max / Σexp) issues under chunk c+1's MFMAs.  The Z stores go through a
// per-wave 4 KB LDS tile (XOR-swizzled, conflict-free both ways) so every
// 16-B store instruction writes eight whole 128-B row segments instead of 32
// rows × 32 B.  Bytes per CU: 128 KB of W rows + 64 KB of h (fp32) in,
// 128 KB of Z out.
//
// Measured at B 4096, S 2048, HF 128 (tools/sampbench.py, MI355X): 24 µs;
// a per-wave stamp breakdown puts ~40% in the prologue (the W rows' fragment
// loads) and the rest at ~2× the MFMA time — see DESIGN.md §4 for the
// variants tried (plane-fed GEMM, LDS-DMA row images, sliced epilogues).
constexpr int SF_NW = 8;   // waves per workgroup (each 32 negatives) up to HF 128
// HF 256: a wave's 32 negatives are 192 VGPRs of operand planes plus 128 of
// fp32 rows in flight, so one wave per SIMD (four per workgroup) and the
// whole 512-entry register file
constexpr int sf_nw(int HF) { return HF <= 128 ? SF_NW : 4; }
constexpr int sf_neg(int HF) { return 32 * sf_nw(HF); }   // negatives per workgroup
constexpr int sf_thr(int HF) { return 64 * sf_nw(HF); }   // threads per workgroup
// rows per workgroup (chunks of 32): 128 up to HF 128; 256 at HF 256, where
// one workgroup fills a CU — the S = 2048, B = 4096 grid (16 × 16) is then
// one round on 256 CUs and every wave splits its negatives' planes once for
// eight h chunks instead of twice for four
constexpr int sf_rows(int HF) { return HF == 256 ? 256 : 128; }

// Diagnostic build only (-DSF_STAMP, tools/sfstamp.py): per-wave s_memrealtime
// stamps at the phase boundaries of k_sampled_logits, read back by rg_sf_stamp_read.
#ifdef SF_STAMP
__device__ uint64_t g_sf_stamp[4096 * 8 * 8];
#define SFD_T(k)                                                                                     \
  do {                                                                                              \
    const uint64_t _t = __builtin_amdgcn_s_memrealtime();                                           \
    if (lane == 0) g_sf_stamp[(((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * 8 + w) * 8 + (k)] = _t; \
  } while (0)
#define SFD_C(k)                                                                                     \
  do {                                                                                              \
    const uint64_t _t = __builtin_amdgcn_s_memtime();                                               \
    if (lane == 0) g_sf_stamp[(((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * 8 + w) * 8 + (k)] = _t; \
  } while (0)
extern "C" int rg_sf_stamp_read(void* dst, int64_t n) {
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_sf_stamp), n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#else
#define SFD_T(k)
#define SFD_C(k)
#endif

// HKP (HF <= 128): h arrives as its bf16 K-planes (hk, written by the GRU
// forward that produced h, rg_gru_fwd_dirs_planes) and each 32-row chunk
// moves global -> LDS by 16-B LDS-DMA: no fp32 h loads, no split, no LDS
// stores in this kernel.
// PF (with PRE, HF <= 128): the pre-gathered rows are fp32 fragments
// (common.h frag_idx), split here right before each slice's MFMAs.
template <int HF, int NT, bool DRAW, bool HKP, bool PRE, bool PF = false>
__global__ __launch_bounds__(sf_thr(HF)) void k_sampled_logits(const float* __restrict__ h, const float* __restrict__ W,
                                                        const float* __restrict__ bias, int32_t* __restrict__ neg,
                                                        uint64_t seed, uint64_t counter, uint64_t A, int B, int S,
                                                        float* __restrict__ Z, int64_t ldz, float* __restrict__ pmax,
                                                        float* __restrict__ psum, float* __restrict__ Wg,
                                                        float* __restrict__ bg, const bf16x8* __restrict__ hk,
                                                        const bf16x8* __restrict__ wp) {
  constexpr int NS = HF / 16;
  constexpr int CH = NS * 192;              // 16-B fragments of one 32-row chunk's planes
  constexpr int ITEMS = 32 * (HF / 8);      // (row, 8-value group) items of one chunk
  constexpr int SF_THR = sf_thr(HF), SF_NEG = sf_neg(HF);
  constexpr int IPT = (ITEMS + SF_THR - 1) / SF_THR;  // per thread (1 at HF <= 128, 8 waves; 4 at HF 256)
  constexpr float L2E = 1.4426950408889634f;
  // HF <= 128: all four h chunks get their own LDS buffer (chunks 1..3 are
  // staged together behind chunk 0's MFMAs: two barriers instead of four,
  // 25.5 -> 22.8 us at C2 shapes); HF 256 (48 KB per chunk) keeps the
  // two-buffer ring with a barrier per chunk
  constexpr bool STAGE = HF <= 128;
  // HF 256 with h's planes (HKP): two-slot ring, chunk c + 1's DMA issued
  // behind the barrier that retires chunk c − 1's slot
  constexpr bool HRING = HKP && !STAGE;
  __shared__ bf16x8 hsA[CH], hsB[CH];
  __shared__ bf16x8 hsC[STAGE ? CH : 1], hsD[STAGE ? CH : 1];
  __shared__ __attribute__((aligned(16))) float sbias[SF_NEG];
  __shared__ f4 ztile[256 * sf_nw(HF)];
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, hh = lane >> 5, l32 = lane & 31;
  SFD_T(0);
  SFD_C(6);
  int bx = blockIdx.x, by = blockIdx.y;
  {
    const int gx = gridDim.x, gy = gridDim.y;
    // XCD x (dispatch i % 8) takes row tiles ≡ x & 3 (mod 4) with negative-tile
    // half x >> 2, so its L2 holds 8 of the 32 h row tiles and half of the
    // negatives' planes (1.5 MB of misses per XCD at C2 instead of 1.9 MB for
    // 4 row tiles × every negative tile: 18.5 -> 17.7 us in the step)
    const int i = blockIdx.y * gx + blockIdx.x;
    if ((gy & 3) == 0 && (gx & 1) == 0) {
      const int k = i >> 3, x = i & 7, hx = gx >> 1;
      by = (x & 3) + 4 * (k / hx);
      bx = (x >> 2) * hx + k % hx;
    } else if ((gy & 7) == 0) {  // row tiles ≡ x (mod 8) with every negative tile
      const int k = i >> 3;
      by = (i & 7) + 8 * (k / gx);
      bx = k % gx;
    }
  }
  const int tile = bx * SF_NEG;
  const int s0 = tile + 32 * w;
  const bool nact = s0 < S;                 // S % 32 == 0
  const bool emit = by == 0;                // row tile 0 publishes ids, Wg, bg
  const int rbase = by * sf_rows(HF);
  const int nch = min(sf_rows(HF), B - rbase) / 32;   // B % 32 == 0
  // ---- h chunk staging: item i -> (group g, row) with the row fastest
  f4 st[IPT][2];
  f4 st2[IPT][2], st3[IPT][2];   // (STAGE: chunks 2, 3)
  auto load_to = [&](f4 (&dst)[IPT][2], int c) __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < IPT; ++q) {
      const int i = tid + SF_THR * q;
      if (i < ITEMS) {
        const float* src = h + (int64_t)(rbase + 32 * c + (i & 31)) * HF + 8 * (i >> 5);
        dst[q][0] = *reinterpret_cast<const f4*>(src);
        dst[q][1] = *reinterpret_cast<const f4*>(src + 4);
      }
    }
  };
  auto load_h = [&](int c) __attribute__((always_inline)) { load_to(st, c); };
  auto store_from = [&](const f4 (&src)[IPT][2], bf16x8* hs) __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < IPT; ++q) {
      const int i = tid + SF_THR * q;
      if (i < ITEMS) {
        const int g = i >> 5, row = i & 31;
        bf16x8 p0, p1, p2;
        split3x8(src[q][0], src[q][1], p0, p1, p2);
        const int e = ((g >> 2) * 2 + (row >> 4)) * 192 + 16 * (g & 3) + (row & 15);   // K-planes (common.h)
        hs[e] = p0;
        hs[e + 64] = p1;
        hs[e + 128] = p2;
      }
    }
  };
  auto store_h = [&](bf16x8* hs) __attribute__((always_inline)) { store_from(st, hs); };
  // chunk c's K-planes (CH contiguous 16-B entries) -> LDS by DMA, sliced over the waves
  auto dma_chunk = [&](bf16x8* hs, int c) __attribute__((always_inline)) {
    const __amdgpu_buffer_rsrc_t r = rg_rsrc(hk + (int64_t)((rbase >> 5) + c) * CH);
#pragma unroll
    for (int q = 0; q < (CH + SF_THR - 1) / SF_THR; ++q) {
      const int e0 = SF_THR * q + 64 * __builtin_amdgcn_readfirstlane(w);   // wave-uniform
      if (e0 < CH) rg_blds16(r, hs + e0, 16 * lane, 16 * e0);
    }
  };
  // ---- this wave's negatives: draw, bias, fp32 rows in A-fragment layout.
  // Vector-memory issue order: bias, h chunk 0, the W rows, h chunk 1;
  // branch-free (a wave without negatives gathers row 0 and stores nothing).
  int id = 0;
  const int s_me = nact ? s0 + l32 : 0;
  if (PRE) {
  } else if (DRAW) {
    id = nact ? draw_id(seed, counter, S, s_me, A) : 0;
  } else {
    id = neg[s_me];
    id = (A > 0 && (uint64_t)(int64_t)id >= A) ? 0 : id;   // guard the gather (callers validate ids)
  }
  const float bl = PRE ? bg[s_me] : bias[id];
  if constexpr (HKP) {
    dma_chunk(hsA, 0);
    __builtin_amdgcn_sched_barrier(0);   // chunk 0's DMA stays ahead of the W loads
  } else {
    load_h(0);
  }
  // PRE: the rows' planes were written in fragment order by the gather launch
  // (rg_gather_neg): 24 whole 1 KB wave-loads, no split here; else the fp32
  // rows straight into the fragment layout, split per slice below
  f4 wr[NS][2];
  bf16x8 a0[NS], a1[NS], a2[NS];
  if constexpr (PF) {
    const int blk = (nact ? s0 : 0) >> 5;
    const f4* wf = reinterpret_cast<const f4*>(wp);
#pragma unroll
    for (int j = 0; j < NS; ++j) {
      wr[j][0] = wf[frag_idx(blk, j, 0, lane, NS)];
      wr[j][1] = wf[frag_idx(blk, j, 1, lane, NS)];
    }
  } else if constexpr (PRE) {
    const int blk = (nact ? s0 : 0) >> 5;
#pragma unroll
    for (int j = 0; j < NS; ++j) {
      a0[j] = wp[plane_idx(blk, j, 0, lane, NS)];
      a1[j] = wp[plane_idx(blk, j, 1, lane, NS)];
      a2[j] = wp[plane_idx(blk, j, 2, lane, NS)];
    }
  } else {
    const float* src = W + (int64_t)id * HF + 8 * hh;
#pragma unroll
    for (int j = 0; j < NS; ++j) {
      wr[j][0] = *reinterpret_cast<const f4*>(src + 16 * j);
      wr[j][1] = *reinterpret_cast<const f4*>(src + 16 * j + 4);
    }
  }
  __builtin_amdgcn_sched_barrier(0);
  // barrier without a memory fence: only the LDS writes must be complete
  // (the W rows and h chunk 1 stay in flight); same for every barrier below
  auto sync_lds = [&]() __attribute__((always_inline)) {
    __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0), vmcnt / expcnt free
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  if constexpr (HRING) {
    if (hh == 0) sbias[32 * w + l32] = bl;
    __syncthreads();   // chunk 0's planes, the W rows / planes and the biases
    if (nch > 1) dma_chunk(hsB, 1);
    SFD_T(1);
  } else if constexpr (HKP) {
    if (hh == 0) sbias[32 * w + l32] = bl;
    // every chunk's DMA is issued up front; one full wait + barrier (the W
    // rows are needed by chunk 0 anyway), then all MFMAs run barrier-free
    // (21.7 -> 21.4 us against a second barrier behind chunk 0; with the
    // pre-gathered planes the two forms measure the same)
    if (nch > 1) dma_chunk(hsB, 1);
    if (nch > 2) dma_chunk(hsC, 2);
    if (nch > 3) dma_chunk(hsD, 3);
    __syncthreads();
    SFD_T(1);
  } else {
    store_h(hsA);
    if (nch > 1) load_h(1);
    if constexpr (STAGE) {
      if (nch > 2) load_to(st2, 2);
      if (nch > 3) load_to(st3, 3);
    }
    if (hh == 0) sbias[32 * w + l32] = bl;
    sync_lds();
  }
  float* __restrict__ pm = pmax + (int64_t)(s0 / 32) * B + rbase + l32;
  float* __restrict__ ps = psum + (int64_t)(s0 / 32) * B + rbase + l32;
  // B fragment of 16-deep slice j (lane (hh, n): row n, k = 16j + 8hh .. +8)
  // inside a chunk's K-planes (common.h: [k32 slice][16-row tile][plane][16·kg + n])
  auto boff = [&](int j) __attribute__((always_inline)) {
    return ((j >> 1) * 2 + (l32 >> 4)) * 192 + 16 * (2 * (j & 1) + hh) + (l32 & 15);
  };
  // chunk 0: each A slice is split right before its MFMAs
  f16v accA = {}, accB = {};
#pragma unroll
  for (int j = 0; j < NS; ++j) {
    if constexpr (!PRE || PF) split3x8(wr[j][0], wr[j][1], a0[j], a1[j], a2[j]);
    accA = mfma_split<NT>(a0[j], a1[j], a2[j], hsA[boff(j)], hsA[boff(j) + 64], hsA[boff(j) + 128], accA);
  }
  // row tile 0 publishes the draw and the gathered rows (the backward's Wg / bg)
  if (!PRE && emit && nact) {
    if (hh == 0) {
      if (DRAW) neg[s0 + l32] = id;
      if (bg) bg[s0 + l32] = bl;
    }
    if (Wg) {
      float* dst = Wg + (int64_t)(s0 + l32) * HF + 8 * hh;
#pragma unroll
      for (int j = 0; j < NS; ++j) {
        *reinterpret_cast<f4*>(dst + 16 * j) = wr[j][0];
        *reinterpret_cast<f4*>(dst + 16 * j + 4) = wr[j][1];
      }
    }
  }
  auto mma = [&](const bf16x8* hs, f16v& acc) __attribute__((always_inline)) {
    acc = f16v{};
#pragma unroll
    for (int j = 0; j < NS; ++j)
      acc = mfma_split<NT>(a0[j], a1[j], a2[j], hs[boff(j)], hs[boff(j) + 64], hs[boff(j) + 128], acc);
  };
  // epilogue of chunk c: lane (hh, n) holds row rbase + 32c + n, negatives
  // s0 + acc32_row(r, hh): four runs of 4 consecutive negatives
  auto epi = [&](f16v& acc, int c) __attribute__((always_inline)) {
    float m = -__builtin_inff();
    f4* zt = ztile + 256 * w;   // this wave's 32 × 32 tile, 16-B group g of row n at n·8 + (g ^ (n & 7))
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f4 bq = *reinterpret_cast<const f4*>(&sbias[32 * w + 8 * q + 4 * hh]);
      f4 z;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        z[u] = acc[4 * q + u] + bq[u];
        acc[4 * q + u] = z[u];
        m = fmaxf(m, z[u]);
      }
      zt[8 * l32 + ((2 * q + hh) ^ (l32 & 7))] = z;
    }
    // whole 128-B row segments: lane (n8, g) stores row 8q + n8, negatives s0 + 4g .. +3
    {
      const int n8 = lane >> 3, g = lane & 7;
      float* zr = Z + (int64_t)(rbase + 32 * c + n8) * ldz + s0 + 4 * g;
#pragma unroll
      for (int q = 0; q < 4; ++q)
        *reinterpret_cast<f4*>(zr + (int64_t)(8 * q) * ldz) = zt[8 * (8 * q + n8) + (g ^ n8)];
    }
    m = fmaxf(m, __shfl_xor(m, 32));
    const float m2 = m * L2E;
    float sum = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) sum += __builtin_amdgcn_exp2f(fmaf(acc[r], L2E, -m2));
    sum += __shfl_xor(sum, 32);
    if (hh == 0) {
      pm[32 * c] = m;
      ps[32 * c] = sum;
    }
  };
  // chunk c (>= 1): its rows (in registers since chunk c-1) are split into LDS
  // buffer c & 1 (last read by chunk c-2, before the previous barrier), chunk
  // c+1's rows are loaded, and its MFMAs carry chunk c-1's epilogue
  auto step = [&](int c, bf16x8* hs_cur, f16v& acc_new, f16v& acc_old) __attribute__((always_inline)) {
    store_h(hs_cur);
    if (c + 1 < nch) load_h(c + 1);
    sync_lds();
    if (nact) {
      mma(hs_cur, acc_new);
      epi(acc_old, c - 1);
    }
  };
  if constexpr (HRING) {
    // step c: chunk c landed and every wave is done with chunk c − 1's slot ->
    // DMA chunk c + 1 into it -> chunk c's MFMAs with chunk c − 1's epilogue
    auto step_k = [&](int c, const bf16x8* hs_cur, bf16x8* hs_nxt, f16v& acc_new, f16v& acc_old)
                      __attribute__((always_inline)) {
      __syncthreads();
      if (c + 1 < nch) dma_chunk(hs_nxt, c + 1);
      if (nact) {
        mma(hs_cur, acc_new);
        epi(acc_old, c - 1);
      }
    };
    int c = 1;
    for (; c + 1 < nch; c += 2) {
      step_k(c, hsB, hsA, accB, accA);
      step_k(c + 1, hsA, hsB, accA, accB);
    }
    if (c < nch) step_k(c, hsB, hsA, accB, accA);
    if (nact) {
      if ((nch - 1) & 1) epi(accB, nch - 1);
      else epi(accA, nch - 1);
    }
  } else if constexpr (HKP) {
    // chunks 1..3 landed at the first barrier
    if (nch > 1) {
      if (nact) {
        mma(hsB, accB);
        epi(accA, 0);
        SFD_T(2);
        if (nch > 2) {
          mma(hsC, accA);
          epi(accB, 1);
          SFD_T(3);
          if (nch > 3) {
            mma(hsD, accB);
            epi(accA, 2);
            SFD_T(4);
            epi(accB, 3);
            SFD_T(5);
            SFD_C(7);
          } else {
            epi(accA, 2);
          }
        } else {
          epi(accB, 1);
        }
      }
    } else if (nact) {
      epi(accA, 0);
    }
  } else if constexpr (STAGE) {
    // chunks 1..3 (loaded before chunk 0's MFMAs) are split into their own LDS
    // buffers behind those MFMAs, one more barrier, then the remaining MFMAs
    // run back to back with the epilogues interleaved: 2 barriers, not 4
    if (nch > 1) {
      store_from(st, hsB);
      if (nch > 2) store_from(st2, hsC);
      if (nch > 3) store_from(st3, hsD);
      sync_lds();
      if (nact) {
        mma(hsB, accB);
        epi(accA, 0);
        if (nch > 2) {
          mma(hsC, accA);
          epi(accB, 1);
          if (nch > 3) {
            mma(hsD, accB);
            epi(accA, 2);
            epi(accB, 3);
          } else {
            epi(accA, 2);
          }
        } else {
          epi(accB, 1);
        }
      }
    } else if (nact) {
      epi(accA, 0);
    }
  } else {
    // chunk c: LDS buffer and accumulator c & 1 (A even, B odd)
    int c = 1;
    for (; c + 1 < nch; c += 2) {
      step(c, hsB, accB, accA);
      step(c + 1, hsA, accA, accB);
    }
    if (c < nch) step(c, hsB, accB, accA);
    if (nact) {
      if ((nch - 1) & 1) epi(accB, nch - 1);
      else epi(accA, nch - 1);
    }
  }
}

// The fused forward (k_sampled_logits): Z row-major (B × ldz, ldz >= S).
// draw: 0 = the S ids are given in neg; 1 = draw them (counter-based stream)
// and publish ids, bg and the rows Wg; 2 = pre-gathered by rg_gather_neg in
// the step's embedding-gather launch: neg / bg / Wg already hold the ids,
// biases and rows and w_planes their fragment-order bf16 planes; 3 = the same
// with w_planes holding the rows as fp32 fragments (rg_gather_neg wfmt 1,
// HF <= 128).
extern "C" int rg_sampled_logits(const float* h, const float* W, const float* bias, int32_t* neg, int draw,
                                 uint64_t seed, uint64_t counter, int64_t A, int B, int S, int HF, int terms,
                                 float* Z, int64_t ldz, float* pmax, float* psum, float* Wg, float* bg,
                                 const void* h_planes, const void* w_planes, hipStream_t stream) {
  if (B <= 0 || S <= 0 || (B % 32) || (S % 32) || !h || !W || !bias || !neg || !Z || !pmax || !psum || !bg)
    return RG_ERR_ARG;
  if (ldz < S || (ldz & 3)) return RG_ERR_ARG;
  if (draw < 0 || draw > 3 || (draw >= 2 && !w_planes)) return RG_ERR_ARG;
  if (draw == 3 && HF > 128) return RG_ERR_ARG;
  if (draw == 1 && (A <= 0 || A > INT32_MAX)) return RG_ERR_ARG;
  if (terms != 6 && terms != 9) return RG_ERR_ARG;
  const int neg_wg = sf_neg(HF);
  const int rows_wg = sf_rows(HF);
  const dim3 grid((unsigned)((S + neg_wg - 1) / neg_wg), (unsigned)((B + rows_wg - 1) / rows_wg));
  const bf16x8* hk = (const bf16x8*)h_planes;
  const bf16x8* wp = (const bf16x8*)w_planes;
#define SFH(HFV, NTV, DRV, HKV, PRV, ...)                                                                          \
  RG_TLAUNCH((k_sampled_logits<HFV, NTV, DRV, HKV, PRV, ##__VA_ARGS__>), grid, dim3(sf_thr(HFV)), 0, stream, h, W, \
             bias, neg, seed, counter, (uint64_t)(A > 0 ? A : 0), B, S, Z, ldz, pmax, psum, Wg, bg, hk, wp)
#define SFG(HFV, NTV)                                     \
  if (hk) {                                               \
    if (draw == 3) SFH(HFV, NTV, false, true, true, HFV <= 128); \
    else if (draw == 2) SFH(HFV, NTV, false, true, true); \
    else if (draw) SFH(HFV, NTV, true, true, false);      \
    else SFH(HFV, NTV, false, true, false);               \
  } else {                                                \
    if (draw == 3) SFH(HFV, NTV, false, false, true, HFV <= 128); \
    else if (draw == 2) SFH(HFV, NTV, false, false, true); \
    else if (draw) SFH(HFV, NTV, true, false, false);     \
    else SFH(HFV, NTV, false, false, false);              \
  }
#define SFT(HFV)    \
  if (terms == 9) { \
    SFG(HFV, 9);    \
  } else {          \
    SFG(HFV, 6);    \
  }
  switch (HF) {
    case 32: SFT(32); break;
    case 64: SFT(64); break;
    case 128: SFT(128); break;
    case 256: SFT(256); break;
    default: return RG_ERR_SHAPE;
  }
#undef SFT
#undef SFG
#undef SFH
  RG_LAUNCH_CHECK();
  return RG_OK;
}

// dZ = exp(Z − lse)·g in place for the row-major Z of rg_sampled_logits, and
// the bias gradient dbg[s] = Σ_b dZ[b][s]: workgroup (s block of 256, row
// block of 128) writes its column sums to slab[row block][s]; the slabs are
// then summed in order (deterministic).
__global__ __launch_bounds__(256) void k_sampled_dz_rows(float* __restrict__ Z, int64_t ldz,
                                                         const float* __restrict__ lse, int B, int S, float g,
                                                         float* __restrict__ slabs) {
  const int s = blockIdx.x * 256 + threadIdx.x;
  const int b0 = blockIdx.y * 128, b1 = min(B, b0 + 128);
  if (s >= S) return;
  float acc = 0.f;
  for (int b = b0; b < b1; ++b) {
    float* p = Z + (int64_t)b * ldz + s;
    const float d = __expf(*p - lse[b]) * g;
    *p = d;
    acc += d;
  }
  slabs[(int64_t)blockIdx.y * S + s] = acc;
}

extern "C" int rg_sampled_dz_rows(float* Z, int64_t ldz, const float* lse, int B, int S, float gscale, float* slabs,
                                  float* dbg, hipStream_t stream) {
  if (B <= 0 || S <= 0 || ldz < S || !Z || !lse || !slabs || !dbg) return RG_ERR_ARG;
  const int nrb = (B + 127) / 128;
  hipLaunchKernelGGL(k_sampled_dz_rows, dim3((S + 255) / 256, nrb), dim3(256), 0, stream, Z, ldz, lse, B, S, gscale,
                     slabs);
  RG_LAUNCH_CHECK();
  return rg_reduce_slabs(slabs, nrb, S, dbg, nullptr, S, 0, stream);
}

// bytes of scratch rg_sampled_fwd_x needs (the negatives' and h's operand planes)
extern "C" int64_t rg_sampled_work_bytes(int B, int S, int HF) {
  if (B <= 0 || S <= 0 || HF <= 0) return RG_ERR_ARG;
  return ((int64_t)S + B) * HF * 6;
}

// Split-bf16 forward (terms = 9: exact products, fp32 accumulation; 6: the
// three sub-ulp terms dropped) in the Zᵀ layout of rg_sampled_fwd; needs
// S % 32 == 0 and B % 32 == 0.  draw = 1: neg is an output, filled with the
// rg_sample_uniform(seed, counter) draw.  Two launches: operand prep (draw,
// the negatives' row gather -> Wg/bg, h's planes), then rg_head_fwd_xp with
// the gathered rows as the items.  (HF <= 128 trainers use the one-launch
// row-major rg_sampled_logits above.)
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
  bf16x8* Hp = reinterpret_cast<bf16x8*>(work) + (int64_t)S * HF / 8 * 3;
  const int64_t items = ((int64_t)S + B) * (HF / 8);
  const dim3 gp((unsigned)((items + 255) / 256));
#define SXP(HFV)                                                                                            \
  hipLaunchKernelGGL(k_sampled_prep<HFV>, gp, dim3(256), 0, stream, h, W, bias, neg, draw, seed, counter, \
                     (uint64_t)A, B, S, Wg, bg, (bf16x8*)nullptr, Hp)
  switch (HF) {
    case 32: SXP(32); break;
    case 64: SXP(64); break;
    case 128: SXP(128); break;
    case 256: SXP(256); break;
    default: return RG_ERR_SHAPE;
  }
#undef SXP
  RG_LAUNCH_CHECK();
  // negatives × rows on k_head_fwd_x (csrc/head_split.hip): each wave holds
  // 32 gathered negatives' planes in VGPRs, h's planes stream through LDS; the
  // rows are split over grid.y so the S/(32·waves) negative groups fill the chip
  const int nw = HF >= 256 ? 4 : 8;
  const int ngx = (S + 32 * nw - 1) / (32 * nw);
  const int ny = max(1, 256 / ngx);
  // rows per workgroup (rows·negatives workgroups ≈ one per CU; the best of
  // 32..512 swept at B 4096, S 2048: 128 at HF 128, 256 at HF 256)
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

// ------------------------------------------------------------------ BPR ----
// Sampled BPR (Rendle et al. 2009; the GRU4Rec paper's pairwise loss) over the
// same logits — build-defined like the sampled softmax (SURVEY §8 A7 ext.,
// north_star "sampled-softmax/BPR logits"):
//   loss = mean_b (1/S) Σ_s −log σ(z_b,pos − z_b,s) = mean_b (1/S) Σ_s softplus(z_b,s − z_b,pos)
//   ∂loss/∂z_b,s = g·σ(z_b,s − z_b,pos)/S,   ∂loss/∂z_b,pos = −Σ_s ∂loss/∂z_b,s      (g = 1/B)
// Z element (b, s) lives at Z[b·zsb + s·zss]: row-major Z of rg_sampled_logits
// (zsb = ldz, zss = 1) or the Zᵀ of rg_sampled_fwd / rg_sampled_fwd_x (zsb = 1,
// zss = ldz).  k_bpr_rows: one wave per row — the positive logit (fp32 dot),
// Σ softplus and Σ σ over the row's S logits, loss row (NaN for a target
// outside [0, A)), zpos, and the positive's gradient rows as k_sampled_lse.
__device__ __forceinline__ float softplusf_acc(float x) { return fmaxf(x, 0.f) + log1pf(expf(-fabsf(x))); }
__device__ __forceinline__ float sigmoidf_acc(float x) {
  if (x >= 0.f) return 1.f / (1.f + expf(-x));
  const float e = expf(x);
  return e / (1.f + e);
}

template <int HF>
__global__ __launch_bounds__(256) void k_bpr_rows(const float* __restrict__ h, const float* __restrict__ W,
                                                  const float* __restrict__ bias, const int64_t* __restrict__ tgt,
                                                  int B, int64_t A, const float* __restrict__ Z, int64_t zsb,
                                                  int64_t zss, int S, float gscale, float* __restrict__ zpos,
                                                  float* __restrict__ loss_row, int32_t* __restrict__ ids,
                                                  float* __restrict__ dzpos, float* __restrict__ gpos,
                                                  float* __restrict__ dhpos) {
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
  float sp = 0.f, sg = 0.f;
  const float* zr = Z + (int64_t)b * zsb;
  for (int s = lane; s < S; s += 64) {
    const float x = zr[(int64_t)s * zss] - zp;
    sp += softplusf_acc(x);
    sg += sigmoidf_acc(x);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    sp += __shfl_xor(sp, o);
    sg += __shfl_xor(sg, o);
  }
  const float inv_s = 1.f / (float)S;
  const float dp = -gscale * sg * inv_s;
  if (lane == 0) {
    zpos[b] = zp;
    loss_row[b] = ok ? sp * inv_s : __builtin_nanf("");
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

extern "C" int rg_bpr_rows(const float* h, const float* W, const float* bias, const int64_t* tgt, int B, int64_t A,
                           int HF, const float* Z, int64_t zsb, int64_t zss, int S, float gscale, float* zpos,
                           float* loss_row, int32_t* ids, float* dzpos, float* gpos, float* dhpos,
                           hipStream_t stream) {
  if (B <= 0 || A <= 0 || S <= 0 || !Z || zsb <= 0 || zss <= 0) return RG_ERR_ARG;
  dim3 grid((B + 3) / 4);
#define BPR(HFV)                                                                                            \
  hipLaunchKernelGGL(k_bpr_rows<HFV>, grid, dim3(256), 0, stream, h, W, bias, tgt, B, A, Z, zsb, zss, S, \
                     gscale, zpos, loss_row, ids, dzpos, gpos, dhpos)
  switch (HF) {
    case 32: BPR(32); break;
    case 64: BPR(64); break;
    case 128: BPR(128); break;
    case 256: BPR(256); break;
    default: return RG_ERR_SHAPE;
  }
#undef BPR
  RG_LAUNCH_CHECK();
  return RG_OK;
}

// dZ(b, s) = g·σ(Z(b, s) − zpos[b])/S in place; workgroup (256 negatives,
// 128 rows) writes its column sums to slab[row block][s], summed in order
// (deterministic) into dbg[s] = Σ_b dZ(b, s).
__global__ __launch_bounds__(256) void k_bpr_dz(float* __restrict__ Z, int64_t zsb, int64_t zss,
                                                const float* __restrict__ zpos, int B, int S, float gs,
                                                float* __restrict__ slabs) {
  const int s = blockIdx.x * 256 + threadIdx.x;
  const int b0 = blockIdx.y * 128, b1 = min(B, b0 + 128);
  if (s >= S) return;
  float acc = 0.f;
  for (int b = b0; b < b1; ++b) {
    float* p = Z + (int64_t)b * zsb + (int64_t)s * zss;
    const float d = sigmoidf_acc(*p - zpos[b]) * gs;
    *p = d;
    acc += d;
  }
  slabs[(int64_t)blockIdx.y * S + s] = acc;
}

extern "C" int rg_bpr_dz(float* Z, int64_t zsb, int64_t zss, const float* zpos, int B, int S, float gscale,
                         float* slabs, float* dbg, hipStream_t stream) {
  if (B <= 0 || S <= 0 || !Z || zsb <= 0 || zss <= 0 || !zpos || !slabs || !dbg) return RG_ERR_ARG;
  const int nrb = (B + 127) / 128;
  hipLaunchKernelGGL(k_bpr_dz, dim3((S + 255) / 256, nrb), dim3(256), 0, stream, Z, zsb, zss, zpos, B, S,
                     gscale / (float)S, slabs);
  RG_LAUNCH_CHECK();
  return rg_reduce_slabs(slabs, nrb, S, dbg, nullptr, S, 0, stream);
}
