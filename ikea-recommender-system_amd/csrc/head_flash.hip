// Full-softmax output head, training step without Z (SURVEY §8 A6/A7/A8;
// reference GRU4Rec/model.py:58-60 Linear, :80 logits, :121/146 CE(mean),
// :149-153 Adam).  Split-bf16 MFMAs (precision f32x9 / f32x6, common.h).
//
// The head's three contractions over the (B × A) logits — Z = h·Wᵀ + b,
// dh = dZ·W, dW = dZᵀ·h with dZ = g·(softmax(Z) − onehot) — are regrouped
// into two passes that never write Z to HBM (16.4 GB at C2):
//
//  pass 1  rg_flash_fwd   workgroup = 256 rows × one item split.  Per
//          32-item chunk: Sᵀ = W_c·hᵀ (h held in VGPRs), online row max /
//          Σexp, P = 2^(S−m) split to bf16 planes IN REGISTERS (the Sᵀ
//          accumulator is already the B-operand layout of the next MFMA),
//          Oᵀ += W_cᵀ·Pᵀ with the running-max rescale.  Per (split, row):
//          m, Σexp, O = Σ_j 2^(S_j−m)·W_j.
//  combine rg_flash_lse   lse over the splits, target logit (fp32 dot).
//          rg_flash_rows  packed (lse·log2e, local target) row records.
//          rg_flash_dh    dh = g·(Σ_splits 2^(m_s−lse)·O_s − W[target]).
//  pass 2  rg_flash_dw_adam  workgroup = 256 items (W in VGPRs), streams h:
//          S = h_c·Wᵀ recomputed, P = g·(2^(S−lse) − onehot) in registers
//          (the S accumulator is the A-operand layout of dW = Pᵀ·h_c),
//          db = Σ_rows P, then Adam on W/b in the epilogue.
// Item shards (multi-GPU): W rows are items [lo, hi); lse is merged over
// ranks between rg_flash_lse and rg_flash_rows; targets outside the shard
// carry −1 and never match a local item.
//
// MFMA 32x32x16 fragment conventions (common.h acc32_row): operand lane l
// carries row/col l%32 and k group l/32 (8 values); accumulator register r
// of lane l is C[acc32_row(r, l/32)][l%32].  The k order inside a 16-deep
// slice is free as long as both operands agree, so a 32-row accumulator
// block (registers 8s..8s+7 = rows 16s + kperm(l/32, i)) feeds the next
// MFMA as its k = 32 operand with no data movement.
//
// Operand planes (16-B bf16x8 entries, one 32-row block contiguous):
//   K-planes  [x/32][s < HF/16][p < 3][lane]: lane = hh·32 + x%32 holds
//             X[x][16s + 8hh + 0..7]                     (k over features)
//   R-planes  [x/32][t < HF/32][s < 2][p < 3][lane]: lane = hh·32 + n holds
//             X[32(x/32) + 16s + kperm(hh, i)][32t + n]  (k over rows)
// Both are lane-linear per wave, so chunks move global → LDS with 16-byte
// LDS-DMA (global_load_lds_dwordx4) and are read back by ds_read_b128.
#include "common.h"

#define NEG_INF (-__builtin_inff())

namespace {

constexpr float L2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;
constexpr int FL_WAVES = 8;   // waves per workgroup (2 per SIMD)
constexpr int FL_T = 64 * FL_WAVES;

// element i of lane half hh inside a 16-deep k slice -> row offset
__device__ __forceinline__ int kperm(int hh, int i) { return (i & 3) + 8 * (i >> 2) + 4 * hh; }

// 16-byte global -> LDS DMA; LDS address = wave-uniform base + 16·lane
__device__ __forceinline__ void glds16(const void* src, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)const_cast<void*>(src),
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

// copy E 16-B entries (E % 64 == 0) from global to LDS, wave-sliced
template <int E>
__device__ __forceinline__ void stage(const bf16x8* __restrict__ src, bf16x8* dst, int w, int lane) {
#pragma unroll
  for (int q = 0; q < (E + FL_T - 1) / FL_T; ++q) {
    const int e0 = FL_T * q + 64 * w;  // wave-uniform
    if (e0 < E) glds16(src + e0 + lane, dst + e0);
  }
}

// ------------------------------------------------------------- planes ----
template <int HF>
__global__ __launch_bounds__(256) void k_planes_k(const float* __restrict__ X, int rows, int rows_pad,
                                                  bf16x8* __restrict__ P) {
  constexpr int G = HF / 8, NS = HF / 16;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)rows_pad * G) return;
  const int x = (int)(i / G), g = (int)(i % G);
  f4 lo = {0.f, 0.f, 0.f, 0.f}, hi = lo;
  if (x < rows) {
    lo = *reinterpret_cast<const f4*>(X + (int64_t)x * HF + 8 * g);
    hi = *reinterpret_cast<const f4*>(X + (int64_t)x * HF + 8 * g + 4);
  }
  bf16x8 p0, p1, p2;
  split3x8(lo, hi, p0, p1, p2);
  const int64_t base = ((int64_t)(x >> 5) * NS + (g >> 1)) * 192 + (g & 1) * 32 + (x & 31);
  P[base] = p0;
  P[base + 64] = p1;
  P[base + 128] = p2;
}

template <int HF>
__global__ __launch_bounds__(256) void k_planes_r(const float* __restrict__ X, int rows, int rows_pad,
                                                  bf16x8* __restrict__ P) {
  constexpr int NTL = HF / 32;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)(rows_pad / 32) * NTL * 2 * 64) return;
  const int lane = (int)(i & 63);
  int64_t q = i >> 6;
  const int s = (int)(q & 1);
  q >>= 1;
  const int t = (int)(q % NTL);
  const int64_t c = q / NTL;
  const int hh = lane >> 5, col = 32 * t + (lane & 31);
  f4 lo, hi;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int64_t row = 32 * c + 16 * s + kperm(hh, e);
    const float v = row < rows ? X[row * HF + col] : 0.f;
    if (e < 4) lo[e] = v; else hi[e - 4] = v;
  }
  bf16x8 p0, p1, p2;
  split3x8(lo, hi, p0, p1, p2);
  const int64_t base = ((c * NTL + t) * 2 + s) * 192 + lane;
  P[base] = p0;
  P[base + 64] = p1;
  P[base + 128] = p2;
}

__global__ void k_pad_bias(const float* __restrict__ bias, int A, int Ap, float* __restrict__ out) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j < Ap) out[j] = j < A ? bias[j] : NEG_INF;
}

// ------------------------------------------------------------- pass 1 ----
// The chunk ring is two SEPARATE LDS arrays per operand and the loop is
// unrolled by two: the compiler orders LDS reads only behind the DMA into the
// same array, so chunk c's MFMAs start while chunk c+1's DMA is in flight
// (with one [2][E] array it waited for the just-issued prefetch every chunk).
template <int HF, int NT>
__global__ __launch_bounds__(FL_T) void k_flash_fwd(const bf16x8* __restrict__ Hk, const bf16x8* __restrict__ Wk,
                                                    const bf16x8* __restrict__ Wr,
                                                    const float* __restrict__ bias_pad, int B, int A, int nrb,
                                                    int nsplit, int cps, float* __restrict__ pm,
                                                    float* __restrict__ pl, float* __restrict__ pO) {
  constexpr int NS = HF / 16, NTL = HF / 32;
  constexpr int EK = NS * 192;        // entries per 32-row block, K-planes
  constexpr int ER = NTL * 2 * 192;   // R-planes (== EK)
  __shared__ bf16x8 sk0[EK], sk1[EK];
  __shared__ bf16x8 sr0[ER], sr1[ER];
  __shared__ __attribute__((aligned(16))) float sb0[32], sb1[32];
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, hh = lane >> 5, l32 = lane & 31;
  // XCD-aware order: the nrb row blocks of one item split are dispatched to
  // the same XCD (round-robin dispatch), so its W chunks are fetched once
  // into that XCD's L2 and re-read from there
  int bid = blockIdx.x;
  const int total = nrb * nsplit;
  if ((total & 7) == 0) bid = (bid & 7) * (total >> 3) + (bid >> 3);
  const int split = bid / nrb, rb = bid % nrb;
  const int r0 = rb * 32 * FL_WAVES + 32 * w;
  const bool active = r0 < B;
  const int nct = (A + 31) / 32;
  const int c0 = split * cps;
  const int nch = max(0, min(nct, c0 + cps) - c0);
#define FL_ISSUE(C, SK, SR, SB)                                                  \
  do {                                                                           \
    stage<EK>(Wk + (int64_t)(C) * EK, SK, w, lane);                              \
    stage<ER>(Wr + (int64_t)(C) * ER, SR, w, lane);                              \
    if (w == 0 && lane < 8) glds16(bias_pad + 32 * (C) + 4 * lane, SB);          \
    __builtin_amdgcn_sched_barrier(0); /* keep the prefetch at the top */ \
  } while (0)
  if (nch > 0) FL_ISSUE(c0, sk0, sr0, sb0);
  // this wave's 32 rows of h (B operand of Sᵀ = W_c·hᵀ) for the whole split
  bf16x8 hk[NS][3];
#pragma unroll
  for (int s = 0; s < NS; ++s)
#pragma unroll
    for (int p = 0; p < 3; ++p)
      hk[s][p] = active ? Hk[((int64_t)(r0 >> 5) * NS + s) * 192 + p * 64 + lane] : bf16x8{};
  f16v o[NTL];
#pragma unroll
  for (int t = 0; t < NTL; ++t) o[t] = f16v{};
  float m = NEG_INF, l = 0.f;
  __syncthreads();
  auto chunk = [&](const bf16x8* sk, const bf16x8* sr, const float* sb) __attribute__((always_inline)) {
    f16v sa = {};
#pragma unroll
    for (int s = 0; s < NS; ++s)
      sa = mfma_split<NT>(sk[s * 192 + lane], sk[s * 192 + 64 + lane], sk[s * 192 + 128 + lane], hk[s][0], hk[s][1],
                          hk[s][2], sa);
    // logits in log2 units (item acc32_row(r, hh) of the chunk, row l32)
    float cm = NEG_INF;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f4 bq = *reinterpret_cast<const f4*>(&sb[8 * q + 4 * hh]);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float z = (sa[4 * q + u] + bq[u]) * L2E;
        sa[4 * q + u] = z;
        cm = fmaxf(cm, z);
      }
    }
    cm = fmaxf(cm, __shfl_xor(cm, 32));
    const float mn = fmaxf(m, cm);
    if (__any(mn > m)) {
      const float a = mn > m ? __builtin_amdgcn_exp2f(m - mn) : 1.f;
#pragma unroll
      for (int t = 0; t < NTL; ++t) o[t] *= a;
      l *= a;
      m = mn;
    }
    const float mm = m == NEG_INF ? 0.f : m;
    float ps = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float p = __builtin_amdgcn_exp2f(sa[r] - mm);
      sa[r] = p;
      ps += p;
    }
    l += ps;
    bf16x8 q0[2], q1[2], q2[2];
#pragma unroll
    for (int s = 0; s < 2; ++s)
      split3x8(f4{sa[8 * s], sa[8 * s + 1], sa[8 * s + 2], sa[8 * s + 3]},
               f4{sa[8 * s + 4], sa[8 * s + 5], sa[8 * s + 6], sa[8 * s + 7]}, q0[s], q1[s], q2[s]);
#pragma unroll
    for (int t = 0; t < NTL; ++t)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int e = (t * 2 + s) * 192 + lane;
        o[t] = mfma_split<NT>(sr[e], sr[e + 64], sr[e + 128], q0[s], q1[s], q2[s], o[t]);
      }
  };
  for (int c = 0; c < nch; c += 2) {
    if (c + 1 < nch) FL_ISSUE(c0 + c + 1, sk1, sr1, sb1);
    if (active) chunk(sk0, sr0, sb0);
    __syncthreads();
    if (c + 1 < nch) {
      if (c + 2 < nch) FL_ISSUE(c0 + c + 2, sk0, sr0, sb0);
      if (active) chunk(sk1, sr1, sb1);
      __syncthreads();
    }
  }
#undef FL_ISSUE
  if (!active) return;
  l += __shfl_xor(l, 32);
  const int row = r0 + l32;
  if (hh == 0) {
    pm[(int64_t)split * B + row] = m;
    pl[(int64_t)split * B + row] = l;
  }
#pragma unroll
  for (int t = 0; t < NTL; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r)
      pO[((int64_t)split * HF + 32 * t + acc32_row(r, hh)) * B + row] = o[t][r];
}

// ------------------------------------------------------------ combine ----
// lse over the splits (natural units) and, when the target is one of this
// shard's items [lo, lo + A), its logit z = h·W[t] + b[t]; 0 for a target
// held by another shard, NaN for one outside [0, A_full) (CrossEntropyLoss
// raises there; the native head writes a NaN loss row, head.hip k_lse_combine)
__global__ __launch_bounds__(256) void k_flash_lse(const float* __restrict__ pm, const float* __restrict__ pl,
                                                   int nsplit, const float* __restrict__ h,
                                                   const float* __restrict__ W, const float* __restrict__ bias,
                                                   const int64_t* __restrict__ tgt, int64_t lo, int A,
                                                   int64_t A_full, int B, int HF, float* __restrict__ lse,
                                                   float* __restrict__ zt) {
  const int b = blockIdx.x * 256 + threadIdx.x;
  if (b >= B) return;
  float M = NEG_INF;
  for (int s = 0; s < nsplit; ++s) M = fmaxf(M, pm[(int64_t)s * B + b]);
  float L = 0.f;
  for (int s = 0; s < nsplit; ++s) {
    const float ms = pm[(int64_t)s * B + b];
    if (ms != NEG_INF) L += pl[(int64_t)s * B + b] * exp2f(ms - M);
  }
  lse[b] = (M + log2f(L)) * LN2;
  if (zt) {
    const int64_t t = tgt[b] - lo;
    float z = (tgt[b] >= 0 && tgt[b] < A_full) ? 0.f : __builtin_nanf("");
    if (t >= 0 && t < A) {
      for (int k = 0; k < HF; ++k) z = fmaf(h[(int64_t)b * HF + k], W[t * HF + k], z);
      z += bias[t];
    }
    zt[b] = z;
  }
}

// (lse·log2e, local target or −1) per row: what pass 2 stages through LDS
__global__ void k_flash_rows(const float* __restrict__ lse, const int64_t* __restrict__ tgt, int64_t lo, int A, int B,
                             float2* __restrict__ rowinfo) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const int64_t t = tgt[b] - lo;
  rowinfo[b] = make_float2(lse[b] * L2E, __int_as_float(t >= 0 && t < A ? (int)t : -1));
}

// dh[b][k] = g·(Σ_s 2^(m_s − lse2_b)·O_s[k][b] − W[t_b][k])
__global__ __launch_bounds__(256) void k_flash_dh(const float* __restrict__ pm, const float* __restrict__ pO,
                                                  const float2* __restrict__ rowinfo, int nsplit,
                                                  const float* __restrict__ W, float g, int B, int HF,
                                                  float* __restrict__ dh) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)B * HF) return;
  const int b = (int)(i % B), k = (int)(i / B);
  const float2 ri = rowinfo[b];
  float acc = 0.f;
  for (int s = 0; s < nsplit; ++s) {
    const float ms = pm[(int64_t)s * B + b];
    if (ms != NEG_INF) acc = fmaf(__builtin_amdgcn_exp2f(ms - ri.x), pO[((int64_t)s * HF + k) * B + b], acc);
  }
  const int t = __float_as_int(ri.y);
  dh[(int64_t)b * HF + k] = g * (t >= 0 ? acc - W[(int64_t)t * HF + k] : acc);
}

// ------------------------------------------------------------- pass 2 ----
// Same two-array ring and two-fold unrolled loop as pass 1.
template <int HF, int NT>
__global__ __launch_bounds__(FL_T) void k_flash_dw(const bf16x8* __restrict__ Hk, const bf16x8* __restrict__ Hr,
                                                   const bf16x8* __restrict__ Wk,
                                                   const float* __restrict__ bias_pad,
                                                   const float2* __restrict__ rowinfo, float g, int B, int A,
                                                   float* __restrict__ W, float* __restrict__ mW,
                                                   float* __restrict__ vW, float* __restrict__ bias,
                                                   float* __restrict__ mb, float* __restrict__ vb, AdamArgs args,
                                                   float* __restrict__ dW_out, float* __restrict__ db_out) {
  constexpr int NS = HF / 16, NTL = HF / 32;
  constexpr int EK = NS * 192;
  constexpr int ER = NTL * 2 * 192;
  __shared__ bf16x8 sk0[EK], sk1[EK];
  __shared__ bf16x8 sr0[ER], sr1[ER];
  __shared__ __attribute__((aligned(16))) float2 si0[32], si1[32];
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, hh = lane >> 5, l32 = lane & 31;
  const int j0 = blockIdx.x * 32 * FL_WAVES + 32 * w;
  const bool active = j0 < A;
  const int item = j0 + l32;
  const int nch = B / 32;
#define FL_ISSUE(C, SK, SR, SI)                                                  \
  do {                                                                           \
    stage<EK>(Hk + (int64_t)(C) * EK, SK, w, lane);                              \
    stage<ER>(Hr + (int64_t)(C) * ER, SR, w, lane);                              \
    if (w == 0 && lane < 16) glds16(rowinfo + 32 * (C) + 2 * lane, SI);          \
    __builtin_amdgcn_sched_barrier(0); /* keep the prefetch at the top */ \
  } while (0)
  FL_ISSUE(0, sk0, sr0, si0);
  // this wave's 32 items of W (B operand of S = h_c·Wᵀ)
  bf16x8 wk[NS][3];
#pragma unroll
  for (int s = 0; s < NS; ++s)
#pragma unroll
    for (int p = 0; p < 3; ++p)
      wk[s][p] = active ? Wk[((int64_t)(j0 >> 5) * NS + s) * 192 + p * 64 + lane] : bf16x8{};
  const float bj = active ? bias_pad[item] : NEG_INF;
  f16v dw[NTL];
#pragma unroll
  for (int t = 0; t < NTL; ++t) dw[t] = f16v{};
  float dbs = 0.f;
  __syncthreads();
  auto chunk = [&](const bf16x8* sk, const bf16x8* sr, const float2* si) __attribute__((always_inline)) {
    f16v sa = {};
#pragma unroll
    for (int s = 0; s < NS; ++s)
      sa = mfma_split<NT>(sk[s * 192 + lane], sk[s * 192 + 64 + lane], sk[s * 192 + 128 + lane], wk[s][0], wk[s][1],
                          wk[s][2], sa);
    // dZ for (row acc32_row(r, hh), item l32); db summed per chunk first
    float cdb = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f4 i0 = *reinterpret_cast<const f4*>(&si[8 * q + 4 * hh]);
      const f4 i1 = *reinterpret_cast<const f4*>(&si[8 * q + 4 * hh + 2]);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float lse2 = u < 2 ? i0[2 * u] : i1[2 * (u - 2)];
        const int tb = __float_as_int(u < 2 ? i0[2 * u + 1] : i1[2 * (u - 2) + 1]);
        const float e = __builtin_amdgcn_exp2f(fmaf(sa[4 * q + u] + bj, L2E, -lse2));
        const float p = g * (e - (tb == item ? 1.f : 0.f));
        sa[4 * q + u] = p;
        cdb += p;
      }
    }
    dbs += cdb;
    bf16x8 q0[2], q1[2], q2[2];
#pragma unroll
    for (int s = 0; s < 2; ++s)
      split3x8(f4{sa[8 * s], sa[8 * s + 1], sa[8 * s + 2], sa[8 * s + 3]},
               f4{sa[8 * s + 4], sa[8 * s + 5], sa[8 * s + 6], sa[8 * s + 7]}, q0[s], q1[s], q2[s]);
#pragma unroll
    for (int t = 0; t < NTL; ++t)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int e = (t * 2 + s) * 192 + lane;
        dw[t] = mfma_split<NT>(q0[s], q1[s], q2[s], sr[e], sr[e + 64], sr[e + 128], dw[t]);
      }
  };
  for (int c = 0; c < nch; c += 2) {
    if (c + 1 < nch) FL_ISSUE(c + 1, sk1, sr1, si1);
    if (active) chunk(sk0, sr0, si0);
    __syncthreads();
    if (c + 1 < nch) {
      if (c + 2 < nch) FL_ISSUE(c + 2, sk0, sr0, si0);
      if (active) chunk(sk1, sr1, si1);
      __syncthreads();
    }
  }
#undef FL_ISSUE
  if (!active) return;
  dbs += __shfl_xor(dbs, 32);
  if (hh == 0 && item < A) {
    if (db_out) {
      db_out[item] = dbs;
    } else {
      float p = bias[item], mq = mb[item], v = vb[item];
      adam_elem(p, mq, v, dbs, args);
      bias[item] = p;
      mb[item] = mq;
      vb[item] = v;
    }
  }
#pragma unroll
  for (int t = 0; t < NTL; ++t) {
    const int col = 32 * t + l32;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int j = j0 + acc32_row(r, hh);
      if (j >= A) continue;
      const int64_t o = (int64_t)j * HF + col;
      if (dW_out) {
        dW_out[o] = dw[t][r];
      } else {
        float p = W[o], mq = mW[o], v = vW[o];
        adam_elem(p, mq, v, dw[t][r], args);
        W[o] = p;
        mW[o] = mq;
        vW[o] = v;
      }
    }
  }
}

inline bool flash_hf_ok(int HF) { return HF == 32 || HF == 64 || HF == 128; }

}  // namespace

// ---------------------------------------------------------------- ABI ----
extern "C" int64_t rg_head_plane_bytes(int rows, int HF) {
  if (rows <= 0 || !flash_hf_ok(HF)) return RG_ERR_ARG;
  return (int64_t)((rows + 31) / 32) * 32 * HF * 6;
}

extern "C" int rg_head_planes(const float* X, int rows, int HF, void* planes_k, void* planes_r,
                              const float* bias, float* bias_pad, hipStream_t stream) {
  if (rows <= 0 || X == nullptr) return RG_ERR_ARG;
  if (!flash_hf_ok(HF)) return RG_ERR_SHAPE;
  const int rp = (rows + 31) / 32 * 32;
  const unsigned gk = (unsigned)(((int64_t)rp * (HF / 8) + 255) / 256);
  const unsigned gr = (unsigned)(((int64_t)(rp / 32) * (HF / 32) * 2 * 64 + 255) / 256);
#define PL(HFV)                                                                                                \
  if (planes_k)                                                                                                \
    hipLaunchKernelGGL(k_planes_k<HFV>, dim3(gk), dim3(256), 0, stream, X, rows, rp, (bf16x8*)planes_k);     \
  if (planes_r) hipLaunchKernelGGL(k_planes_r<HFV>, dim3(gr), dim3(256), 0, stream, X, rows, rp, (bf16x8*)planes_r)
  switch (HF) {
    case 32: PL(32); break;
    case 64: PL(64); break;
    case 128: PL(128); break;
  }
#undef PL
  if (bias && bias_pad)
    hipLaunchKernelGGL(k_pad_bias, dim3((rp + 255) / 256), dim3(256), 0, stream, bias, rows, rp, bias_pad);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_flash_fwd(const void* Hk, const void* Wk, const void* Wr, const float* bias_pad, int B, int A,
                            int HF, int terms, int nsplit, float* pm, float* pl, float* pO, hipStream_t stream) {
  if (B <= 0 || A <= 0 || (B % 32) || nsplit <= 0 || !Hk || !Wk || !Wr || !bias_pad || !pm || !pl || !pO)
    return RG_ERR_ARG;
  if (terms != 6 && terms != 9) return RG_ERR_ARG;
  if (!flash_hf_ok(HF)) return RG_ERR_SHAPE;
  const int nct = (A + 31) / 32;
  const int cps = (nct + nsplit - 1) / nsplit;
  const int nrb = (B + 32 * FL_WAVES - 1) / (32 * FL_WAVES);
  const dim3 grid((unsigned)(nrb * nsplit));
#define FF(HFV, NTV)                                                                                          \
  hipLaunchKernelGGL((k_flash_fwd<HFV, NTV>), grid, dim3(FL_T), 0, stream, (const bf16x8*)Hk, (const bf16x8*)Wk, \
                     (const bf16x8*)Wr, bias_pad, B, A, nrb, nsplit, cps, pm, pl, pO)
#define FT(HFV)          \
  if (terms == 9) {      \
    FF(HFV, 9);          \
  } else {               \
    FF(HFV, 6);          \
  }
  switch (HF) {
    case 32: FT(32); break;
    case 64: FT(64); break;
    case 128: FT(128); break;
  }
#undef FT
#undef FF
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_flash_lse(const float* pm, const float* pl, int nsplit, const float* h, const float* W,
                            const float* bias, const int64_t* tgt, int64_t lo, int A, int64_t A_full, int B, int HF,
                            float* lse, float* zt, hipStream_t stream) {
  if (B <= 0 || A <= 0 || nsplit <= 0 || !pm || !pl || !lse) return RG_ERR_ARG;
  if (zt && (!h || !W || !bias || !tgt || A_full < lo + A)) return RG_ERR_ARG;
  hipLaunchKernelGGL(k_flash_lse, dim3((B + 255) / 256), dim3(256), 0, stream, pm, pl, nsplit, h, W, bias, tgt, lo,
                     A, A_full, B, HF, lse, zt);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_flash_rows(const float* lse, const int64_t* tgt, int64_t lo, int A, int B, void* rowinfo,
                             hipStream_t stream) {
  if (B <= 0 || A <= 0 || !lse || !tgt || !rowinfo) return RG_ERR_ARG;
  hipLaunchKernelGGL(k_flash_rows, dim3((B + 255) / 256), dim3(256), 0, stream, lse, tgt, lo, A, B,
                     (float2*)rowinfo);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_flash_dh(const float* pm, const float* pO, const void* rowinfo, int nsplit, const float* W,
                           float gscale, int B, int HF, float* dh, hipStream_t stream) {
  if (B <= 0 || nsplit <= 0 || HF <= 0 || !pm || !pO || !rowinfo || !W || !dh) return RG_ERR_ARG;
  hipLaunchKernelGGL(k_flash_dh, dim3((unsigned)(((int64_t)B * HF + 255) / 256)), dim3(256), 0, stream, pm, pO,
                     (const float2*)rowinfo, nsplit, W, gscale, B, HF, dh);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_flash_dw_adam(const void* Hk, const void* Hr, const void* Wk, const float* bias_pad,
                                const void* rowinfo, float gscale, int B, int A, int HF, int terms, float* W,
                                float* mW, float* vW, float* bias, float* mb, float* vb, const float* adam6,
                                float* dW_out, float* db_out, hipStream_t stream) {
  if (B <= 0 || A <= 0 || (B % 32) || !Hk || !Hr || !Wk || !bias_pad || !rowinfo) return RG_ERR_ARG;
  if (terms != 6 && terms != 9) return RG_ERR_ARG;
  if (!flash_hf_ok(HF)) return RG_ERR_SHAPE;
  if (dW_out ? !db_out : (!adam6 || !W || !mW || !vW || !bias || !mb || !vb)) return RG_ERR_ARG;
  AdamArgs a{};
  if (adam6) a = AdamArgs{adam6[0], adam6[1], adam6[2], adam6[3], adam6[4], adam6[5]};
  const dim3 grid((unsigned)((A + 32 * FL_WAVES - 1) / (32 * FL_WAVES)));
#define FW(HFV, NTV)                                                                                          \
  hipLaunchKernelGGL((k_flash_dw<HFV, NTV>), grid, dim3(FL_T), 0, stream, (const bf16x8*)Hk, (const bf16x8*)Hr, \
                     (const bf16x8*)Wk, bias_pad, (const float2*)rowinfo, gscale, B, A, W, mW, vW, bias, mb, vb, \
                     a, dW_out, db_out)
#define FT(HFV)          \
  if (terms == 9) {      \
    FW(HFV, 9);          \
  } else {               \
    FW(HFV, 6);          \
  }
  switch (HF) {
    case 32: FT(32); break;
    case 64: FT(64); break;
    case 128: FT(128); break;
  }
#undef FT
#undef FW
  RG_LAUNCH_CHECK();
  return RG_OK;
}
