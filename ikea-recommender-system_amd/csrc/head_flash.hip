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
// MFMA shape: v_mfma_f32_16x16x32_bf16 (common.h mfma16_split: 0.84 of the
// bf16 peak in this LDS-fed split loop against 0.73 for 32x32x16).  A wave
// owns 32 rows (pass 1) / 32 items (pass 2) as two 16-wide tiles; operand
// lane l carries row / col l%16 and k group l/16 (8 values); accumulator
// register i of lane l is C[4(l/16) + i][l%16].  The k order inside a
// 32-deep slice is free as long as both operands agree, so the two 16-row
// accumulator tiles of a 32-row block (rows 4kg + i and 16 + 4kg + i of lane
// group kg, common.h kperm16) feed the next MFMA as its 32-deep operand with
// no data movement.
//
// Operand planes (16-B bf16x8 entries, one 32-row block contiguous; layout
// in common.h): K-planes (k over features) and R-planes (k over rows, in
// kperm16 order).  Both are lane-linear per wave, so chunks move global → LDS
// with 16-byte LDS-DMA (global_load_lds_dwordx4) and are read back by
// ds_read_b128.
#include "common.h"
#include "topk_scan.h"

#define NEG_INF (-__builtin_inff())

namespace {

constexpr float L2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;
// waves per workgroup: 8 (2 per SIMD) up to HF 128; at HF 256 a wave's
// operand planes (192 VGPRs) and O / dW accumulators (128) need the whole
// 512-register file, so 4 (1 per SIMD).  (Two 32-row blocks per wave at one
// wave per SIMD, halving the LDS reads per MFMA, lost at C2: pass 2 10.7 vs
// 9.7 ms, pass 1 spilled.)
constexpr int fl_nw(int HF, int) { return HF <= 128 ? 8 : 4; }
constexpr int fl_rows(int HF, int pass) { return 32 * fl_nw(HF, pass); }

// raw buffer resource over `base` (SGPRs; num_records = 2^31 - 1 bytes)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7fffffff, 0x00020000);
}

// 16-byte buffer -> LDS DMA: lane reads base + voff + soff, LDS address =
// wave-uniform base + 16·lane.  Addresses cost one VGPR (voff) per wave.
__device__ __forceinline__ void blds16(__amdgpu_buffer_rsrc_t r, void* lds_wave_base, int voff, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds_wave_base, 16, voff,
                                           soff, 0, 0);
}

// copy E 16-B entries (E % 64 == 0) from global to LDS, sliced over NW waves
// (w wave-uniform, lane16 = 16·lane), one 64-entry group per wave and step.
// P2 = false: the third plane of every [p < 3][lane] triple of groups is not
// copied (the 3-term contractions never read it); the kept groups are dealt
// to the waves evenly.  The only condition is gk < NK, and only when the
// groups do not divide evenly (per-step conditions were hoisted out of the
// chunk loop as VGPR booleans and spilled at HF 256)
template <int E, int NW, int NP = 3>
__device__ __forceinline__ void stage(const bf16x8* __restrict__ src, bf16x8* dst, int w, int lane16) {
  const __amdgpu_buffer_rsrc_t r = rsrc_of(src);
  constexpr int NGR = E / 64;                       // 64-entry groups
  constexpr int NK = NP == 3 ? NGR : NGR / 3 * NP;  // groups copied: planes 0 .. NP − 1 of each triple
  static_assert(NP == 3 || NGR % 3 == 0, "plane triples");
#pragma unroll
  for (int q = 0; q < (NK + NW - 1) / NW; ++q) {
    const int gk = NW * q + w;                       // wave-uniform
    const int g = NP == 3 ? gk : (gk / NP) * 3 + (gk % NP);
    if (NK % NW == 0 || gk < NK) blds16(r, dst + 64 * g, lane16, 1024 * g);
  }
}

// ------------------------------------------------------------- planes ----
// K- / R-planes of the 16x16x32 shape (common.h kplane16 / kperm16)
template <int HF>
__global__ __launch_bounds__(256) void k_planes_k(const float* __restrict__ X, int rows, int rows_pad,
                                                  bf16x8* __restrict__ P) {
  constexpr int G = HF / 8;
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
  const int64_t base = kplane16(x, g, HF);
  P[base] = p0;
  P[base + 64] = p1;
  P[base + 128] = p2;
}

template <int HF>
__global__ __launch_bounds__(256) void k_planes_r(const float* __restrict__ X, int rows, int rows_pad,
                                                  bf16x8* __restrict__ P) {
  constexpr int NF = HF / 16;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)(rows_pad / 32) * NF * 64) return;
  const int lane = (int)(i & 63);
  const int64_t q = i >> 6;
  const int fb = (int)(q % NF);
  const int64_t c = q / NF;
  const int kg = lane >> 4, col = 16 * fb + (lane & 15);
  f4 lo, hi;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int64_t row = 32 * c + kperm16(kg, e);
    const float v = row < rows ? X[row * HF + col] : 0.f;
    if (e < 4) lo[e] = v; else hi[e - 4] = v;
  }
  bf16x8 p0, p1, p2;
  split3x8(lo, hi, p0, p1, p2);
  const int64_t base = (c * NF + fb) * 192 + lane;
  P[base] = p0;
  P[base + 64] = p1;
  P[base + 128] = p2;
}

__global__ void k_pad_bias(const float* __restrict__ bias, int A, int Ap, float* __restrict__ out) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j < Ap) out[j] = j < A ? bias[j] : NEG_INF;
}

// ------------------------------------------------------------- pass 1 ----
// The chunk ring is SEPARATE LDS arrays per slot and the loop is unrolled by
// two: the compiler orders LDS reads only behind the DMA into the same array,
// so chunk c's MFMAs start while chunk c+1's DMA is in flight (with one [2][E]
// array it waited for the just-issued prefetch every chunk).  HF 256: the
// R-planes (48 KB per chunk) are single-buffered: chunk c+1's R DMA is issued
// after chunk c's O-MFMAs and lands under chunk c+1's S-MFMAs and softmax.
// AM (top-k outputs): 1 every chunk's row maximum (cmax) — what the fused
// top-k of SMORL's rewards reads (rg_flash_topk re-scores the candidate
// chunks); 2 also the row's top-1 (value, item) per split (rg_flash_argmax),
// whose per-logit compare-and-select is a third of the softmax section's
// VALU — only evaluation's rg_flash_score and the ABI's pbest / parg take it.
// NG = 0 (rg_flash_score, evaluation): the S-part alone — lse partials,
// per-split top-1 and chunk maxima, no O contraction, no R-planes read.
// Diagnostic build only (-DFL_STAMP, tools/flstamp.py): per-wave core cycles
// spent in pass 1's chunk barriers and in the whole wave.
#ifdef FL_STAMP
__device__ uint64_t g_fl_stamp[4096 * 2];
extern "C" int rg_fl_stamp_read(void* dst, int64_t n) {
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_fl_stamp), n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#define FL_SYNC()                                           \
  do {                                                      \
    const uint64_t _tb = __builtin_amdgcn_s_memtime();      \
    __syncthreads();                                        \
    fl_bw += __builtin_amdgcn_s_memtime() - _tb;            \
  } while (0)
#else
#define FL_SYNC() __syncthreads()
#endif

template <int HF, int NT, int NG, int AM, bool ZS = false>
__global__ __launch_bounds__(64 * fl_nw(HF, 1)) void k_flash_fwd(
    const bf16x8* __restrict__ Hk, const bf16x8* __restrict__ Wk, const bf16x8* __restrict__ Wr,
    const float* __restrict__ bias_pad, int B, int A, int nrb, int nsplit, int cps, float* __restrict__ pm,
    float* __restrict__ pl, float* __restrict__ pO, float* __restrict__ pbest, int32_t* __restrict__ parg,
    float* __restrict__ cmax, float* __restrict__ zs) {
  constexpr int NW = fl_nw(HF, 1);
  constexpr bool DR = HF <= 128;      // double-buffered R-planes
  constexpr int NS = HF / 32, NF = HF / 16;
  constexpr int EK = NS * 2 * 192;    // entries per 32-row block, K-planes
  constexpr int ER = NF * 192;        // R-planes (== EK)
  __shared__ bf16x8 sk0[EK], sk1[EK];
  __shared__ bf16x8 sr0[NG ? ER : 1], sr1[(DR && NG) ? ER : 1];
  __shared__ __attribute__((aligned(16))) float sb0[32], sb1[32];
  const int tid = threadIdx.x, lane = tid & 63, kg = lane >> 4, l16 = lane & 15, lane16 = 16 * lane;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
#ifdef FL_STAMP
  uint64_t fl_bw = 0;
  const uint64_t fl_t0 = __builtin_amdgcn_s_memtime();
#endif
  // XCD-aware order: the nrb row blocks of one item split are dispatched to
  // the same XCD (round-robin dispatch), so its W chunks are fetched once
  // into that XCD's L2 and re-read from there
  int bid = blockIdx.x;
  const int total = nrb * nsplit;
  if ((total & 7) == 0) bid = (bid & 7) * (total >> 3) + (bid >> 3);
  const int split = bid / nrb, rblk = bid % nrb;
  const int r0 = rblk * fl_rows(HF, 1) + 32 * w;   // this wave's first row
  const bool active = r0 < B;
  const int nct = (A + 31) / 32;
  const int c0 = split * cps;
  // stored logits z = S + b (zs != NULL; pass 2 reads them instead of
  // recomputing S): one 1024-float tile per (32-item chunk, 32-row block),
  // chunk-major; inside, the 16×16 quadrant (ib, rb), then this kernel's
  // accumulator order, lane-linear: each lane stores its four logits of a
  // quadrant as one 16-B store (whole 1 KB per instruction; pass 2 transposes
  // through LDS).  Launched by rg_flash_fwd_top only for B a multiple of the
  // row block (256 rows; 128 at HF 256), so every wave is active and its four
  // stores per chunk are unconditional — the compiler then counts them
  // exactly against the barrier's vmcnt(4).  HF 256 (ZSI): the wave's 512
  // registers are full, so z leaves straight from the S accumulators inside
  // the softmax section (no held copy), and the single-R-buffer loop's two
  // barriers per chunk wait vmcnt(4) (the ring's DMA, not the z stores) and
  // LDS only
  static_assert(!ZS || NG > 0, "stored logits: training pass");
  constexpr bool ZSI = ZS && HF > 128;
  // lane (kg, l16) stores its f4 at slot 16kg + 4(l16 >> 2) + ((l16 & 3) ^ kg) of
  // the quadrant (a bijection: still 1 KB contiguous per instruction), so that
  // pass 2, which DMAs the tile into LDS unchanged, reads it back transposed
  // with conflict-free 4-B reads (zs_slot, k_flash_dw)
  float* __restrict__ zrow =
      ZS ? zs + (int64_t)(r0 >> 5) * 1024 + 4 * (16 * kg + 4 * (l16 >> 2) + ((l16 & 3) ^ kg)) : nullptr;
  const int nch = max(0, min(nct, c0 + cps) - c0);
#define FL_ISSUE_K(C, SK, SB)                                                  \
  do {                                                                         \
    stage<EK, NW>(Wk + (int64_t)(C) * EK, SK, w, lane16);                      \
    if (w == 0 && lane < 8) blds16(rsrc_of(bias_pad + 32 * (C)), SB, lane16, 0); \
  } while (0)
#define FL_ISSUE_R(C, SR)                                                                \
  do {                                                                                   \
    if constexpr (NG > 0) stage<ER, NW, NG == 3 ? 2 : 3>(Wr + (int64_t)(C) * ER, SR, w, lane16); \
  } while (0)
  if (nch > 0) {
    FL_ISSUE_K(c0, sk0, sb0);
    FL_ISSUE_R(c0, sr0);
  }
  // this wave's 32 rows of h as two 16-row B operands (Sᵀ = W_c·hᵀ), for the whole split
  bf16x8 hk[NS][2][3];
#pragma unroll
  for (int s = 0; s < NS; ++s)
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int p = 0; p < 3; ++p)
        hk[s][rb][p] = active ? Hk[(((int64_t)(r0 >> 5) * NS + s) * 2 + rb) * 192 + p * 64 + lane] : bf16x8{};
  // Oᵀ tiles (feature block fb, row block rb): lane (kg, n) holds features
  // 16fb + 4kg + i of row 16rb + n; m / l / best per row block: row 16rb + l16
  f4 o[NF][2];
  float m[2], l[2], bv[2];
  int bi[2];
#pragma unroll
  for (int rb = 0; rb < 2; ++rb) {
#pragma unroll
    for (int fb = 0; fb < NF; ++fb) o[fb][rb] = f4{0.f, 0.f, 0.f, 0.f};
    m[rb] = NEG_INF;
    l[rb] = 0.f;
    bv[rb] = NEG_INF;
    bi[rb] = INT32_MAX;
  }
  __syncthreads();
  // S-part of chunk c: Sᵀ tiles (item block ib, row block rb), (ARG) top-1 /
  // chunk max, online max / Σexp, P planes (q*[rb]: the B operand of the O-part)
  // ZS: the chunk's z tiles leave after its O-part MFMAs are issued (stores
  // in the softmax section, between the two MFMA phases, measured 0.15 ms slower)
  f4 zsv[ZS && HF <= 128 ? 2 : 1][2];
  auto zflush = [&](int c) __attribute__((always_inline)) {
#pragma unroll
    for (int ib = 0; ib < 2; ++ib)
#pragma unroll
      for (int rb = 0; rb < 2; ++rb)
        __builtin_nontemporal_store(zsv[ib][rb], reinterpret_cast<f4*>(zrow + (int64_t)(c0 + c) * (B / 32) * 1024 +
                                                                       (2 * ib + rb) * 256));
  };
  auto spart = [&](const bf16x8* sk, const float* sb, int c, bf16x8 (&q0)[2], bf16x8 (&q1)[2], bf16x8 (&q2)[2])
                   __attribute__((always_inline)) {
    f4 sa[2][2];
#pragma unroll
    for (int ib = 0; ib < 2; ++ib)
#pragma unroll
      for (int rb = 0; rb < 2; ++rb) sa[ib][rb] = f4{0.f, 0.f, 0.f, 0.f};
    // W fragments software-pipelined one (slice, item block) ahead; the sched
    // barriers stop the scheduler from hoisting every step's LDS reads
    bf16x8 a0 = sk[lane], a1 = sk[64 + lane], a2 = sk[128 + lane];
#pragma unroll
    for (int t = 0; t < 2 * NS; ++t) {
      const int s = t >> 1, ib = t & 1;
      const int en = (t + 1 < 2 * NS ? t + 1 : t) * 192 + lane;
      const bf16x8 n0 = sk[en], n1 = sk[en + 64], n2 = sk[en + 128];
#pragma unroll
      for (int rb = 0; rb < 2; ++rb)
        sa[ib][rb] = mfma16_split<NT>(a0, a1, a2, hk[s][rb][0], hk[s][rb][1], hk[s][rb][2], sa[ib][rb]);
      a0 = n0;
      a1 = n1;
      a2 = n2;
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
      // logits (items 16ib + 4kg + u of the chunk, row 16rb + l16)
      float cm = NEG_INF;
#pragma unroll
      for (int ib = 0; ib < 2; ++ib) {
        const f4 bq = *reinterpret_cast<const f4*>(&sb[16 * ib + 4 * kg]);
        if constexpr (ZS && !ZSI) zsv[ib][rb] = sa[ib][rb] + bq;   // stored after the O-part (zflush)
        if constexpr (ZSI)
          __builtin_nontemporal_store(sa[ib][rb] + bq, reinterpret_cast<f4*>(zrow + (int64_t)(c0 + c) * (B / 32) * 1024 +
                                                                             (2 * ib + rb) * 256));
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const float z = sa[ib][rb][u] + bq[u];
          if (AM == 2 && z > bv[rb]) {  // items increase with (ib, u): strict > keeps the first maximum
            bv[rb] = z;
            bi[rb] = 32 * (c0 + c) + 16 * ib + 4 * kg + u;
          }
          sa[ib][rb][u] = z * L2E;
          cm = fmaxf(cm, z);
        }
      }
      cm = fmaxf(cm, __shfl_xor(cm, 16));
      cm = fmaxf(cm, __shfl_xor(cm, 32));
      if (AM >= 1 && cmax != nullptr && kg == 0) cmax[(int64_t)(c0 + c) * B + r0 + 16 * rb + l16] = cm;
      cm *= L2E;
      const float mn = fmaxf(m[rb], cm);
      if (__any(mn > m[rb])) {
        const float a = mn > m[rb] ? __builtin_amdgcn_exp2f(m[rb] - mn) : 1.f;
#pragma unroll
        for (int fb = 0; fb < NF; ++fb) o[fb][rb] *= a;
        l[rb] *= a;
        m[rb] = mn;
      }
      const float mm = m[rb] == NEG_INF ? 0.f : m[rb];
      float ps = 0.f;
#pragma unroll
      for (int ib = 0; ib < 2; ++ib)
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const float p = __builtin_amdgcn_exp2f(sa[ib][rb][u] - mm);
          sa[ib][rb][u] = p;
          ps += p;
        }
      l[rb] += ps;
      // k slots of the O-part: items kperm16(kg, e)
      split3x8(sa[0][rb], sa[1][rb], q0[rb], q1[rb], q2[rb]);
    }
  };
  // O-part: Oᵀ += W_cᵀ·Pᵀ, one R-plane fragment per feature block
  auto opart = [&](const bf16x8* sr, const bf16x8 (&q0)[2], const bf16x8 (&q1)[2], const bf16x8 (&q2)[2])
                   __attribute__((always_inline)) {
    if constexpr (NG > 0) {
      bf16x8 a0 = sr[lane], a1 = sr[64 + lane], a2 = sr[128 + lane];
#pragma unroll
      for (int fb = 0; fb < NF; ++fb) {
        const int en = (fb + 1 < NF ? fb + 1 : fb) * 192 + lane;
        const bf16x8 n0 = sr[en], n1 = sr[en + 64], n2 = NG == 3 ? n0 : sr[en + 128];
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) o[fb][rb] = mfma16_split<NG>(a0, a1, a2, q0[rb], q1[rb], q2[rb], o[fb][rb]);
        a0 = n0;
        a1 = n1;
        a2 = n2;
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };
  // chunk barrier; a wave storing logits waits for the ring's DMA only
  // (issued before the chunk's four z stores: vmcnt(4)), not for its stores'
  // write acknowledgements (a full vmcnt(0) here cost pass 1 ~0.7 µs per chunk)
  auto csync = [&]() __attribute__((always_inline)) {
    if constexpr (ZS) {
      __builtin_amdgcn_s_waitcnt((4 & 15) | 0x70);   // vmcnt(4) lgkmcnt(0)
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    } else {
      FL_SYNC();
    }
  };
  for (int c = 0; c < nch; c += 2) {
    bf16x8 q0[2], q1[2], q2[2];
    if (DR || NG == 0) {
      if (c + 1 < nch) {
        FL_ISSUE_K(c0 + c + 1, sk1, sb1);
        FL_ISSUE_R(c0 + c + 1, sr1);
      }
      __builtin_amdgcn_sched_barrier(0);   // keep the prefetch at the top
      if (ZS || active) {
        spart(sk0, sb0, c, q0, q1, q2);
        opart(sr0, q0, q1, q2);
        if constexpr (ZS && !ZSI) zflush(c);
      }
      csync();
      if (c + 1 < nch) {
        if (c + 2 < nch) {
          FL_ISSUE_K(c0 + c + 2, sk0, sb0);
          FL_ISSUE_R(c0 + c + 2, sr0);
        }
        __builtin_amdgcn_sched_barrier(0);
        if (ZS || active) {
          spart(sk1, sb1, c + 1, q0, q1, q2);
          opart(sr1, q0, q1, q2);
          if constexpr (ZS && !ZSI) zflush(c + 1);
        }
        csync();
      }
    } else {
      // single R buffer: R(c) was issued after the previous chunk's O-part.
      // ZSI: the first barrier waits for the ring's DMA (older than the
      // chunk's z stores: vmcnt(4)), the second for LDS reads only
      auto sync_dma = [&]() __attribute__((always_inline)) {
        if constexpr (ZSI) {
          __builtin_amdgcn_s_waitcnt((4 & 15) | 0x70);   // vmcnt(4) lgkmcnt(0)
          __builtin_amdgcn_s_barrier();
          __builtin_amdgcn_sched_barrier(0);
        } else {
          __syncthreads();
        }
      };
      auto sync_lds = [&]() __attribute__((always_inline)) {
        if constexpr (ZSI) {
          __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0), vmcnt / expcnt free
          __builtin_amdgcn_s_barrier();
          __builtin_amdgcn_sched_barrier(0);
        } else {
          __syncthreads();
        }
      };
      if (c + 1 < nch) FL_ISSUE_K(c0 + c + 1, sk1, sb1);
      __builtin_amdgcn_sched_barrier(0);
      if (ZS || active) spart(sk0, sb0, c, q0, q1, q2);
      sync_dma();   // R(c) and K(c+1) landed for every wave
      if (ZS || active) opart(sr0, q0, q1, q2);
      sync_lds();   // every wave is done with sr0 and sk0
      if (c + 1 < nch) {
        FL_ISSUE_R(c0 + c + 1, sr0);
        if (c + 2 < nch) FL_ISSUE_K(c0 + c + 2, sk0, sb0);
        __builtin_amdgcn_sched_barrier(0);
        if (ZS || active) spart(sk1, sb1, c + 1, q0, q1, q2);
        sync_dma();
        if (ZS || active) opart(sr0, q0, q1, q2);
        sync_lds();
        if (c + 2 < nch) FL_ISSUE_R(c0 + c + 2, sr0);
      }
    }
  }
#undef FL_ISSUE_K
#undef FL_ISSUE_R
#ifdef FL_STAMP
  if (lane == 0 && blockIdx.x < 512) {
    g_fl_stamp[(blockIdx.x * NW + w) * 2] = fl_bw;
    g_fl_stamp[(blockIdx.x * NW + w) * 2 + 1] = __builtin_amdgcn_s_memtime() - fl_t0;
  }
#endif
  if (!active) return;
#pragma unroll
  for (int rb = 0; rb < 2; ++rb) {
    float lt = l[rb] + __shfl_xor(l[rb], 16);
    lt += __shfl_xor(lt, 32);
    const int row = r0 + 16 * rb + l16;
    float bvj = bv[rb];
    int bij = bi[rb];
    if (AM == 2) {  // merge the four lane groups: larger value, ties to the smaller item
#pragma unroll
      for (int d = 16; d <= 32; d *= 2) {
        const float v2 = __shfl_xor(bvj, d);
        const int i2 = __shfl_xor(bij, d);
        if (v2 > bvj || (v2 == bvj && i2 < bij)) {
          bvj = v2;
          bij = i2;
        }
      }
    }
    if (kg == 0) {
      pm[(int64_t)split * B + row] = m[rb];
      pl[(int64_t)split * B + row] = lt;
      if (AM == 2) {
        pbest[(int64_t)split * B + row] = bvj;
        parg[(int64_t)split * B + row] = bij;
      }
    }
    if constexpr (NG > 0) {
#pragma unroll
      for (int fb = 0; fb < NF; ++fb)
#pragma unroll
        for (int i = 0; i < 4; ++i) pO[((int64_t)split * HF + 16 * fb + 4 * kg + i) * B + row] = o[fb][rb][i];
    }
  }
}

// --------------------------------------------------------- argmax only ----
// argmax_j (h·Wᵀ + b)[row, j] on split-bf16 MFMAs without storing logits: the
// S-part of pass 1 alone (no softmax, no O) with the first-maximum tracking —
// the double-Q target a* = argmax_a Q(s', a) of SQN / SMORL (sqn_gru.py:
// 222-226, tensor_operations.py:50-70 via the combined head).  Same
// workgroup / split / XCD layout and K-plane DMA ring as pass 1; per split the
// row's best logit and item go to pbest / parg (merged by rg_flash_argmax).
// CM (screening, NT = 3 or 1): also every 32-item chunk's row maximum (cmax,
// ceil(A/32) × B) for the exact re-scoring of rg_flash_argmax_exact; the
// operand planes past the ones it multiplies (2, or 1 and 2) are never read
// (not even DMA'd).
template <int HF, int NT, bool CM>
__global__ __launch_bounds__(64 * fl_nw(HF, 1)) void k_flash_amax(
    const bf16x8* __restrict__ Hk, const bf16x8* __restrict__ Wk, const float* __restrict__ bias_pad, int B, int A,
    int nrb, int nsplit, int cps, float* __restrict__ pbest, int32_t* __restrict__ parg, float* __restrict__ cmax) {
  constexpr int NW = fl_nw(HF, 1);
  constexpr int NS = HF / 32;
  constexpr int EK = NS * 2 * 192;
  // chunks per LDS slot: NT = 1 multiplies plane 0 only, so a slot's plane-1
  // and plane-2 positions hold the next two chunks' plane 0 — three chunks
  // between barriers (the 1-product loop is otherwise barrier- and
  // DMA-latency-bound: 16 MFMAs per wave and chunk)
  constexpr int PG = NT == 1 ? 3 : 1;
  __shared__ bf16x8 sk0[EK], sk1[EK];
  __shared__ __attribute__((aligned(16))) float sb0[32 * PG], sb1[32 * PG];
  const int tid = threadIdx.x, lane = tid & 63, kg = lane >> 4, l16 = lane & 15, lane16 = 16 * lane;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  int bid = blockIdx.x;
  const int total = nrb * nsplit;
  if ((total & 7) == 0) bid = (bid & 7) * (total >> 3) + (bid >> 3);
  const int split = bid / nrb, rblk = bid % nrb;
  const int r0 = rblk * 32 * NW + 32 * w;
  const bool active = r0 < B;
  const int nct = (A + 31) / 32;
  const int c0 = split * cps;
  const int nch = max(0, min(nct, c0 + cps) - c0);
  // chunks CR .. CR + PG − 1 (relative) into one slot
#define FA_ISSUE(CR, SK, SB)                                                                       \
  do {                                                                                             \
    _Pragma("unroll") for (int q_ = 0; q_ < PG; ++q_) {                                            \
      if ((CR) + q_ < nch) {                                                                       \
        stage<EK, NW, NT == 1 ? 1 : NT == 3 ? 2 : 3>(Wk + (int64_t)(c0 + (CR) + q_) * EK, (SK) + 64 * q_, w, \
                                                     lane16);                                      \
        if (w == 0 && lane < 8) blds16(rsrc_of(bias_pad + 32 * (c0 + (CR) + q_)), (SB) + 32 * q_, lane16, 0); \
      }                                                                                            \
    }                                                                                              \
  } while (0)
  if (nch > 0) FA_ISSUE(0, sk0, sb0);
  bf16x8 hk[NS][2][3];
#pragma unroll
  for (int s = 0; s < NS; ++s)
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int p = 0; p < 3; ++p)
        hk[s][rb][p] = active && p < (NT == 1 ? 1 : NT == 3 ? 2 : 3)
                           ? Hk[(((int64_t)(r0 >> 5) * NS + s) * 2 + rb) * 192 + p * 64 + lane]
                           : bf16x8{};
  float bv[2] = {NEG_INF, NEG_INF};
  int bi[2] = {INT32_MAX, INT32_MAX};
  __syncthreads();
  auto chunk = [&](const bf16x8* sk, const float* sb, int c) __attribute__((always_inline)) {
    f4 sa[2][2];
#pragma unroll
    for (int ib = 0; ib < 2; ++ib)
#pragma unroll
      for (int rb = 0; rb < 2; ++rb) sa[ib][rb] = f4{0.f, 0.f, 0.f, 0.f};
    bf16x8 a0 = sk[lane], a1 = NT == 1 ? a0 : sk[64 + lane], a2 = NT <= 3 ? a0 : sk[128 + lane];
#pragma unroll
    for (int t = 0; t < 2 * NS; ++t) {
      const int s = t >> 1, ib = t & 1;
      const int en = (t + 1 < 2 * NS ? t + 1 : t) * 192 + lane;
      const bf16x8 n0 = sk[en], n1 = NT == 1 ? n0 : sk[en + 64], n2 = NT <= 3 ? n0 : sk[en + 128];
#pragma unroll
      for (int rb = 0; rb < 2; ++rb)
        sa[ib][rb] = mfma16_split<NT>(a0, a1, a2, hk[s][rb][0], hk[s][rb][1], hk[s][rb][2], sa[ib][rb]);
      a0 = n0;
      a1 = n1;
      a2 = n2;
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
      float cm = NEG_INF;
#pragma unroll
      for (int ib = 0; ib < 2; ++ib) {
        const f4 bq = *reinterpret_cast<const f4*>(&sb[16 * ib + 4 * kg]);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const float z = sa[ib][rb][u] + bq[u];
          cm = fmaxf(cm, z);
          if (z > bv[rb]) {  // items increase with (ib, u): strict > keeps the first maximum
            bv[rb] = z;
            bi[rb] = 32 * (c0 + c) + 16 * ib + 4 * kg + u;
          }
        }
      }
      if (CM) {
        cm = fmaxf(cm, __shfl_xor(cm, 16));
        cm = fmaxf(cm, __shfl_xor(cm, 32));
        if (kg == 0) cmax[(int64_t)(c0 + c) * B + r0 + 16 * rb + l16] = cm;
      }
    }
  };
  auto group = [&](const bf16x8* sk, const float* sb, int c) __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < PG; ++q)
      if (c + q < nch) chunk(sk + 64 * q, sb + 32 * q, c + q);
  };
  for (int c = 0; c < nch; c += 2 * PG) {
    if (c + PG < nch) FA_ISSUE(c + PG, sk1, sb1);
    __builtin_amdgcn_sched_barrier(0);
    if (active) group(sk0, sb0, c);
    __syncthreads();
    if (c + PG < nch) {
      if (c + 2 * PG < nch) FA_ISSUE(c + 2 * PG, sk0, sb0);
      __builtin_amdgcn_sched_barrier(0);
      if (active) group(sk1, sb1, c + PG);
      __syncthreads();
    }
  }
#undef FA_ISSUE
  if (!active) return;
#pragma unroll
  for (int rb = 0; rb < 2; ++rb) {
    float bvj = bv[rb];
    int bij = bi[rb];
#pragma unroll
    for (int d = 16; d <= 32; d *= 2) {
      const float v2 = __shfl_xor(bvj, d);
      const int i2 = __shfl_xor(bij, d);
      if (v2 > bvj || (v2 == bvj && i2 < bij)) {
        bvj = v2;
        bij = i2;
      }
    }
    if (kg == 0) {
      pbest[(int64_t)split * B + r0 + 16 * rb + l16] = bvj;
      parg[(int64_t)split * B + r0 + 16 * rb + l16] = bij;
    }
  }
}

// ------------------------------------------------------------ combine ----
// lse over the splits (natural units) and, when the target is one of this
// shard's items [lo, lo + A), its logit z = h·W[t] + b[t]; 0 for a target
// held by another shard, NaN for one outside [0, A_full) (CrossEntropyLoss
// raises there; the native head writes a NaN loss row, head.hip k_lse_combine)
// (HF a template parameter: the row's h and W[t] arrive as 16-B loads issued
// up front; the dot is the same sequential fmaf chain over k; 64-row blocks)
template <int HF>
__global__ __launch_bounds__(64) void k_flash_lse(const float* __restrict__ pm, const float* __restrict__ pl,
                                                  int nsplit, const float* __restrict__ h,
                                                  const float* __restrict__ W, const float* __restrict__ bias,
                                                  const int64_t* __restrict__ tgt, int64_t lo, int A, int64_t A_full,
                                                  int B, float* __restrict__ lse, float* __restrict__ zt) {
  const int b = blockIdx.x * 64 + threadIdx.x;
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
      const f4* hr = reinterpret_cast<const f4*>(h + (int64_t)b * HF);
      const f4* wr = reinterpret_cast<const f4*>(W + t * HF);
      f4 hv[HF / 4], wv[HF / 4];
#pragma unroll
      for (int k = 0; k < HF / 4; ++k) {
        hv[k] = hr[k];
        wv[k] = wr[k];
      }
#pragma unroll
      for (int k = 0; k < HF / 4; ++k)
#pragma unroll
        for (int u = 0; u < 4; ++u) z = fmaf(hv[k][u], wv[k][u], z);
      z += bias[t];
    }
    zt[b] = z;
  }
}

// Row records, what pass 2 stages through LDS (256 B per 32-row chunk): per
// chunk the 32 rows' lse·log2e, then their local targets (or −1) — split, so
// pass 2 reads four consecutive rows' values of one kind as a vector and
// works on them in packed pairs
__device__ __forceinline__ int ri_lse(int b) { return 64 * (b >> 5) + (b & 31); }
__device__ __forceinline__ int ri_tgt(int b) { return 64 * (b >> 5) + 32 + (b & 31); }

__global__ void k_flash_rows(const float* __restrict__ lse, const int64_t* __restrict__ tgt, int64_t lo, int A, int B,
                             float* __restrict__ rowinfo) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const int64_t t = tgt[b] - lo;
  rowinfo[ri_lse(b)] = lse[b] * L2E;
  rowinfo[ri_tgt(b)] = __int_as_float(t >= 0 && t < A ? (int)t : -1);
}

// dh[b][k] = g·(Σ_s 2^(m_s − lse2_b)·O_s[k][b] − W[t_b][k])
__global__ __launch_bounds__(256) void k_flash_dh(const float* __restrict__ pm, const float* __restrict__ pO,
                                                  const float* __restrict__ rowinfo, int nsplit,
                                                  const float* __restrict__ W, float g, int B, int HF,
                                                  float* __restrict__ dh) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)B * HF) return;
  const int b = (int)(i % B), k = (int)(i / B);
  const float lse2 = rowinfo[ri_lse(b)];
  float acc = 0.f;
  for (int s = 0; s < nsplit; ++s) {
    const float ms = pm[(int64_t)s * B + b];
    if (ms != NEG_INF) acc = fmaf(__builtin_amdgcn_exp2f(ms - lse2), pO[((int64_t)s * HF + k) * B + b], acc);
  }
  const int t = __float_as_int(rowinfo[ri_tgt(b)]);
  dh[(int64_t)b * HF + k] = g * (t >= 0 ? acc - W[(int64_t)t * HF + k] : acc);
}

// ------------------------------------------------------------- pass 2 ----
// Same ring scheme as pass 1 (HF 256: single-buffered R-planes of h); a wave
// owns 32 items (two 16-item tiles).
//
// Tail: the item blocks past the last whole round of workgroups (nfull
// blocks) are split over tsplit workgroups each, every one taking a
// contiguous range of the row chunks; they write partial dW / db (tail_dw:
// tsplit × ntail × HF, tail_db: tsplit × ntail, ntail = A − 256·nfull) and
// k_flash_tail sums them in order and finishes (Adam, planes).  At C2 the
// 67 leftover blocks of 3907 would otherwise run as a 16th round on 26% of
// the CUs.
// Diagnostic build only (-DFL2_STAMP, tools/fl2stamp.py): per-wave phase
// cycles of pass 2 — prologue, S-part MFMA issue, dZ VALU, W-part MFMA issue,
// chunk barriers, epilogue — plus the wave's start / end (s_memrealtime).
#ifdef FL2_STAMP
constexpr int FL2_MAXB = 4608, FL2_F = 8;
__device__ uint64_t g_fl2_stamp[FL2_MAXB * 8 * FL2_F];
extern "C" int rg_fl2_stamp_read(void* dst, int64_t n) {
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_fl2_stamp), n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#define FL2_DECL uint64_t f2_acc[6] = {0, 0, 0, 0, 0, 0}; uint64_t f2_t = __builtin_amdgcn_s_memtime(); \
  const uint64_t f2_r0 = __builtin_amdgcn_s_memrealtime();
#define FL2_MARK(k)                                    \
  do {                                                 \
    const uint64_t _n = __builtin_amdgcn_s_memtime();  \
    f2_acc[k] += _n - f2_t;                            \
    f2_t = _n;                                         \
  } while (0)
#define FL2_SYNC()   \
  do {               \
    FL2_MARK(3);     \
    __syncthreads(); \
    FL2_MARK(4);     \
  } while (0)
#define FL2_STORE()                                                                          \
  do {                                                                                       \
    if (lane == 0 && blockIdx.x < FL2_MAXB) {                                                \
      uint64_t* _d = g_fl2_stamp + ((int64_t)blockIdx.x * 8 + w) * FL2_F;                    \
      _d[0] = f2_r0;                                                                         \
      _d[1] = __builtin_amdgcn_s_memrealtime();                                              \
      for (int _k = 0; _k < 6; ++_k) _d[2 + _k] = f2_acc[_k];                                \
    }                                                                                        \
  } while (0)
#else
#define FL2_DECL
#define FL2_MARK(k)
#define FL2_SYNC() __syncthreads()
#define FL2_STORE()
#endif
// phases: 0 prologue, 1 S-part MFMA issue, 2 dZ VALU + split, 3 W-part MFMA
// issue, 4 barrier wait, 5 epilogue (db / Adam / planes, or the tail partials)

// s_waitcnt immediate: vmcnt <= n (6 bits, split), expcnt free, lgkmcnt 0
constexpr int sf2_wc_vm(int n) { return (n & 15) | ((n >> 4) << 14) | 0x70; }

// ZL: the logits z = S + b come from pass 1's store (zs, k_flash_fwd) instead
// of the S-part: no K-planes of h or W are read, the chunk is dZ VALU + the
// W-part only, and h's R-planes run through a two-slot ring in the (then idle)
// K-plane arrays at every HF.  Each wave's z tile (16 floats per lane, pass
// 1's lane order) is loaded into registers two chunks ahead — the chunk
// barriers wait for the ring's DMA only (vmcnt), not for the newest z loads —
// and turned into this kernel's accumulator order through 1 KB of LDS per wave
// (a 16×16 transpose per quadrant: four conflict-free 4-B writes, one 16-B read).
template <int HF, int NT, bool ZL>
__global__ __launch_bounds__(64 * fl_nw(HF, 2)) void k_flash_dw(
    const bf16x8* __restrict__ Hk0, const bf16x8* __restrict__ Hr0, const bf16x8* Wk, const float* bias_pad,
    const float* __restrict__ rowinfo0, float g, int B, int A, float* __restrict__ W, float* __restrict__ mW,
    float* __restrict__ vW, float* __restrict__ bias, float* __restrict__ mb, float* __restrict__ vb, AdamArgs args,
    float* __restrict__ dW_out, float* __restrict__ db_out, bf16x8* Wk_out, bf16x8* Wr_out, float* bias_pad_out,
    int nfull, int tsplit, float* __restrict__ tail_dw, float* __restrict__ tail_db, const float* __restrict__ zs) {
  constexpr int NW = fl_nw(HF, 2);
  constexpr bool DR = HF <= 128;
  constexpr int NS = HF / 32, NF = HF / 16;
  constexpr int EK = NS * 2 * 192;
  constexpr int ER = NF * 192;
  __shared__ bf16x8 sk0[EK], sk1[EK];
  __shared__ bf16x8 sr0[ZL ? 1 : ER], sr1[(DR && !ZL) ? ER : 1];   // (ZL: h's R-planes ring in sk0 / sk1)
  __shared__ __attribute__((aligned(16))) float si0[64], si1[64];   // row records of a chunk
  // ZL: three-slot ring of the waves' z tiles (4 KB per wave and slot, DMA'd
  // straight from pass 1's store; separate arrays, so the compiler's LDS-DMA
  // tracking orders reads of a slot behind its own DMA only)
  __shared__ __attribute__((aligned(16))) float zr0[ZL ? 1024 * NW : 1], zr1[ZL ? 1024 * NW : 1],
      zr2[ZL ? 1024 * NW : 1];
  __shared__ __attribute__((aligned(16))) float si2[ZL ? 64 : 1];   // ZL: third row-record slot
  const int tid = threadIdx.x, lane = tid & 63, kg = lane >> 4, l16 = lane & 15, lane16 = 16 * lane;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  FL2_DECL
  const int bx = blockIdx.x;
  const bool tail = bx >= nfull;
  const int blk = tail ? nfull + (bx - nfull) / tsplit : bx;
  const int j0 = blk * fl_rows(HF, 2) + 32 * w;   // this wave's first item
  const bool active = j0 < A;
  const int nct = B / 32, cper = (nct + tsplit - 1) / tsplit;
  const int cb = tail ? (bx - nfull) % tsplit * cper : 0;
  const int nch = tail ? max(0, min(nct, cb + cper) - cb) : nct;
  const bf16x8* __restrict__ Hk = Hk0 + (int64_t)cb * EK;
  const bf16x8* __restrict__ Hr = Hr0 + (int64_t)cb * ER;
  const float* __restrict__ rowinfo = rowinfo0 + 64 * cb;
#define FL_ISSUE_K(C, SK, SI)                                                  \
  do {                                                                         \
    stage<EK, NW>(Hk + (int64_t)(C) * EK, SK, w, lane16);                      \
    if (w == 0 && lane < 16) blds16(rsrc_of(rowinfo + 64 * (C)), SI, lane16, 0); \
  } while (0)
#define FL_ISSUE_R(C, SR) stage<ER, NW>(Hr + (int64_t)(C) * ER, SR, w, lane16)
  // ZL: chunk C's R-planes into ring slot SR (a K-plane array: EK == ER) and its row records
#define FL_ISSUE_Z(C, SR, SI)                                                  \
  do {                                                                         \
    stage<ER, NW>(Hr + (int64_t)(C) * ER, SR, w, lane16);                      \
    if (w == 0 && lane < 16) blds16(rsrc_of(rowinfo + 64 * (C)), SI, lane16, 0); \
  } while (0)
  // a part with no row chunks (nch == 0) reads nothing: every DMA below and in
  // the loops indexes chunks 0 .. nch − 1 only
  if (nch > 0) {
    if constexpr (ZL) {
      FL_ISSUE_Z(0, sk0, si0);
      if (w == 0 && lane < 16) blds16(rsrc_of(rowinfo + 64 * min(1, nch - 1)), si1, lane16, 0);
    } else {
      FL_ISSUE_K(0, sk0, si0);
      FL_ISSUE_R(0, sr0);
    }
  }
  // this wave's 32 items of W as two 16-item B operands of S = h_c·Wᵀ
  bf16x8 wk[NS][2][3];
  float bj[2];
#pragma unroll
  for (int ib = 0; ib < 2; ++ib) {
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
      for (int p = 0; p < 3; ++p)
        wk[s][ib][p] = (active && !ZL) ? Wk[(((int64_t)(j0 >> 5) * NS + s) * 2 + ib) * 192 + p * 64 + lane]
                                       : bf16x8{};
    bj[ib] = ZL ? 0.f : active ? bias_pad[j0 + 16 * ib + l16] : NEG_INF;
  }
  // dW tiles (item block ib, feature block fb): lane (kg, n) holds items
  // 16ib + 4kg + i, feature 16fb + n; db per item block: this lane's item 16ib + l16
  f4 dw[2][NF];
  float dbs[2] = {0.f, 0.f};
#pragma unroll
  for (int ib = 0; ib < 2; ++ib)
#pragma unroll
    for (int fb = 0; fb < NF; ++fb) dw[ib][fb] = f4{0.f, 0.f, 0.f, 0.f};
  // ZL: this wave's z tiles (item block j0 / 32, row chunks from cb), DMA'd
  // 1 KB per quadrant into the wave's 4 KB of a ring slot (branch-free: a
  // wave past A reads item block 0's tiles, a chunk index past the range
  // re-reads the last chunk — neither result is used — so every step issues
  // the same four DMA ops)
  const float* __restrict__ zt = ZL ? zs + ((int64_t)(active ? j0 >> 5 : 0) * (B / 32) + cb) * 1024 : nullptr;
  auto zdma = [&](int c, float* slot) __attribute__((always_inline)) {
    const __amdgpu_buffer_rsrc_t r = rsrc_of(zt + (int64_t)min(c, nch - 1) * 1024);
#pragma unroll
    for (int q = 0; q < 4; ++q) blds16(r, slot + 1024 * w + 256 * q, lane16, 1024 * q);
  };
  if constexpr (ZL) {
    if (nch > 0) {
      zdma(0, zr0);
      zdma(1, zr1);
      zdma(2, zr2);
    }
  }
  __syncthreads();
  FL2_MARK(0);
  // dZ = g·(2^((S + b)·log2e − lse·log2e) − onehot) from the chunk's S tiles
  // (ZL: z = S + b, bj = 0), db; dZᵀ planes (q*[ib]: the A operand of dW, k
  // over the chunk's rows in kperm16 order).  Scalar fp32 only: packed f32
  // ops (v_pk_*) cost more issue beside the MFMAs than two scalar ones
  auto dzpart = [&](f4 (&sa)[2][2], const float* si, bf16x8 (&q0)[2], bf16x8 (&q1)[2], bf16x8 (&q2)[2],
                    bool add_db = true) __attribute__((always_inline)) {
#pragma unroll
    for (int ib = 0; ib < 2; ++ib) {
      const int item = j0 + 16 * ib + l16;
      float cdb = 0.f;
#pragma unroll
      for (int rb = 0; rb < 2; ++rb) {
        const f4 ls = *reinterpret_cast<const f4*>(&si[16 * rb + 4 * kg]);
        const f4 tb = *reinterpret_cast<const f4*>(&si[32 + 16 * rb + 4 * kg]);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const float zz = ZL ? sa[rb][ib][u] : sa[rb][ib][u] + bj[ib];
          const float e = __builtin_amdgcn_exp2f(fmaf(zz, L2E, -ls[u]));
          const float p = fmaf(g, e, __float_as_int(tb[u]) == item ? -g : 0.f);   // g·(e − onehot)
          sa[rb][ib][u] = p;
          cdb += p;
        }
      }
      dbs[ib] += add_db ? cdb : 0.f;
      split3x8_pair(sa[0][ib], sa[1][ib], q0[ib], q1[ib], q2[ib]);
    }
    FL2_MARK(2);
  };
  // S = h_c·Wᵀ recomputed, then dzpart
  auto spart = [&](const bf16x8* sk, const float* si, bf16x8 (&q0)[2], bf16x8 (&q1)[2], bf16x8 (&q2)[2])
                   __attribute__((always_inline)) {
    f4 sa[2][2];   // [rb][ib]: lane (kg, n) holds rows 16rb + 4kg + u, item 16ib + n
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int ib = 0; ib < 2; ++ib) sa[rb][ib] = f4{0.f, 0.f, 0.f, 0.f};
    bf16x8 a0 = sk[lane], a1 = sk[64 + lane], a2 = sk[128 + lane];
#pragma unroll
    for (int t = 0; t < 2 * NS; ++t) {
      const int s = t >> 1, rb = t & 1;
      const int en = (t + 1 < 2 * NS ? t + 1 : t) * 192 + lane;
      const bf16x8 n0 = sk[en], n1 = sk[en + 64], n2 = sk[en + 128];
#pragma unroll
      for (int ib = 0; ib < 2; ++ib)
        sa[rb][ib] = mfma16_split<NT>(a0, a1, a2, wk[s][ib][0], wk[s][ib][1], wk[s][ib][2], sa[rb][ib]);
      a0 = n0;
      a1 = n1;
      a2 = n2;
      __builtin_amdgcn_sched_barrier(0);
    }
    FL2_MARK(1);
    dzpart(sa, si, q0, q1, q2);
  };
  // dW += dZᵀ·h_c, one R-plane fragment of h per feature block
  auto wpart = [&](const bf16x8* sr, const bf16x8 (&q0)[2], const bf16x8 (&q1)[2], const bf16x8 (&q2)[2])
                   __attribute__((always_inline)) {
    bf16x8 b0 = sr[lane], b1 = sr[64 + lane], b2 = sr[128 + lane];
#pragma unroll
    for (int fb = 0; fb < NF; ++fb) {
      const int en = (fb + 1 < NF ? fb + 1 : fb) * 192 + lane;
      const bf16x8 n0 = sr[en], n1 = sr[en + 64], n2 = sr[en + 128];
#pragma unroll
      for (int ib = 0; ib < 2; ++ib) dw[ib][fb] = mfma16_split<NT>(q0[ib], q1[ib], q2[ib], b0, b1, b2, dw[ib][fb]);
      b0 = n0;
      b1 = n1;
      b2 = n2;
      __builtin_amdgcn_sched_barrier(0);
    }
    FL2_MARK(3);
  };
#define FL2_CHUNK(SK, SI, SR)      \
  do {                             \
    bf16x8 q0_[2], q1_[2], q2_[2]; \
    spart(SK, SI, q0_, q1_, q2_);  \
    wpart(SR, q0_, q1_, q2_);      \
  } while (0)
  if constexpr (ZL) {
    // pass 1's quadrant value (item 4a + u, row b) sits at 4·(16a + 4(b >> 2) +
    // ((b & 3) ^ a)) + u; this lane (kg, l16) needs rows 4kg + r of item l16
    // (a = l16 >> 2, u = l16 & 3): four 4-B reads per quadrant, each
    // instruction over 64 distinct banks
    auto zread = [&](const float* slot, f4 (&d)[2][2]) __attribute__((always_inline)) {
      const float* zb = slot + 1024 * w + 64 * (l16 >> 2) + 16 * kg + (l16 & 3);
#pragma unroll
      for (int rb = 0; rb < 2; ++rb)
#pragma unroll
        for (int ib = 0; ib < 2; ++ib)
#pragma unroll
          for (int r = 0; r < 4; ++r) d[rb][ib][r] = zb[256 * (2 * ib + rb) + 4 * (r ^ (l16 >> 2))];
    };
    // Software-pipelined by one chunk: step c runs chunk c + 1's transpose and
    // dZ VALU (z tile in registers, row records in a three-slot ring) beside
    // chunk c's W-part MFMAs, whose dZ planes the previous step made — the two
    // are independent, so a wave's softmax no longer idles the MFMA pipe.
    // Step c issues chunk c + 1's R-plane DMA (two-slot ring), chunk c + 2's
    // row records and z(c + 3) (three register buffers); its barrier waits
    // for everything but those four z loads (vmcnt(4)).  Branch-free (a wave
    // past A computes on item block 0's tiles and never stores; past the last
    // chunk the DMA / loads repeat the last chunk into idle slots), and slots /
    // buffers are static per call site — unrolled by 6 — so the compiler's
    // LDS-DMA tracking orders reads of a slot behind its own DMA only.
    // the W-part with no sched barriers inside (unlike wpart), so the compiler
    // weaves chunk c + 1's dZ VALU into its MFMA stream (explicit
    // sched_group_barrier patterns — 1 MFMA + 2 VALU, 2 + 4, VALU front-loaded
    // — measured 0.2–0.5 ms slower at C2, profiles/r05/flashx_pass2_interleave.txt)
    auto wpart_il = [&](const bf16x8* sr, const bf16x8 (&q0)[2], const bf16x8 (&q1)[2], const bf16x8 (&q2)[2])
                        __attribute__((always_inline)) {
      bf16x8 b0 = sr[lane], b1 = sr[64 + lane], b2 = sr[128 + lane];
#pragma unroll
      for (int fb = 0; fb < NF; ++fb) {
        const int en = (fb + 1 < NF ? fb + 1 : fb) * 192 + lane;
        const bf16x8 n0 = sr[en], n1 = sr[en + 64], n2 = sr[en + 128];
#pragma unroll
        for (int ib = 0; ib < 2; ++ib) dw[ib][fb] = mfma16_split<NT>(q0[ib], q1[ib], q2[ib], b0, b1, b2, dw[ib][fb]);
        b0 = n0;
        b1 = n1;
        b2 = n2;
      }
    };
    bf16x8 qa0[2], qa1[2], qa2[2], qb0[2], qb1[2], qb2[2];
    if (nch > 0) {
      f4 z0[2][2];
      zread(zr0, z0);
      dzpart(z0, si0, qa0, qa1, qa2);
    }
    auto step = [&](int c, const float* zn1, float* zn3, const bf16x8* rcur, bf16x8* rnext,
                    const float* sin1, float* sin2, const bf16x8 (&qc0)[2], const bf16x8 (&qc1)[2],
                    const bf16x8 (&qc2)[2], bf16x8 (&qn0)[2], bf16x8 (&qn1)[2], bf16x8 (&qn2)[2])
                    __attribute__((always_inline)) {
      f4 z1[2][2];
      zread(zn1, z1);   // z(c + 1) landed by the previous barrier; no DMA in flight yet
      __builtin_amdgcn_sched_barrier(0);
      stage<ER, NW>(Hr + (int64_t)min(c + 1, nch - 1) * ER, rnext, w, lane16);
      if (w == 0 && lane < 16) blds16(rsrc_of(rowinfo + 64 * min(c + 2, nch - 1)), sin2, lane16, 0);
      zdma(c + 3, zn3);
      __builtin_amdgcn_sched_barrier(0);
      dzpart(z1, sin1, qn0, qn1, qn2, c + 1 < nch);   // (past the last chunk: planes unused, no db)
      wpart_il(rcur, qc0, qc1, qc2);
      // pin chunk c + 1's dZ planes (and db) to this step: without it the IR
      // sinks the whole dZ VALU into the next step, next to the MFMAs that
      // consume it, and the pipelining is undone (each step then opened with
      // ~170 VALU before its first MFMA); pinned, the scheduler weaves them
      // into this step's W-part: pass 2 6.49 -> 6.22 ms at C2
      // (profiles/r06/flashx_pass2_pin.txt)
#pragma unroll
      for (int ib = 0; ib < 2; ++ib) asm volatile("" : "+v"(qn0[ib]), "+v"(qn1[ib]), "+v"(qn2[ib]), "+v"(dbs[ib]));
      __builtin_amdgcn_sched_barrier(0);
      FL2_MARK(3);
      __builtin_amdgcn_s_waitcnt(sf2_wc_vm(4));
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      FL2_MARK(4);
    };
    // whole groups of six steps unguarded (straight-line, so the compiler's
    // wait counting across the loop's back edge stays exact), then the rest
    int c = 0;
    for (; c + 6 <= nch; c += 6) {
      step(c, zr1, zr0, sk0, sk1, si1, si2, qa0, qa1, qa2, qb0, qb1, qb2);
      step(c + 1, zr2, zr1, sk1, sk0, si2, si0, qb0, qb1, qb2, qa0, qa1, qa2);
      step(c + 2, zr0, zr2, sk0, sk1, si0, si1, qa0, qa1, qa2, qb0, qb1, qb2);
      step(c + 3, zr1, zr0, sk1, sk0, si1, si2, qb0, qb1, qb2, qa0, qa1, qa2);
      step(c + 4, zr2, zr1, sk0, sk1, si2, si0, qa0, qa1, qa2, qb0, qb1, qb2);
      step(c + 5, zr0, zr2, sk1, sk0, si0, si1, qb0, qb1, qb2, qa0, qa1, qa2);
    }
    if (c < nch) step(c, zr1, zr0, sk0, sk1, si1, si2, qa0, qa1, qa2, qb0, qb1, qb2);
    if (c + 1 < nch) step(c + 1, zr2, zr1, sk1, sk0, si2, si0, qb0, qb1, qb2, qa0, qa1, qa2);
    if (c + 2 < nch) step(c + 2, zr0, zr2, sk0, sk1, si0, si1, qa0, qa1, qa2, qb0, qb1, qb2);
    if (c + 3 < nch) step(c + 3, zr1, zr0, sk1, sk0, si1, si2, qb0, qb1, qb2, qa0, qa1, qa2);
    if (c + 4 < nch) step(c + 4, zr2, zr1, sk0, sk1, si2, si0, qa0, qa1, qa2, qb0, qb1, qb2);
  } else
  for (int c = 0; c < nch; c += 2) {
    bf16x8 q0[2], q1[2], q2[2];
    if (DR) {
      if (c + 1 < nch) {
        FL_ISSUE_K(c + 1, sk1, si1);
        FL_ISSUE_R(c + 1, sr1);
      }
      __builtin_amdgcn_sched_barrier(0);   // keep the prefetch at the top
      if (active) FL2_CHUNK(sk0, si0, sr0);
      FL2_SYNC();
      if (c + 1 < nch) {
        if (c + 2 < nch) {
          FL_ISSUE_K(c + 2, sk0, si0);
          FL_ISSUE_R(c + 2, sr0);
        }
        __builtin_amdgcn_sched_barrier(0);
        if (active) FL2_CHUNK(sk1, si1, sr1);
        FL2_SYNC();
      }
    } else {
      if (c + 1 < nch) FL_ISSUE_K(c + 1, sk1, si1);
      __builtin_amdgcn_sched_barrier(0);
      if (active) spart(sk0, si0, q0, q1, q2);
      FL2_SYNC();
      if (active) wpart(sr0, q0, q1, q2);
      FL2_SYNC();
      if (c + 1 < nch) {
        FL_ISSUE_R(c + 1, sr0);
        if (c + 2 < nch) FL_ISSUE_K(c + 2, sk0, si0);
        __builtin_amdgcn_sched_barrier(0);
        if (active) spart(sk1, si1, q0, q1, q2);
        FL2_SYNC();
        if (active) wpart(sr0, q0, q1, q2);
        FL2_SYNC();
        if (c + 2 < nch) FL_ISSUE_R(c + 2, sr0);
      }
    }
  }
#undef FL_ISSUE_K
#undef FL_ISSUE_R
#undef FL_ISSUE_Z
  // Epilogue, 32 feature columns (two feature blocks) at a time through a
  // per-wave LDS tile (32 items × 32 columns, rows padded to 36 floats): the
  // raw dW tile goes in, every lane then takes four (item, 4-column) pieces —
  // 16-B loads / stores of W, mW, vW (or dW_out), eight 128-B row segments
  // per instruction — and writes the updated values back; with Wk_out /
  // Wr_out (Adam mode) the updated rows also leave as the next pass 1's
  // operand planes, read from the tile (R-planes: items kperm16(kg, e) of a
  // column; K-planes: 8 consecutive columns of an item)
  // (the ring arrays are idle after the main loop's last barrier; HF 32's are
  // too small, so it has its own)
  constexpr int TRP = 36, TRW = 32 * TRP;         // floats per wave (16-B aligned rows)
  constexpr int WPA = EK * 16 / (TRW * 4);        // waves per ring array
  __shared__ __attribute__((aligned(16))) float trd[(HF == 32 && !ZL) ? NW * TRW : 4];
  float* tr;
  if constexpr (ZL) {
    // (the z ring is idle after the last barrier; each array holds 1024·NW floats)
    constexpr int WPZ = 1024 * NW / TRW;
    static_assert(WPZ * 3 >= NW, "epilogue tiles fit the z ring");
    tr = (w / WPZ == 0 ? zr0 : w / WPZ == 1 ? zr1 : zr2) + (w % WPZ) * TRW;
  } else if (HF == 32) {
    tr = trd + w * TRW;
  } else {
    const int ai = w / WPA, ao = (w % WPA) * TRW;
    bf16x8* base = ai == 0 ? sk0 : ai == 1 ? sk1 : ai == 2 ? sr0 : sr1;
    tr = reinterpret_cast<float*>(base) + ao;
  }
  if (!active) {
    FL2_STORE();
    return;
  }
  const bool planes = Wk_out != nullptr && dW_out == nullptr;
  float dbt[2];
#pragma unroll
  for (int ib = 0; ib < 2; ++ib) {
    dbt[ib] = dbs[ib] + __shfl_xor(dbs[ib], 16);
    dbt[ib] += __shfl_xor(dbt[ib], 32);
  }
  if (tail) {
    const int i0 = nfull * fl_rows(HF, 2), ntail = A - i0, part = (bx - nfull) % tsplit;
#pragma unroll
    for (int ib = 0; ib < 2; ++ib) {
      const int item = j0 + 16 * ib + l16;
      if (kg == 0 && item < A) tail_db[(int64_t)part * ntail + item - i0] = dbt[ib];
#pragma unroll
      for (int fb = 0; fb < NF; ++fb)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int it = j0 + 16 * ib + 4 * kg + i;
          if (it < A) tail_dw[((int64_t)part * ntail + it - i0) * HF + 16 * fb + l16] = dw[ib][fb][i];
        }
    }
    FL2_MARK(5);
    FL2_STORE();
    return;
  }
#pragma unroll
  for (int ib = 0; ib < 2; ++ib) {
    const int item = j0 + 16 * ib + l16;
    if (kg == 0 && item < A) {
      if (db_out) {
        db_out[item] = dbt[ib];
      } else {
        float p = bias[item], mq = mb[item], v = vb[item];
        adam_elem(p, mq, v, dbt[ib], args);
        bias[item] = p;
        mb[item] = mq;
        vb[item] = v;
        if (planes) bias_pad_out[item] = p;
      }
    }
  }
  const int64_t blk32 = j0 >> 5;
  const int c4 = lane & 7;
  // W / mW / vW of the 32-column slab s, loaded one slab ahead and
  // unconditionally (rows past A clamp to A − 1; only the stores are guarded),
  // so the 16 (slab, q) steps do not each wait a full memory round trip (the
  // guarded per-q loads could not be hoisted: 3 loads, vmcnt(0), Adam, 3
  // stores, 16 times over)
  f4 pwp[2][4], mqp[2][4], vvp[2][4];
  auto ldp = [&](int s, int slot) __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int it = min(j0 + (lane >> 3) + 8 * q, A - 1);
      const int64_t o = (int64_t)it * HF + 32 * s + 4 * c4;
      pwp[slot][q] = *reinterpret_cast<const f4*>(W + o);
      mqp[slot][q] = *reinterpret_cast<const f4*>(mW + o);
      vvp[slot][q] = *reinterpret_cast<const f4*>(vW + o);
    }
  };
  if (!dW_out) ldp(0, 0);
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    if (!dW_out && s + 1 < NS) ldp(s + 1, (s + 1) & 1);
#pragma unroll
    for (int f2 = 0; f2 < 2; ++f2)
#pragma unroll
      for (int ib = 0; ib < 2; ++ib)
#pragma unroll
        for (int i = 0; i < 4; ++i) tr[(16 * ib + 4 * kg + i) * TRP + 16 * f2 + l16] = dw[ib][2 * s + f2][i];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int ii = (lane >> 3) + 8 * q, it = j0 + ii;
      f4* tp = reinterpret_cast<f4*>(tr + ii * TRP + 4 * c4);
      f4 gv = *tp;
      if (it < A) {
        const int64_t o = (int64_t)it * HF + 32 * s + 4 * c4;
        if (dW_out) {
          *reinterpret_cast<f4*>(dW_out + o) = gv;
        } else {
          f4 pw = pwp[s & 1][q], mq = mqp[s & 1][q], v = vvp[s & 1][q];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            float pu = pw[u], mu = mq[u], vu = v[u];
            adam_elem(pu, mu, vu, gv[u], args);
            pw[u] = pu;
            mq[u] = mu;
            v[u] = vu;
          }
          *reinterpret_cast<f4*>(W + o) = pw;
          *reinterpret_cast<f4*>(mW + o) = mq;
          *reinterpret_cast<f4*>(vW + o) = v;
          gv = pw;
        }
      } else {
        gv = f4{0.f, 0.f, 0.f, 0.f};   // rows past A: zero planes, as rg_head_planes writes them
      }
      if (planes) *tp = gv;
    }
    if (planes) {
#pragma unroll
      for (int f2 = 0; f2 < 2; ++f2) {
        f4 lo, hi;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float x = tr[kperm16(kg, e) * TRP + 16 * f2 + l16];
          if (e < 4) lo[e] = x; else hi[e - 4] = x;
        }
        bf16x8 p0, p1, p2;
        split3x8(lo, hi, p0, p1, p2);
        bf16x8* dst = Wr_out + (blk32 * NF + 2 * s + f2) * 192 + lane;
        dst[0] = p0;
        dst[64] = p1;
        dst[128] = p2;
      }
      // (item, 8-column group) entries of columns 32s .. 32s + 31: 32 items × 4 groups
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int e = lane + 64 * q, ii = e & 31, grp = e >> 5;
        const f4* src = reinterpret_cast<const f4*>(tr + ii * TRP + 8 * grp);
        bf16x8 p0, p1, p2;
        split3x8(src[0], src[1], p0, p1, p2);
        bf16x8* dst = Wk_out + ((blk32 * NS + s) * 2 + (ii >> 4)) * 192 + 16 * grp + (ii & 15);
        dst[0] = p0;
        dst[64] = p1;
        dst[128] = p2;
      }
    }
  }
  FL2_MARK(5);
  FL2_STORE();
}

// -------------------------------------------------------- fused top-k ----
// Top-1: merge the per-split (best, item) of pass 1 (splits ascend in item
// order, so keeping the earlier split on a tie keeps the first maximum).
__global__ void k_flash_argmax(const float* __restrict__ pbest, const int32_t* __restrict__ parg, int nsplit, int B,
                               int32_t* __restrict__ out, float* __restrict__ out_max) {
  const int row = blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= B) return;
  float bv = NEG_INF;
  int bi = INT32_MAX;
  for (int s = 0; s < nsplit; ++s) {
    const float v = pbest[(int64_t)s * B + row];
    const int i = parg[(int64_t)s * B + row];
    if (i != INT32_MAX && (v > bv || bi == INT32_MAX)) {
      bv = v;
      bi = i;
    }
  }
  out[row] = bi == INT32_MAX ? -1 : bi;
  if (out_max) out_max[row] = bv;
}

// Top-K (K <= TK_MAX): the K largest 32-item chunk maxima of a row bound its
// K-th largest logit from below (they hold K distinct items), so every top-K
// item lies in a chunk whose maximum is >= that bound tau.  Chunks with
// cmax >= tau - tol (tol covers the split-bf16 error of cmax) are the
// candidates; their items are rescored in plain fp32 and ranked in the
// canonical (value desc, index asc) order.
constexpr int TK_MAX = 32;
constexpr int TK_CAP = 64;   // candidate chunks per row (2048 items)

__device__ __forceinline__ void tk_insert(float (&t)[TK_MAX], float v) {
#pragma unroll
  for (int i = 0; i < TK_MAX; ++i) {
    const float hi = fmaxf(t[i], v);
    v = fminf(t[i], v);
    t[i] = hi;
  }
}

// tau = the K-th largest chunk maximum of every row, in two stages so the
// chunk range is read by the whole chip (one workgroup per row block scanning
// all ceil(A/32) chunks was latency-bound: ~8 ms at C4 for K = 1).
// Stage 1: grid (row blocks of 64, P parts of the chunk range), lane = row,
// the 4 waves interleave the part's chunks; each wave keeps its top-K, the
// part's top-K (merged in LDS) goes to part[p][i][row].
__global__ __launch_bounds__(256) void k_topk_part(const float* __restrict__ cmax, int nct, int ldc, int B, int K,
                                                   float* __restrict__ part) {
  __shared__ float st[4][TK_MAX][64];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int row = blockIdx.x * 64 + lane;
  const bool ok = row < B;
  const int P = gridDim.y, per = (nct + P - 1) / P;
  const int c0 = blockIdx.y * per, c1 = min(nct, c0 + per);
  float t[TK_MAX];
#pragma unroll
  for (int i = 0; i < TK_MAX; ++i) t[i] = NEG_INF;
  float thr = NEG_INF;   // t[K-1]
  for (int c = c0 + w; c < c1; c += 16) {
    float v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {   // four independent loads in flight per lane
      const int cc = c + 4 * u;
      v[u] = (ok && cc < c1) ? cmax[(int64_t)cc * ldc + row] : NEG_INF;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (v[u] > thr) {
        tk_insert(t, v[u]);
#pragma unroll
        for (int i = 0; i < TK_MAX; ++i)
          if (i == K - 1) thr = t[i];
      }
    }
  }
#pragma unroll
  for (int i = 0; i < TK_MAX; ++i) st[w][i][lane] = t[i];
  __syncthreads();
  if (w == 0) {
    for (int q = 1; q < 4; ++q)
      for (int i = 0; i < K; ++i) {
        const float v = st[q][i][lane];
        if (v > thr) {
          tk_insert(t, v);
#pragma unroll
          for (int j = 0; j < TK_MAX; ++j)
            if (j == K - 1) thr = t[j];
        }
      }
    if (ok)
#pragma unroll
      for (int i = 0; i < TK_MAX; ++i)
        if (i < K) part[((int64_t)blockIdx.y * K + i) * ldc + row] = t[i];
  }
}

// Stage 2: per row the K-th largest of the P·K part values -> the candidate
// limit lim = tau − (tol_abs + tol_rel·|tau|) (−inf while fewer than K finite
// maxima exist: every chunk is then a candidate); ncand := 0.  With wnorm
// (screened chunk maxima, 3 plane products): tol_abs = tol·||h_b||_2·wnorm[0]
// per row — the screening argmax's bound (rg_flash_argmax_exact).
__global__ void k_topk_lim(const float* __restrict__ part, int P, int K, int ldc, int B, float tol_abs, float tol_rel,
                           float* __restrict__ lim, int32_t* __restrict__ ncand, const float* __restrict__ h, int HF,
                           const float* __restrict__ wnorm) {
  const int row = blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= B) return;
  if (wnorm) {
    float hn = 0.f;
    for (int k = 0; k < HF; ++k) hn = fmaf(h[(int64_t)row * HF + k], h[(int64_t)row * HF + k], hn);
    tol_abs = tol_abs * sqrtf(hn) * wnorm[0];
  }
  float t[TK_MAX];
#pragma unroll
  for (int i = 0; i < TK_MAX; ++i) t[i] = NEG_INF;
  float thr = NEG_INF;
  for (int j = 0; j < P * K; ++j) {
    const float v = part[(int64_t)j * ldc + row];
    if (v > thr) {
      tk_insert(t, v);
#pragma unroll
      for (int i = 0; i < TK_MAX; ++i)
        if (i == K - 1) thr = t[i];
    }
  }
  lim[row] = thr > NEG_INF ? thr - (tol_abs + tol_rel * fabsf(thr)) : NEG_INF;
  ncand[row] = 0;
}

// The fp32 logit of one item: the native fp32 head's own chain (csrc/head.hip
// k_head_fwd*: v_mfma_f32_32x32x2_f32 with k = s from lane half 0 and k =
// HF/2 + s from half 1, i.e. fmaf over s of (h[s]·w[s], then h[HF/2+s]·w[HF/2+s]),
// then + bias), so a re-scored logit is bitwise the one the model's forward()
// stores and the top-K equals the canonical top-K of those logits.
__device__ __forceinline__ float head_logit(const float* hs, const float* __restrict__ W,
                                            const float* __restrict__ bias, int item, int HF) {
  const f4* wr = reinterpret_cast<const f4*>(W + (int64_t)item * HF);
  const int kh4 = HF / 8;   // float4s per half
  float acc = 0.f;
  for (int s4 = 0; s4 < kh4; ++s4) {
    const f4 xa = wr[s4], xb = wr[kh4 + s4];
    const int ka = 4 * s4, kb = HF / 2 + 4 * s4;
    acc = fmaf(hs[ka], xa[0], acc);
    acc = fmaf(hs[kb], xb[0], acc);
    acc = fmaf(hs[ka + 1], xa[1], acc);
    acc = fmaf(hs[kb + 1], xb[1], acc);
    acc = fmaf(hs[ka + 2], xa[2], acc);
    acc = fmaf(hs[kb + 2], xb[2], acc);
    acc = fmaf(hs[ka + 3], xa[3], acc);
    acc = fmaf(hs[kb + 3], xb[3], acc);
  }
  return acc + bias[item];
}

__device__ __forceinline__ bool tk_overflow(int nc) { return nc < 0 || nc > TK_CAP; }

// one workgroup (256 threads) per row: fp32 logits (head_logit) of the
// candidate items, canonical top-K.  A row with more than TK_CAP candidate
// chunks (a tie run past the cap) is left to k_flash_topk_scan.
__global__ __launch_bounds__(256) void k_flash_topk_eval(const float* __restrict__ h, const float* __restrict__ W,
                                                         const float* __restrict__ bias, const int32_t* __restrict__ cand,
                                                         const int32_t* __restrict__ ncand, int A, int HF, int K,
                                                         int32_t* __restrict__ out_idx, float* __restrict__ out_val) {
  __shared__ __attribute__((aligned(16))) float hs[256];
  __shared__ float cv[TK_CAP * 32];
  __shared__ int ci[TK_CAP * 32];
  __shared__ float rv[4];
  __shared__ int ri[4], rs[4];
  const int row = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (tk_overflow(ncand[row])) return;
  for (int k = tid; k < HF; k += 256) hs[k] = h[(int64_t)row * HF + k];
  const int n = ncand[row] * 32;
  __syncthreads();
  for (int e = tid; e < n; e += 256) {
    const int item = cand[(int64_t)row * TK_CAP + (e >> 5)] * 32 + (e & 31);
    const float z = item < A ? head_logit(hs, W, bias, item, HF) : NEG_INF;
    cv[e] = z;
    ci[e] = item < A ? item : INT32_MAX;
  }
  __syncthreads();
  for (int k = 0; k < K; ++k) {
    float bv = NEG_INF;
    int bi = INT32_MAX, bs = -1;
    for (int e = tid; e < n; e += 256) {
      const float v = cv[e];
      const int i = ci[e];
      if (i != INT32_MAX && (v > bv || (v == bv && i < bi) || bs < 0)) {
        bv = v;
        bi = i;
        bs = e;
      }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      const float v2 = __shfl_xor(bv, o);
      const int i2 = __shfl_xor(bi, o), s2 = __shfl_xor(bs, o);
      if (s2 >= 0 && (bs < 0 || v2 > bv || (v2 == bv && i2 < bi))) {
        bv = v2;
        bi = i2;
        bs = s2;
      }
    }
    if (lane == 0) {
      rv[w] = bv;
      ri[w] = bi;
      rs[w] = bs;
    }
    __syncthreads();
    if (tid == 0) {
      for (int q = 1; q < 4; ++q)
        if (rs[q] >= 0 && (rs[0] < 0 || rv[q] > rv[0] || (rv[q] == rv[0] && ri[q] < ri[0]))) {
          rv[0] = rv[q];
          ri[0] = ri[q];
          rs[0] = rs[q];
        }
      out_idx[(int64_t)row * K + k] = rs[0] >= 0 ? ri[0] : -1;
      if (out_val) out_val[(int64_t)row * K + k] = rv[0];
      if (rs[0] >= 0) ci[rs[0]] = INT32_MAX;   // taken
    }
    __syncthreads();
  }
}

// the overflowed rows of k_flash_topk_eval (ncand > TK_CAP): every item of
// the row re-scored by head_logit, canonical top-K (topk_scan.h); every other
// row's workgroup exits at once.  err (optional) counts the rows scanned.
struct HeadRowSrc {
  const float* h;
  const float* W;
  const float* bias;
  float* hs;
  int HF;
  __device__ void prepare(int row) {
    for (int k = threadIdx.x; k < HF; k += 256) hs[k] = h[(int64_t)row * HF + k];
    __syncthreads();
  }
  __device__ float operator()(int item) const { return head_logit(hs, W, bias, item, HF); }
};

__global__ __launch_bounds__(256) void k_flash_topk_scan(const float* __restrict__ h, const float* __restrict__ W,
                                                         const float* __restrict__ bias, const int32_t* __restrict__ ncand,
                                                         int A, int HF, int K, int32_t* __restrict__ out_idx,
                                                         float* __restrict__ out_val, int32_t* __restrict__ err) {
  __shared__ __attribute__((aligned(16))) float hs[256];
  const int row = blockIdx.x;
  if (!tk_overflow(ncand[row])) return;
  if (err && threadIdx.x == 0) atomicAdd(err, 1);
  HeadRowSrc src{h, W, bias, hs, HF};
  topk_scan_row(src, row, A, K, out_idx, out_val);
}

// out[0] = max_a ||W_a||_2 (float bits ordered as uint: max is order-independent);
// out[0] must be 0 on entry.  32 lanes per row, HF / 4 <= 64 float4s per row.
__global__ __launch_bounds__(256) void k_row_norm_max(const float* __restrict__ W, int64_t A, int HF,
                                                      float* __restrict__ out) {
  const int lane = threadIdx.x & 31, n4 = HF / 4;
  float best = 0.f;
  for (int64_t a = (blockIdx.x * 256 + threadIdx.x) / 32; a < A; a += (int64_t)gridDim.x * 8) {
    const f4* wr = reinterpret_cast<const f4*>(W + a * HF);
    float s = 0.f;
    for (int k = lane; k < n4; k += 32) {
      const f4 x = wr[k];
      s = fmaf(x[0], x[0], fmaf(x[1], x[1], fmaf(x[2], x[2], fmaf(x[3], x[3], s))));
    }
#pragma unroll
    for (int o = 16; o >= 1; o >>= 1) s += __shfl_xor(s, o);
    best = fmaxf(best, sqrtf(s));
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) best = fmaxf(best, __shfl_xor(best, o));
  if ((threadIdx.x & 63) == 0) atomicMax(reinterpret_cast<unsigned int*>(out), __float_as_uint(best));
}

// per row: lim = tau − (tol·||h_b||_2·wnorm[0] + 1e-6·|tau|), tau = the screening's best (value)
__global__ void k_amax_lim(const float* __restrict__ best, const float* __restrict__ h, int B, int HF,
                           const float* __restrict__ wnorm, float tol, float* __restrict__ lim) {
  const int row = blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= B) return;
  float hn = 0.f;
  for (int k = 0; k < HF; ++k) hn = fmaf(h[(int64_t)row * HF + k], h[(int64_t)row * HF + k], hn);
  const float tau = best[row];
  lim[row] = tau > NEG_INF ? tau - (tol * sqrtf(hn) * wnorm[0] + 1e-6f * fabsf(tau)) : NEG_INF;
}

// candidate chunks (cmax >= lim) of every row, chunk range split over grid.y;
// appended in any order through a per-row counter (the re-scoring keeps the
// first maximum by (value, item), so the order does not matter)
__global__ __launch_bounds__(256) void k_amax_cand(const float* __restrict__ cmax, int nct, int ldc, int B,
                                                   const float* __restrict__ lim, int32_t* __restrict__ cand,
                                                   int32_t* __restrict__ ncand) {
  const int row = blockIdx.x * 256 + threadIdx.x;
  if (row >= B) return;
  const int per = (nct + gridDim.y - 1) / gridDim.y;
  const int c0 = blockIdx.y * per, c1 = min(nct, c0 + per);
  const float l = lim[row];
  for (int c = c0; c < c1; ++c) {
    if (cmax[(int64_t)c * ldc + row] >= l) {
      const int p = atomicAdd(&ncand[row], 1);
      if (p < TK_CAP) cand[(int64_t)row * TK_CAP + p] = c;
    }
  }
}

// pass 2's tail: sum the tsplit partials of every leftover item in part
// order, then the raw gradient (dW_out / db_out) or Adam on W / b
__global__ __launch_bounds__(256) void k_flash_tail(const float* __restrict__ tail_dw, const float* __restrict__ tail_db,
                                                    int tsplit, int i0, int ntail, int HF, float* __restrict__ W,
                                                    float* __restrict__ mW, float* __restrict__ vW,
                                                    float* __restrict__ bias, float* __restrict__ mb,
                                                    float* __restrict__ vb, AdamArgs args, float* __restrict__ dW_out,
                                                    float* __restrict__ db_out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t n = (int64_t)ntail * HF;
  if (i < n) {
    float gs = 0.f;
    for (int p = 0; p < tsplit; ++p) gs += tail_dw[(int64_t)p * n + i];
    const int64_t o = (int64_t)i0 * HF + i;
    if (dW_out) {
      dW_out[o] = gs;
    } else {
      float pw = W[o], mq = mW[o], v = vW[o];
      adam_elem(pw, mq, v, gs, args);
      W[o] = pw;
      mW[o] = mq;
      vW[o] = v;
    }
  }
  if (i < ntail) {
    float gs = 0.f;
    for (int p = 0; p < tsplit; ++p) gs += tail_db[(int64_t)p * ntail + i];
    if (db_out) {
      db_out[i0 + i] = gs;
    } else {
      float pb = bias[i0 + i], mq = mb[i0 + i], v = vb[i0 + i];
      adam_elem(pb, mq, v, gs, args);
      bias[i0 + i] = pb;
      mb[i0 + i] = mq;
      vb[i0 + i] = v;
    }
  }
}

// pass 2's grid: nfull whole item blocks, then the leftover blocks split tsplit
// ways over the row chunks when they would fill less than ~3/4 of a round
struct FlTail {
  int nfull, tsplit, ntail;
};
inline FlTail fl_tail(int B, int A, int HF) {
  const int rpb = fl_rows(HF, 2), nblk = (A + rpb - 1) / rpb, nct = B / 32;
  const int nfull = nblk / 256 * 256, left = nblk - nfull;
  if (nfull == 0 || left == 0 || left > 192) return FlTail{nblk, 1, 0};
  int ts = min(min(8, 256 / left), nct);
  // no part without row chunks: k_flash_dw's prologue DMAs its part's first
  // chunk (rows past the last chunk otherwise) before it knows nch
  const int cper = (nct + ts - 1) / ts;
  ts = (nct + cper - 1) / cper;
  if (ts < 2) return FlTail{nblk, 1, 0};
  return FlTail{nfull, ts, A - nfull * rpb};
}

inline bool flash_hf_ok(int HF) { return HF == 32 || HF == 64 || HF == 128 || HF == 256; }
inline bool flash_terms_ok(int t) { return t == 6 || t == 9 || t == RG_TERMS_X6D3; }

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
  const unsigned gr = (unsigned)(((int64_t)(rp / 32) * (HF / 16) * 64 + 255) / 256);
#define PL(HFV)                                                                                                \
  if (planes_k)                                                                                                \
    hipLaunchKernelGGL(k_planes_k<HFV>, dim3(gk), dim3(256), 0, stream, X, rows, rp, (bf16x8*)planes_k);     \
  if (planes_r) hipLaunchKernelGGL(k_planes_r<HFV>, dim3(gr), dim3(256), 0, stream, X, rows, rp, (bf16x8*)planes_r)
  switch (HF) {
    case 32: PL(32); break;
    case 64: PL(64); break;
    case 128: PL(128); break;
    case 256: PL(256); break;
  }
#undef PL
  if (bias && bias_pad)
    hipLaunchKernelGGL(k_pad_bias, dim3((rp + 255) / 256), dim3(256), 0, stream, bias, rows, rp, bias_pad);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_flash_rows_per_block(int HF) { return flash_hf_ok(HF) ? fl_rows(HF, 1) : RG_ERR_SHAPE; }

extern "C" int64_t rg_flash_zs_bytes(int B, int A) {
  if (B <= 0 || A <= 0 || (B % 32)) return RG_ERR_ARG;
  return (int64_t)((A + 31) / 32) * 32 * B * 4;
}

extern "C" int rg_flash_fwd_top(const void* Hk, const void* Wk, const void* Wr, const float* bias_pad, int B, int A,
                                int HF, int terms, int nsplit, float* pm, float* pl, float* pO, float* pbest,
                                int32_t* parg, float* cmax, float* zs, hipStream_t stream) {
  if (B <= 0 || A <= 0 || (B % 32) || nsplit <= 0 || !Hk || !Wk || !Wr || !bias_pad || !pm || !pl || !pO)
    return RG_ERR_ARG;
  if (!flash_terms_ok(terms)) return RG_ERR_ARG;
  if (!flash_hf_ok(HF)) return RG_ERR_SHAPE;
  const bool arg = pbest != nullptr;
  if (arg != (parg != nullptr)) return RG_ERR_ARG;
  const int rpb = fl_rows(HF, 1);
  if (zs && B % rpb) return RG_ERR_SHAPE;   // stored logits: whole row blocks
  const int nct = (A + 31) / 32;
  const int cps = (nct + nsplit - 1) / nsplit;
  const int nrb = (B + rpb - 1) / rpb;
  const dim3 grid((unsigned)(nrb * nsplit));
#define FF(HFV, NTV, NGV, ARGV, ZSV)                                                                          \
  hipLaunchKernelGGL((k_flash_fwd<HFV, NTV, NGV, ARGV, ZSV>), grid, dim3(64 * fl_nw(HFV, 1)), 0, stream,           \
                     (const bf16x8*)Hk, (const bf16x8*)Wk, (const bf16x8*)Wr, bias_pad, B, A, nrb, nsplit, cps, pm, \
                     pl, pO, pbest, parg, cmax, zs)
#define FZ1(HFV, NTV, NGV, ARGV)            \
  if (zs) {                                 \
    FF(HFV, NTV, NGV, ARGV, true);          \
  } else {                                  \
    FF(HFV, NTV, NGV, ARGV, false);         \
  }
#define FA(HFV, NTV, NGV)      \
  if (arg) {                   \
    FZ1(HFV, NTV, NGV, 2);     \
  } else if (cmax) {           \
    FZ1(HFV, NTV, NGV, 1);     \
  } else {                     \
    FZ1(HFV, NTV, NGV, 0);     \
  }
#define FT(HFV)                        \
  if (terms == 9) {                    \
    FA(HFV, 9, 9);                     \
  } else if (terms == RG_TERMS_X6D3) { \
    FA(HFV, 6, 3);                     \
  } else {                             \
    FA(HFV, 6, 6);                     \
  }
  switch (HF) {
    case 32: FT(32); break;
    case 64: FT(64); break;
    case 128: FT(128); break;
    case 256: FT(256); break;
  }
#undef FT
#undef FZ1
#undef FA
#undef FF
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_flash_fwd(const void* Hk, const void* Wk, const void* Wr, const float* bias_pad, int B, int A,
                            int HF, int terms, int nsplit, float* pm, float* pl, float* pO, hipStream_t stream) {
  return rg_flash_fwd_top(Hk, Wk, Wr, bias_pad, B, A, HF, terms, nsplit, pm, pl, pO, nullptr, nullptr, nullptr,
                          nullptr, stream);
}

// Evaluation scoring (no O contraction): pass 1's S-part over the fp32
// logits at `terms` plane products — per-(split, row) max / Σexp (-> lse via
// rg_flash_lse), per-split first maximum and every 32-item chunk's row
// maximum (-> exact canonical top-K via rg_flash_topk).
extern "C" int rg_flash_score(const void* Hk, const void* Wk, const float* bias_pad, int B, int A, int HF, int terms,
                              int nsplit, float* pm, float* pl, float* pbest, int32_t* parg, float* cmax,
                              hipStream_t stream) {
  if (B <= 0 || A <= 0 || (B % 32) || nsplit <= 0 || !Hk || !Wk || !bias_pad || !pm || !pl || !pbest || !parg ||
      !cmax)
    return RG_ERR_ARG;
  if (terms == RG_TERMS_X6D3) terms = 6;   // logits only
  if (terms != 6 && terms != 9) return RG_ERR_ARG;
  if (!flash_hf_ok(HF)) return RG_ERR_SHAPE;
  const int nct = (A + 31) / 32;
  const int cps = (nct + nsplit - 1) / nsplit;
  const int rpb = fl_rows(HF, 1);
  const int nrb = (B + rpb - 1) / rpb;
  const dim3 grid((unsigned)(nrb * nsplit));
#define FSC(HFV, NTV)                                                                                             \
  hipLaunchKernelGGL((k_flash_fwd<HFV, NTV, 0, 2>), grid, dim3(64 * fl_nw(HFV, 1)), 0, stream, (const bf16x8*)Hk, \
                     (const bf16x8*)Wk, (const bf16x8*)nullptr, bias_pad, B, A, nrb, nsplit, cps, pm, pl,         \
                     (float*)nullptr, pbest, parg, cmax, (float*)nullptr)
#define FT(HFV)          \
  if (terms == 9) {      \
    FSC(HFV, 9);         \
  } else {               \
    FSC(HFV, 6);         \
  }
  switch (HF) {
    case 32: FT(32); break;
    case 64: FT(64); break;
    case 128: FT(128); break;
    case 256: FT(256); break;
  }
#undef FT
#undef FSC
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_flash_amax_fwd(const void* Hk, const void* Wk, const float* bias_pad, int B, int A, int HF,
                                 int terms, int nsplit, float* pbest, int32_t* parg, hipStream_t stream) {
  if (B <= 0 || A <= 0 || (B % 32) || nsplit <= 0 || !Hk || !Wk || !bias_pad || !pbest || !parg) return RG_ERR_ARG;
  if (terms == RG_TERMS_X6D3) terms = 6;   // logits only
  if (terms != 6 && terms != 9) return RG_ERR_ARG;
  if (!flash_hf_ok(HF)) return RG_ERR_SHAPE;
  const int nct = (A + 31) / 32;
  const int cps = (nct + nsplit - 1) / nsplit;
  const int rpb = fl_rows(HF, 1);
  const int nrb = (B + rpb - 1) / rpb;
  const dim3 grid((unsigned)(nrb * nsplit));
#define FM(HFV, NTV)                                                                                            \
  hipLaunchKernelGGL((k_flash_amax<HFV, NTV, false>), grid, dim3(64 * fl_nw(HFV, 1)), 0, stream, (const bf16x8*)Hk, \
                     (const bf16x8*)Wk, bias_pad, B, A, nrb, nsplit, cps, pbest, parg, (float*)nullptr)
#define FT(HFV)          \
  if (terms == 9) {      \
    FM(HFV, 9);          \
  } else {               \
    FM(HFV, 6);          \
  }
  switch (HF) {
    case 32: FT(32); break;
    case 64: FT(64); break;
    case 128: FT(128); break;
    case 256: FT(256); break;
  }
#undef FT
#undef FM
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_flash_argmax(const float* pbest, const int32_t* parg, int nsplit, int B, int32_t* out,
                               float* out_max, hipStream_t stream) {
  if (B <= 0 || nsplit <= 0 || !pbest || !parg || !out) return RG_ERR_ARG;
  hipLaunchKernelGGL(k_flash_argmax, dim3((B + 255) / 256), dim3(256), 0, stream, pbest, parg, nsplit, B, out,
                     out_max);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_flash_topk_cap(void) { return TK_CAP; }

// parts of the chunk range for tau (stage 1): ~2048 workgroups, >= 64 chunks each
inline int topk_parts(int B, int nct) { return max(1, min(64, min(2048 / ((B + 63) / 64), nct / 64))); }

extern "C" int64_t rg_flash_topk_work_bytes(int B, int A, int K) {
  if (B <= 0 || A <= 0 || K <= 0 || K > TK_MAX) return RG_ERR_ARG;
  return ((int64_t)topk_parts(B, (A + 31) / 32) * K * B + B) * 4;
}

// rows [0, B) of a chunk whose chunk maxima have row stride ldc >= B (cmax:
// ceil(A/32) × ldc; work sized for ldc rows, rg_flash_topk_work_bytes(ldc, …))
static int flash_topk(const float* cmax, int ldc, int B, int A, int K, float tol_abs, float tol_rel, const float* wnorm,
                      const float* h, const float* W, const float* bias, int HF, int32_t* cand, int32_t* ncand,
                      int32_t* out_idx, float* out_val, int32_t* err, void* work, hipStream_t stream) {
  if (B <= 0 || ldc < B || A <= 0 || K <= 0 || K > TK_MAX || K > A || HF <= 0 || HF > 256 || (HF % 8))
    return RG_ERR_ARG;
  if (!cmax || !h || !W || !bias || !cand || !ncand || !out_idx || !work) return RG_ERR_ARG;
  const int nct = (A + 31) / 32;
  const int P = topk_parts(ldc, nct);
  float* part = (float*)work;
  float* lim = part + (int64_t)P * K * ldc;
  hipLaunchKernelGGL(k_topk_part, dim3((B + 63) / 64, P), dim3(256), 0, stream, cmax, nct, ldc, B, K, part);
  hipLaunchKernelGGL(k_topk_lim, dim3((B + 255) / 256), dim3(256), 0, stream, part, P, K, ldc, B, tol_abs, tol_rel,
                     lim, ncand, h, HF, wnorm);
  const int ys = max(1, min(256, 2048 / ((B + 255) / 256)));   // ~2048 workgroups over the chunk range
  hipLaunchKernelGGL(k_amax_cand, dim3((B + 255) / 256, ys), dim3(256), 0, stream, cmax, nct, ldc, B, lim, cand,
                     ncand);
  hipLaunchKernelGGL(k_flash_topk_eval, dim3(B), dim3(256), 0, stream, h, W, bias, cand, ncand, A, HF, K, out_idx,
                     out_val);
  hipLaunchKernelGGL(k_flash_topk_scan, dim3(B), dim3(256), 0, stream, h, W, bias, ncand, A, HF, K, out_idx, out_val,
                     err);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_flash_topk(const float* cmax, int ldc, int B, int A, int K, float tol_abs, float tol_rel,
                             const float* h, const float* W, const float* bias, int HF, int32_t* cand, int32_t* ncand,
                             int32_t* out_idx, float* out_val, int32_t* err, void* work, hipStream_t stream) {
  return flash_topk(cmax, ldc, B, A, K, tol_abs, tol_rel, nullptr, h, W, bias, HF, cand, ncand, out_idx, out_val, err,
                    work, stream);
}

// Top-K from SCREENED chunk maxima (rg_flash_amax_screen: 3 plane products):
// candidates within tol·||h_b||_2·wnorm[0] + 1e-6·|tau| of tau (wnorm from
// rg_row_norm_max), re-scored exactly as rg_flash_topk (a row past the
// candidate cap is scanned whole, as there).
extern "C" int rg_flash_topk_screened(const float* cmax, int ldc, int B, int A, int K, float tol, const float* wnorm,
                                      const float* h, const float* W, const float* bias, int HF, int32_t* cand,
                                      int32_t* ncand, int32_t* out_idx, float* out_val, int32_t* err, void* work,
                                      hipStream_t stream) {
  if (!wnorm) return RG_ERR_ARG;
  return flash_topk(cmax, ldc, B, A, K, tol, 1e-6f, wnorm, h, W, bias, HF, cand, ncand, out_idx, out_val, err, work,
                    stream);
}

extern "C" int rg_flash_lse(const float* pm, const float* pl, int nsplit, const float* h, const float* W,
                            const float* bias, const int64_t* tgt, int64_t lo, int A, int64_t A_full, int B, int HF,
                            float* lse, float* zt, hipStream_t stream) {
  if (B <= 0 || A <= 0 || nsplit <= 0 || !pm || !pl || !lse) return RG_ERR_ARG;
  if (zt && (!h || !W || !bias || !tgt || A_full < lo + A)) return RG_ERR_ARG;
  if (zt && !flash_hf_ok(HF)) return RG_ERR_SHAPE;
#define FLS(HFV)                                                                                                 \
  hipLaunchKernelGGL(k_flash_lse<HFV>, dim3((B + 63) / 64), dim3(64), 0, stream, pm, pl, nsplit, h, W, bias, tgt, lo, \
                     A, A_full, B, lse, zt)
  switch (zt ? HF : 32) {
    case 32: FLS(32); break;
    case 64: FLS(64); break;
    case 128: FLS(128); break;
    case 256: FLS(256); break;
  }
#undef FLS
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_flash_rows(const float* lse, const int64_t* tgt, int64_t lo, int A, int B, void* rowinfo,
                             hipStream_t stream) {
  // records of 32-row chunks (ri_lse / ri_tgt): the fused head's batches are whole chunks
  if (B <= 0 || A <= 0 || (B % 32) || !lse || !tgt || !rowinfo) return RG_ERR_ARG;
  hipLaunchKernelGGL(k_flash_rows, dim3((B + 255) / 256), dim3(256), 0, stream, lse, tgt, lo, A, B,
                     (float*)rowinfo);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_flash_dh(const float* pm, const float* pO, const void* rowinfo, int nsplit, const float* W,
                           float gscale, int B, int HF, float* dh, hipStream_t stream) {
  if (B <= 0 || nsplit <= 0 || HF <= 0 || !pm || !pO || !rowinfo || !W || !dh) return RG_ERR_ARG;
  hipLaunchKernelGGL(k_flash_dh, dim3((unsigned)(((int64_t)B * HF + 255) / 256)), dim3(256), 0, stream, pm, pO,
                     (const float*)rowinfo, nsplit, W, gscale, B, HF, dh);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_flash_dw_adam_planes(const void* Hk, const void* Hr, const void* Wk, const float* bias_pad,
                                       const void* rowinfo, float gscale, int B, int A, int HF, int terms, float* W,
                                       float* mW, float* vW, float* bias, float* mb, float* vb, const float* adam6,
                                       float* dW_out, float* db_out, void* Wk_out, void* Wr_out, float* bias_pad_out,
                                       void* work, int64_t work_bytes, const float* zs, hipStream_t stream) {
  if (B <= 0 || A <= 0 || (B % 32) || !Hk || !Hr || !Wk || !bias_pad || !rowinfo) return RG_ERR_ARG;
  if (!flash_terms_ok(terms)) return RG_ERR_ARG;
  if (!flash_hf_ok(HF)) return RG_ERR_SHAPE;
  if (dW_out ? !db_out : (!adam6 || !W || !mW || !vW || !bias || !mb || !vb)) return RG_ERR_ARG;
  if ((Wk_out != nullptr) != (Wr_out != nullptr) || (Wk_out && (dW_out || !bias_pad_out))) return RG_ERR_ARG;
  AdamArgs a{};
  if (adam6) a = AdamArgs{adam6[0], adam6[1], adam6[2], adam6[3], adam6[4], adam6[5]};
  const int rpb = fl_rows(HF, 2);
  FlTail tl = fl_tail(B, A, HF);
  if (tl.ntail && (int64_t)tl.tsplit * tl.ntail * (HF + 1) * 4 > (work ? work_bytes : 0)) tl = FlTail{(A + rpb - 1) / rpb, 1, 0};
  float* tail_dw = (float*)work;
  float* tail_db = tl.ntail ? tail_dw + (int64_t)tl.tsplit * tl.ntail * HF : nullptr;
  const int nblk = (A + rpb - 1) / rpb;
  const dim3 grid((unsigned)(tl.nfull + (nblk - tl.nfull) * tl.tsplit));
#define FW(HFV, NTV, ZLV)                                                                                     \
  hipLaunchKernelGGL((k_flash_dw<HFV, NTV, ZLV>), grid, dim3(64 * fl_nw(HFV, 2)), 0, stream, (const bf16x8*)Hk, \
                     (const bf16x8*)Hr, (const bf16x8*)Wk, bias_pad, (const float*)rowinfo, gscale, B, A, W, mW, vW, \
                     bias, mb, vb, a, dW_out, db_out, (bf16x8*)Wk_out, (bf16x8*)Wr_out, bias_pad_out, tl.nfull,    \
                     tl.tsplit, tail_dw, tail_db, zs)
#define FZ(HFV, NTV)               \
  if (zs) {                        \
    FW(HFV, NTV, true);            \
  } else {                         \
    FW(HFV, NTV, false);           \
  }
#define FT(HFV)          \
  if (terms == 9) {      \
    FZ(HFV, 9);          \
  } else {               \
    FZ(HFV, 6);          \
  }
  switch (HF) {
    case 32: FT(32); break;
    case 64: FT(64); break;
    case 128: FT(128); break;
    case 256: FT(256); break;
  }
#undef FT
#undef FZ
#undef FW
  if (tl.ntail) {
    const int i0 = tl.nfull * rpb;
    hipLaunchKernelGGL(k_flash_tail, dim3((unsigned)(((int64_t)tl.ntail * HF + 255) / 256)), dim3(256), 0, stream,
                       tail_dw, tail_db, tl.tsplit, i0, tl.ntail, HF, W, mW, vW, bias, mb, vb, a, dW_out, db_out);
    if (Wk_out && !dW_out) {   // the leftover rows' planes and padded bias, from the updated W / b
      const int ap = (A + 31) / 32 * 32;
      const float* Xs = W + (int64_t)i0 * HF;
      bf16x8* Pk = (bf16x8*)Wk_out + (int64_t)(i0 / 32) * (HF / 16) * 192;
      bf16x8* Pr = (bf16x8*)Wr_out + (int64_t)(i0 / 32) * (HF / 16) * 192;
      const int rows = A - i0, rp = ap - i0;
      const unsigned gk = (unsigned)(((int64_t)rp * (HF / 8) + 255) / 256);
      const unsigned gr = (unsigned)(((int64_t)(rp / 32) * (HF / 16) * 64 + 255) / 256);
#define PLT(HFV)                                                                                   \
  hipLaunchKernelGGL(k_planes_k<HFV>, dim3(gk), dim3(256), 0, stream, Xs, rows, rp, Pk);          \
  hipLaunchKernelGGL(k_planes_r<HFV>, dim3(gr), dim3(256), 0, stream, Xs, rows, rp, Pr)
      switch (HF) {
        case 32: PLT(32); break;
        case 64: PLT(64); break;
        case 128: PLT(128); break;
        case 256: PLT(256); break;
      }
#undef PLT
      hipLaunchKernelGGL(k_pad_bias, dim3((rp + 255) / 256), dim3(256), 0, stream, bias + i0, rows, rp,
                         bias_pad_out + i0);
    }
  }
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int64_t rg_flash_dw_work_bytes(int B, int A, int HF) {
  if (B <= 0 || A <= 0 || (B % 32) || !flash_hf_ok(HF)) return RG_ERR_ARG;
  const FlTail tl = fl_tail(B, A, HF);
  return (int64_t)tl.tsplit * tl.ntail * (HF + 1) * 4;
}

extern "C" int rg_flash_dw_adam(const void* Hk, const void* Hr, const void* Wk, const float* bias_pad,
                                const void* rowinfo, float gscale, int B, int A, int HF, int terms, float* W,
                                float* mW, float* vW, float* bias, float* mb, float* vb, const float* adam6,
                                float* dW_out, float* db_out, hipStream_t stream) {
  return rg_flash_dw_adam_planes(Hk, Hr, Wk, bias_pad, rowinfo, gscale, B, A, HF, terms, W, mW, vW, bias, mb, vb, adam6,
                                 dW_out, db_out, nullptr, nullptr, nullptr, nullptr, 0, nullptr, stream);
}

// Exact argmax through screening (the double-Q target of SQN / SMORL at the
// cost of 3 plane products — or 1 — instead of 6): k_flash_amax<NT = terms>
// leaves the per-split first maximum and every chunk's row maximum of the
// screened logits; the caller merges the former (rg_flash_argmax) and then
// rg_flash_argmax_exact re-scores, in fp32 (fmaf chain over k, + bias), every
// item of every chunk whose screened maximum lies within the error bound
// tol·||h_b||_2·max_a||W_a||_2 of the row's best, and keeps the first maximum.
// The bound on |z − z_screened| per item: 3 products drop terms of 2^-16
// |a||b| and smaller (≈ 3·2^-18 summed), 1 product keeps a0·b0 only:
// |ab − a0 b0| ≤ (2^-8 + 2^-18)|a||b| (RNE to bf16: |a − a0| ≤ 2^-9 |a|),
// so ≤ 3.91e-3·||h||·||W_a|| over k; the candidates need twice that (the
// screened best may itself be over-estimated) — the caller's tol.
extern "C" int rg_flash_amax_screen(const void* Hk, const void* Wk, const float* bias_pad, int B, int A, int HF,
                                    int nsplit, int terms, float* pbest, int32_t* parg, float* cmax,
                                    hipStream_t stream) {
  if (B <= 0 || A <= 0 || (B % 32) || nsplit <= 0 || (terms != 1 && terms != 3) || !Hk || !Wk || !bias_pad ||
      !pbest || !parg || !cmax)
    return RG_ERR_ARG;
  if (!flash_hf_ok(HF)) return RG_ERR_SHAPE;
  const int nct = (A + 31) / 32;
  const int cps = (nct + nsplit - 1) / nsplit;
  const int rpb = fl_rows(HF, 1);
  const int nrb = (B + rpb - 1) / rpb;
  const dim3 grid((unsigned)(nrb * nsplit));
#define FS1(HFV, NTV)                                                                                             \
  hipLaunchKernelGGL((k_flash_amax<HFV, NTV, true>), grid, dim3(64 * fl_nw(HFV, 1)), 0, stream, (const bf16x8*)Hk, \
                     (const bf16x8*)Wk, bias_pad, B, A, nrb, nsplit, cps, pbest, parg, cmax)
#define FS(HFV)      \
  if (terms == 1) {  \
    FS1(HFV, 1);     \
  } else {           \
    FS1(HFV, 3);     \
  }
  switch (HF) {
    case 32: FS(32); break;
    case 64: FS(64); break;
    case 128: FS(128); break;
    case 256: FS(256); break;
  }
#undef FS
#undef FS1
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_row_norm_max(const float* W, int64_t A, int HF, float* out, hipStream_t stream) {
  if (A <= 0 || HF <= 0 || HF > 256 || (HF % 4) || !W || !out) return RG_ERR_ARG;
  if (hipMemsetAsync(out, 0, sizeof(float), stream) != hipSuccess) return RG_ERR_LAUNCH;
  const int64_t blocks = (A + 7) / 8;
  hipLaunchKernelGGL(k_row_norm_max, dim3((unsigned)(blocks < 4096 ? blocks : 4096)), dim3(256), 0, stream, W, A, HF,
                     out);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_flash_argmax_exact(const float* cmax, int B, int A, const float* h, const float* W, const float* bias,
                                     int HF, const float* wnorm, float tol, float* lim, int32_t* cand, int32_t* ncand,
                                     int32_t* out_idx, float* out_val, int32_t* err, hipStream_t stream) {
  if (B <= 0 || A <= 0 || HF <= 0 || HF > 256 || (HF % 8)) return RG_ERR_ARG;
  if (!cmax || !h || !W || !bias || !wnorm || !lim || !cand || !ncand || !out_idx || !out_val) return RG_ERR_ARG;
  const int nct = (A + 31) / 32;
  if (hipMemsetAsync(ncand, 0, sizeof(int32_t) * B, stream) != hipSuccess) return RG_ERR_LAUNCH;
  hipLaunchKernelGGL(k_amax_lim, dim3((B + 255) / 256), dim3(256), 0, stream, out_val, h, B, HF, wnorm, tol, lim);
  const int ys = max(1, min(256, 2048 / ((B + 255) / 256)));   // ~2048 workgroups
  hipLaunchKernelGGL(k_amax_cand, dim3((B + 255) / 256, ys), dim3(256), 0, stream, cmax, nct, B, B, lim, cand,
                     ncand);
  hipLaunchKernelGGL(k_flash_topk_eval, dim3(B), dim3(256), 0, stream, h, W, bias, cand, ncand, A, HF, 1, out_idx,
                     out_val);
  // a row past the candidate cap: the first maximum of the whole fp32 row
  hipLaunchKernelGGL(k_flash_topk_scan, dim3(B), dim3(256), 0, stream, h, W, bias, ncand, A, HF, 1, out_idx, out_val,
                     err);
  RG_LAUNCH_CHECK();
  return RG_OK;
}
