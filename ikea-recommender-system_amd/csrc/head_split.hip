// Full-softmax output head on split-bf16 MFMAs (precision f32x9 / f32x6,
// csrc/common.h) — the same Zᵀ / partial contract as head.hip's
// rg_head_fwd (reference GRU4Rec/model.py:58-60,80,121).
//
// Every fp32 operand x is split exactly into three bf16 planes x0+x1+x2; a
// product is Σ a_p·b_q over 9 (exact products, fp32 accumulation) or 6 plane
// pairs (the three sub-ulp terms dropped) on v_mfma_f32_32x32x16_bf16, which
// runs 16× the fp32 MFMA rate: 9/16 resp. 6/16 of the f32 MFMA time.
//
//  k_split_rows   : rows of h (B × HF) → fragment-order planes
//                   [32-row block][k slice][plane][lane] × 16 B (once per
//                   call; 1.5× the bytes of h).
//  k_head_fwd_x   : a workgroup owns NW·32 items; wave w holds the planes of
//                   its 32 W rows in VGPRs (split once in the prologue) and
//                   streams every 32-row chunk of h's planes through a
//                   double-buffered LDS ring (whole 1 KB fragments, one
//                   barrier per chunk).  Chunks alternate two accumulator
//                   sets so the Zᵀ stores of chunk c drain under chunk c+1's
//                   MFMAs.  Epilogue: bias, Zᵀ store, online (max, Σexp,
//                   argmax) per (32-item block, row) — RG_PBLK partials,
//                   ties to the lower item index, exactly as rg_head_fwd.
#include "common.h"

#define NEG_INF (-__builtin_inff())

// merge of two lane halves' (max, Σexp, argmax); ties to the lower index;
// an empty half has arg INT32_MAX
__device__ __forceinline__ void stat_merge_x(float& m, float& s, int& a, float m2, float s2, int a2) {
  if (a2 == INT32_MAX) return;
  if (a == INT32_MAX) {
    m = m2;
    s = s2;
    a = a2;
    return;
  }
  if (m2 > m || (m2 == m && a2 < a)) {
    s = s * __expf(m - m2) + s2;
    m = m2;
    a = a2;
  } else {
    s = s + s2 * __expf(m2 - m);
  }
}

// ------------------------------------------------------------ planes ----
// One thread per (row, 8-value group); threads of one row read consecutive
// 32 B of it.  Plane entry (block x/32, slice g/2, plane p, lane (g&1)·32 + x%32).
template <int HF>
__global__ __launch_bounds__(256) void k_split_rows(const float* __restrict__ X, int rows,
                                                    bf16x8* __restrict__ P) {
  constexpr int G = HF / 8;
  constexpr int NS = HF / 16;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)rows * G) return;
  const int x = (int)(i / G), g = (int)(i % G);
  const float* src = X + (int64_t)x * HF + 8 * g;
  const f4 lo = *reinterpret_cast<const f4*>(src);
  const f4 hi = *reinterpret_cast<const f4*>(src + 4);
  bf16x8 p0, p1, p2;
  split3x8(lo, hi, p0, p1, p2);
  const int lane = (g & 1) * 32 + (x & 31);
  const int64_t base = ((int64_t)(x >> 5) * NS + (g >> 1)) * 3 * 64 + lane;
  P[base] = p0;
  P[base + 64] = p1;
  P[base + 128] = p2;
}

// ---------------------------------------------------------------- fwd ----
#define HX_WAVES_OF(HF) ((HF) >= 256 ? 4 : 8)

template <int HF, int NT, bool SZ, bool WS>
__global__ __launch_bounds__(64 * HX_WAVES_OF(HF)) void k_head_fwd_x(const bf16x8* __restrict__ Hp,
                                                                     const float* __restrict__ W,
                                                                     const float* __restrict__ bias, int B, int A,
                                                                     float* __restrict__ ZT, int64_t ldz,
                                                                     float* __restrict__ pmax,
                                                                     float* __restrict__ psum,
                                                                     int32_t* __restrict__ parg, int rpb) {
  constexpr int NW = HX_WAVES_OF(HF);
  constexpr int NS = HF / 16;
  constexpr int NE = NS * 3 * 64;  // 16-B fragments per 32-row chunk
  constexpr int EPT = (NE + 64 * NW - 1) / (64 * NW);
  constexpr float L2E = 1.4426950408889634f;
  __shared__ bf16x8 hs[2][3][NS][2][32];
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, half = lane >> 5, l32 = lane & 31;
  const int jw = blockIdx.x * (32 * NW) + 32 * w;
  const bool active = jw < A;
  const bool full = jw + 32 <= A;
  // rows [rbase, rbase + 32·nch) of this workgroup (grid.y splits B so that a
  // small A — a sampled head's negatives — still fills the chip)
  const int rbase = blockIdx.y * rpb;
  const int nch = min(rpb, B - rbase) / 32;  // B, rpb % 32 == 0
  const bf16x8* __restrict__ Hb = Hp + (int64_t)(rbase / 32) * NE;
  // chunk 0's fragments first (independent of W), then this wave's W rows
  bf16x8 st[EPT];
  // the scheduling barrier keeps the prefetch at the top of the chunk (left
  // to itself the compiler sinks it next to its LDS commit, which exposes
  // the full L2 latency every chunk)
  auto load_chunk = [&](int c) __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < EPT; ++q) {
      const int e = tid + 64 * NW * q;
      if (e < NE) st[q] = Hb[(int64_t)c * NE + e];
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  auto store_chunk = [&](int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < EPT; ++q) {
      const int e = tid + 64 * NW * q;
      if (e < NE) {
        const int j = e / 192, p = (e / 64) % 3, ln = e & 63;
        hs[buf][p][j][ln >> 5][ln & 31] = st[q];
      }
    }
  };
  load_chunk(0);
  bf16x8 a0[NS], a1[NS], a2[NS];
  float bj[16];
  {
    const int jr = jw + l32;
    f4 wl[NS][2];
    const bool ok = jr < A;
    const float* src = W + (int64_t)(ok ? jr : 0) * HF + 8 * half;
#pragma unroll
    for (int j = 0; j < NS; ++j) {
      wl[j][0] = ok ? *reinterpret_cast<const f4*>(src + 16 * j) : f4{0.f, 0.f, 0.f, 0.f};
      wl[j][1] = ok ? *reinterpret_cast<const f4*>(src + 16 * j + 4) : f4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {  // items past A: z = 0 + (−inf), dropped everywhere below
      const int j = jw + acc32_row(r, half);
      bj[r] = j < A ? bias[j] : NEG_INF;
    }
    store_chunk(0);
#pragma unroll
    for (int j = 0; j < NS; ++j) split3x8(wl[j][0], wl[j][1], a0[j], a1[j], a2[j]);
  }
  __syncthreads();
  float* pm = pmax + (int64_t)(jw / RG_PBLK) * B + rbase + l32;
  float* ps = WS ? psum + (int64_t)(jw / RG_PBLK) * B + rbase + l32 : nullptr;
  int32_t* pa = parg ? parg + (int64_t)(jw / RG_PBLK) * B + rbase + l32 : nullptr;
  // Zᵀ stores through a buffer descriptor over this wave's item rows that
  // exist: stores of items past A fall outside num_records and are dropped,
  // so the epilogue has no per-lane branch (the stores sit between MFMAs)
  const int nrows = active ? min(32, A - jw) : 0;
  const uint64_t zb = SZ ? (uint64_t)(ZT + (int64_t)(active ? jw : 0) * ldz) : 0;
  const uint32_t zlo = __builtin_amdgcn_readfirstlane((uint32_t)zb);
  const uint32_t zhi = __builtin_amdgcn_readfirstlane((uint32_t)(zb >> 32));
  const uint32_t znb = __builtin_amdgcn_readfirstlane(SZ ? (uint32_t)(nrows * ldz * 4) : 0u);
  const __amdgpu_buffer_rsrc_t zrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)zhi << 32) | zlo), 0, znb, 0x00020000);
  const int zlane = (4 * half * (int)ldz + l32) * 4;  // bytes
  const int zrow4 = __builtin_amdgcn_readfirstlane((int)ldz * 4);
  // Epilogue of a finished chunk, sliced over the NS MFMA groups of the next
  // chunk: slices [0, NS/2) take PER values each (bias, Zᵀ store, max /
  // argmax), slices [NS/2, NS) the Σexp; epi_finish merges the lane halves
  // and writes the partial.  Branch-free: missing items carry z = −inf.
  constexpr int PER = NS >= 32 ? 1 : 32 / NS;
  float em = NEG_INF, es = 0.f;
  int ea = INT32_MAX;
  auto epi_slice = [&](f16v& acc, int cc, int j) __attribute__((always_inline)) {
    if (j < NS / 2) {
#pragma unroll
      for (int q = 0; q < PER; ++q) {
        const int r = j * PER + q;
        if (r < 16) {
          const float z = acc[r] + bj[r];
          acc[r] = z;
          if (SZ)
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(z), zrs, zlane,
                                                  ((r & 3) + 8 * (r >> 2)) * zrow4 + (rbase + 32 * cc) * 4, 0);
          const bool gt = z > em;
          em = gt ? z : em;
          ea = gt ? jw + acc32_row(r, half) : ea;
        }
      }
    } else if (WS) {
      const float m2 = em == NEG_INF ? 0.f : em * L2E;
#pragma unroll
      for (int q = 0; q < PER; ++q) {
        const int r = (j - NS / 2) * PER + q;
        if (r < 16) es += __builtin_amdgcn_exp2f(fmaf(acc[r], L2E, -m2));
      }
    }
  };
  auto epi_finish = [&](int cc) __attribute__((always_inline)) {
    stat_merge_x(em, es, ea, __shfl_xor(em, 32), __shfl_xor(es, 32), __shfl_xor(ea, 32));
    if (half == 0) {
      pm[cc * 32] = em;
      if (WS) ps[cc * 32] = es;
      if (pa) pa[cc * 32] = ea;
    }
    em = NEG_INF;
    es = 0.f;
    ea = INT32_MAX;
  };
  // MFMAs of the chunk in LDS buffer `buf` into acc, carrying the epilogue
  // slices of the previous chunk (prev, cprev) when epi
  auto chunk = [&](int buf, f16v& acc, f16v& prev, int cprev, bool epi) __attribute__((always_inline)) {
    acc = f16v{};
#pragma unroll
    for (int j = 0; j < NS; ++j) {
      const bf16x8 b0 = hs[buf][0][j][half][l32];
      const bf16x8 b1 = hs[buf][1][j][half][l32];
      const bf16x8 b2 = hs[buf][2][j][half][l32];
      acc = mfma_split<NT>(a0[j], a1[j], a2[j], b0, b1, b2, acc);
      if (epi) epi_slice(prev, cprev, j);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  f16v accA = {}, accB = {};
  // chunk 0 -> accA (buffer 0)
  if (nch > 1) load_chunk(1);
  if (active) chunk(0, accA, accB, 0, false);
  if (nch > 1) store_chunk(1);
  __syncthreads();
  int c = 1;
  for (; c + 1 < nch; c += 2) {
    // chunk c -> accB (buffer 1), epilogue of c-1 (accA)
    load_chunk(c + 1);
    if (active) {
      chunk(1, accB, accA, c - 1, true);
      epi_finish(c - 1);
    }
    store_chunk(0);
    __syncthreads();
    // chunk c+1 -> accA (buffer 0), epilogue of c (accB)
    const bool more = c + 2 < nch;
    if (more) load_chunk(c + 2);
    if (active) {
      chunk(0, accA, accB, c, true);
      epi_finish(c);
    }
    if (more) store_chunk(1);
    __syncthreads();
  }
  if (active) {
    if (c < nch) {  // last chunk c sits in buffer 1
      chunk(1, accB, accA, c - 1, true);
      epi_finish(c - 1);
#pragma unroll
      for (int j = 0; j < NS; ++j) epi_slice(accB, c, j);
      epi_finish(c);
    } else {
#pragma unroll
      for (int j = 0; j < NS; ++j) epi_slice(accA, c - 1, j);
      epi_finish(c - 1);
    }
  }
}

// bytes of scratch rg_head_fwd_x needs (h's planes)
extern "C" int64_t rg_head_work_bytes(int B, int HF) {
  if (B <= 0 || HF <= 0) return RG_ERR_ARG;
  return (int64_t)B * HF * 6;
}

// rg_head_fwd on split-bf16 MFMAs (terms 9 / 6) from h's planes (k_split_rows
// layout).  Same outputs (Zᵀ, per (RG_PBLK items, row) max / Σexp / argmax
// partials; parg optional); rpb = rows per workgroup (multiple of 32; B for
// one row block, less to spread a small A over the chip).  B % 32 == 0.
extern "C" int rg_head_fwd_xp(const void* hplanes, const float* W, const float* bias, int B, int A, int HF,
                              int terms, int rpb, float* ZT, int64_t ldz, float* pmax, float* psum, int32_t* parg,
                              int want_sum, hipStream_t stream) {
  if (B <= 0 || A <= 0 || (B % 32) || rpb <= 0 || (rpb % 32) || hplanes == nullptr) return RG_ERR_ARG;
  if (ZT && ldz < B) return RG_ERR_ARG;
  if (want_sum && psum == nullptr) return RG_ERR_ARG;
  if (terms != 6 && terms != 9) return RG_ERR_ARG;
  const bf16x8* Hp = reinterpret_cast<const bf16x8*>(hplanes);
  const int nw = HX_WAVES_OF(HF);
  const dim3 gf((A + 32 * nw - 1) / (32 * nw), (B + rpb - 1) / rpb);
#define HXL(HFV, NTV, SZV, WSV)                                                                                \
  hipLaunchKernelGGL((k_head_fwd_x<HFV, NTV, SZV, WSV>), gf, dim3(64 * nw), 0, stream, Hp, W, bias, B, A, ZT, \
                     ldz, pmax, psum, parg, rpb)
#define HXT(HFV, NTV)                          \
  if (ZT && want_sum) HXL(HFV, NTV, true, true); \
  else if (ZT) HXL(HFV, NTV, true, false);       \
  else if (want_sum) HXL(HFV, NTV, false, true); \
  else HXL(HFV, NTV, false, false);
#define HXH(HFV)  \
  if (terms == 9) { \
    HXT(HFV, 9)   \
  } else {        \
    HXT(HFV, 6)   \
  }
  switch (HF) {
    case 32: HXH(32); break;
    case 64: HXH(64); break;
    case 128: HXH(128); break;
    case 256: HXH(256); break;
    default: return RG_ERR_SHAPE;
  }
#undef HXH
#undef HXT
#undef HXL
  RG_LAUNCH_CHECK();
  return RG_OK;
}

// rg_head_fwd on split-bf16 MFMAs (terms 9 / 6).  Same outputs (Zᵀ, per
// (RG_PBLK items, row) max / Σexp / argmax partials); B % 32 == 0.
extern "C" int rg_head_fwd_x(const float* h, const float* W, const float* bias, int B, int A, int HF, int terms,
                             float* ZT, int64_t ldz, float* pmax, float* psum, int32_t* parg, int want_sum,
                             void* work, hipStream_t stream) {
  if (B <= 0 || A <= 0 || (B % 32) || work == nullptr) return RG_ERR_ARG;
  if (terms != 6 && terms != 9) return RG_ERR_ARG;
  bf16x8* Hp = reinterpret_cast<bf16x8*>(work);
  const dim3 gs((unsigned)(((int64_t)B * (HF / 8) + 255) / 256));
  switch (HF) {
    case 32: hipLaunchKernelGGL(k_split_rows<32>, gs, dim3(256), 0, stream, h, B, Hp); break;
    case 64: hipLaunchKernelGGL(k_split_rows<64>, gs, dim3(256), 0, stream, h, B, Hp); break;
    case 128: hipLaunchKernelGGL(k_split_rows<128>, gs, dim3(256), 0, stream, h, B, Hp); break;
    case 256: hipLaunchKernelGGL(k_split_rows<256>, gs, dim3(256), 0, stream, h, B, Hp); break;
    default: return RG_ERR_SHAPE;
  }
  return rg_head_fwd_xp(Hp, W, bias, B, A, HF, terms, B, ZT, ldz, pmax, psum, parg, want_sum, stream);
}
