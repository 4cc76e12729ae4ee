// Full-softmax output head (SURVEY §8 A6, A7, A8-for-the-head, A14 argmax).
//
// Reference: Z = h·Wᵀ + b (nn.Linear(H→A), GRU4Rec/model.py:58-60,80),
// loss = CrossEntropyLoss(mean)(Z, a) (:121,146), dense Adam step (:149-153).
//
// Layout choice: logits are kept TRANSPOSED, Zᵀ[j][b] (A × ldz, ldz ≥ B), so
// every store and every re-read in backward is a run of consecutive batch
// rows (128-B segments per half-wave) — the MFMA D layout writes columns, and
// both backward GEMMs stream Zᵀ rows.
//
//  k_head_fwd_w1: Zᵀ tile = W_tile · h_chunkᵀ on v_mfma_f32_32x32x2_f32, one
//                 wave per 32 items with the W rows resident in VGPRs (64
//                 regs/lane at HF=128) and h streamed from L2 into registers;
//                 the epilogue (bias, Zᵀ stores, per-(32-item block, row)
//                 online (max, Σexp, argmax) partials) of each 32-row chunk is
//                 interleaved with the next chunk's MFMAs — the softmax never
//                 re-reads Zᵀ.  k_head_fwd: the same with h staged through LDS
//                 for 4 waves, used for the remainder items and ragged B.
//  k_lse_*      : merge partials -> lse[b], argmax[b], loss_b = lse_b − Z[a_b,b].
//  k_head_dh    : dh = dZ·W, dZ = (exp(Z−lse) − onehot)·g recomputed on load;
//                 split over the item axis into deterministic slabs.
//  k_head_dw_adam: dW = dZᵀ·h and db = Σ_b dZ for a 128-item tile, accumulated
//                 over all rows in VGPRs, then the Adam update of those W/b rows
//                 in the same kernel (no gradient tensor ever reaches HBM).
#include "common.h"

#define NEG_INF (-__builtin_inff())

__device__ __forceinline__ void stat_merge(float& m, float& s, int& a, float m2, float s2, int a2) {
  if (a2 == INT32_MAX) return;  // empty partial
  if (a == INT32_MAX) {
    m = m2;
    s = s2;
    a = a2;
    return;
  }
  if (m2 > m || (m2 == m && a2 < a)) {
    s = s * expf(m - m2) + s2;
    m = m2;
    a = a2;
  } else {
    s = s + s2 * expf(m2 - m);
  }
}

// ------------------------------------------------------------------ fwd ----
template <int HF>
__global__ __launch_bounds__(256) void k_head_fwd(const float* __restrict__ h, const float* __restrict__ W,
                                                  const float* __restrict__ bias, int B, int A,
                                                  float* __restrict__ ZT, int64_t ldz, float* __restrict__ pmax,
                                                  float* __restrict__ psum, int32_t* __restrict__ parg,
                                                  int want_sum, int j0) {
  constexpr int KH = HF / 2;
  constexpr int LDB = HF + 4;
  constexpr int NV = 8 * HF;                 // float4 per 32-row chunk
  constexpr int NL = (NV + 255) / 256;       // float4 per thread per chunk
  __shared__ __attribute__((aligned(16))) float hbuf[2][32][LDB];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, half = lane >> 5, l32 = lane & 31;
  const int jw = j0 + blockIdx.x * 128 + 32 * w;  // this wave's 32 items = one partial block

  float Wreg[KH];
  {
    const int jr = jw + l32;
    if (jr < A) {
      const float* src = W + (int64_t)jr * HF + half * KH;
#pragma unroll
      for (int s = 0; s < KH; s += 4) {
        f4 v = *reinterpret_cast<const f4*>(src + s);
        Wreg[s] = v.x;
        Wreg[s + 1] = v.y;
        Wreg[s + 2] = v.z;
        Wreg[s + 3] = v.w;
      }
    } else {
#pragma unroll
      for (int s = 0; s < KH; ++s) Wreg[s] = 0.f;
    }
  }
  float bj[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    int j = jw + acc32_row(r, half);
    bj[r] = (j < A) ? bias[j] : 0.f;
  }
  const int nch = (B + 31) / 32;
  f4 pre[NL];
  float keep[NL];
  auto load_chunk = [&](int c) {
    // branch-free: clamp the row and zero it when committing to LDS, so the
    // loads stay in flight across the MFMA phase
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int e = tid + 256 * i;
      const int rr = (e < NV ? e : 0) / (HF / 4), c4 = e % (HF / 4);
      const int b = c * 32 + rr;
      const int bc = b < B ? b : B - 1;
      pre[i] = *reinterpret_cast<const f4*>(h + (int64_t)bc * HF + 4 * c4);
      keep[i] = (e < NV && b < B) ? 1.f : 0.f;
    }
  };
  auto store_chunk = [&](int buf) {
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      int e = tid + 256 * i;
      if (e < NV) {
        int rr = e / (HF / 4), c4 = e % (HF / 4);
        *reinterpret_cast<f4*>(&hbuf[buf][rr][4 * c4]) = pre[i] * keep[i];
      }
    }
  };
  load_chunk(0);
  store_chunk(0);
  __syncthreads();
  int cur = 0;
  for (int c = 0; c < nch; ++c) {
    if (c + 1 < nch) load_chunk(c + 1);
    f16v acc = {};
    const float* hb = &hbuf[cur][l32][half * KH];
    // LDS reads run one 4-MFMA group ahead of their use (pinned by a
    // scheduling barrier) so their latency hides under the MFMAs in flight:
    // −1.7 % kernel time at C2 (tools/ab_head.sh); the same change in the
    // backward kernels measured neutral (dh) or slower (dW) and is not used.
    f4 hv = *reinterpret_cast<const f4*>(hb);
#pragma unroll
    for (int s = 0; s < KH; s += 4) {
      f4 hn = hv;
      if (s + 4 < KH) hn = *reinterpret_cast<const f4*>(hb + s + 4);
      acc = mfma32(Wreg[s], hv.x, acc);
      acc = mfma32(Wreg[s + 1], hv.y, acc);
      acc = mfma32(Wreg[s + 2], hv.z, acc);
      acc = mfma32(Wreg[s + 3], hv.w, acc);
      hv = hn;
      __builtin_amdgcn_sched_barrier(0);
    }
    // Commit the prefetched chunk to LDS before this chunk's Zᵀ stores are
    // issued: vmcnt counts loads and stores in issue order, so waiting for the
    // prefetch after the stores would stall the wave until the stores retire.
    if (c + 1 < nch) store_chunk(cur ^ 1);
    const int b = c * 32 + l32;
    const bool bv = b < B;
    float m = NEG_INF, sum = 0.f;
    int arg = INT32_MAX;
    if (jw + 32 <= A) {  // wave-uniform: every item row of this wave exists
      if (ZT && bv) {
        float* zc = ZT + b;
#pragma unroll
        for (int r = 0; r < 16; ++r) zc[(int64_t)(jw + acc32_row(r, half)) * ldz] = acc[r] + bj[r];
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float z = acc[r] + bj[r];
        acc[r] = z;
        const bool gt = z > m;
        m = gt ? z : m;
        arg = gt ? jw + acc32_row(r, half) : arg;
      }
      if (want_sum) {
        const float m2 = m * 1.4426950408889634f;
#pragma unroll
        for (int r = 0; r < 16; ++r) sum += __builtin_amdgcn_exp2f(fmaf(acc[r], 1.4426950408889634f, -m2));
      }
    } else {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int j = jw + acc32_row(r, half);
        const float z = acc[r] + bj[r];
        acc[r] = z;
        if (j < A) {
          if (ZT && bv) ZT[(int64_t)j * ldz + b] = z;
          if (z > m) {
            m = z;
            arg = j;
          }
        }
      }
      if (want_sum && arg != INT32_MAX) {
        const float m2 = m * 1.4426950408889634f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int j = jw + acc32_row(r, half);
          if (j < A) sum += __builtin_amdgcn_exp2f(fmaf(acc[r], 1.4426950408889634f, -m2));
        }
      }
    }
    {
      float m2 = __shfl_xor(m, 32);
      float s2 = __shfl_xor(sum, 32);
      int a2 = __shfl_xor(arg, 32);
      stat_merge(m, sum, arg, m2, s2, a2);
    }
    if (half == 0 && bv && jw < A) {  // one partial per 32-item block (RG_PBLK)
      const int64_t o = (int64_t)(jw / RG_PBLK) * B + b;
      pmax[o] = m;
      if (psum) psum[o] = sum;
      parg[o] = arg;
    }
    __syncthreads();
    cur ^= 1;
  }
}

// Interior fast path: one wave per 32 items (every item exists, B % 32 == 0).
// W rows stay in VGPRs; h is streamed straight from L2 into registers through
// a 4-group prefetch ring (no LDS, no barriers — nothing couples the waves),
// and the epilogue of chunk c−1 (bias, Zᵀ stores, max/argmax, Σexp, the
// per-block partial) is interleaved in program order with the MFMAs of chunk
// c, two accumulator sets alternating.  Same arithmetic and tie rules as
// k_head_fwd.
template <int HF, bool SZ, bool WS>
__global__ __launch_bounds__(64) void k_head_fwd_w1(const float* __restrict__ h, const float* __restrict__ W,
                                                    const float* __restrict__ bias, int B,
                                                    float* __restrict__ ZT, int64_t ldz,
                                                    float* __restrict__ pmax, float* __restrict__ psum,
                                                    int32_t* __restrict__ parg) {
  constexpr int KH = HF / 2;
  constexpr int NG = KH / 4;                   // 4-MFMA groups per 32-row chunk
  constexpr int PD = NG < 4 ? NG : 4;          // h prefetch distance in groups
  constexpr int PER = NG >= 32 ? 1 : 32 / NG;  // epilogue values per group (two passes over 16)
  constexpr float L2E = 1.4426950408889634f;
  const int lane = threadIdx.x, half = lane >> 5, l32 = lane & 31;
  const int jw = blockIdx.x * 32;
  float Wreg[KH];
  {
    const float* src = W + (int64_t)(jw + l32) * HF + half * KH;
#pragma unroll
    for (int s = 0; s < KH; s += 4) {
      const f4 v = *reinterpret_cast<const f4*>(src + s);
      Wreg[s] = v.x;
      Wreg[s + 1] = v.y;
      Wreg[s + 2] = v.z;
      Wreg[s + 3] = v.w;
    }
  }
  float bj[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) bj[r] = bias[jw + acc32_row(r, half)];
  // Zᵀ stores through a buffer descriptor over the 32 item rows (wave-uniform
  // base, scalar row offsets): one 32-bit lane offset serves all 16 rows
  const uint64_t zb = SZ ? (uint64_t)(ZT + (int64_t)jw * ldz) : 0;
  const uint32_t zlo = __builtin_amdgcn_readfirstlane((uint32_t)zb);
  const uint32_t zhi = __builtin_amdgcn_readfirstlane((uint32_t)(zb >> 32));
  const uint32_t znb = __builtin_amdgcn_readfirstlane(SZ ? (uint32_t)(32 * ldz * 4) : 0u);
  const __amdgpu_buffer_rsrc_t zrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)zhi << 32) | zlo), 0, znb, 0x00020000);
  const int zlane = (4 * half * (int)ldz + l32) * 4;  // bytes
  const int zrow4 = __builtin_amdgcn_readfirstlane((int)ldz * 4);
  const int nch = B / 32;
  const float* hl = h + (int64_t)l32 * HF + half * KH;  // + chunk·32·HF + 4·group
  float* pm = pmax + (int64_t)blockIdx.x * B + l32;
  float* ps = WS ? psum + (int64_t)blockIdx.x * B + l32 : nullptr;
  int32_t* pa = parg + (int64_t)blockIdx.x * B + l32;
  f4 ring[PD];
#pragma unroll
  for (int p = 0; p < PD; ++p) ring[p] = *reinterpret_cast<const f4*>(hl + 4 * p);
  float em = NEG_INF, es = 0.f;
  int ea = INT32_MAX;
  auto epi_slice = [&](f16v& acc, int cc, int g) __attribute__((always_inline)) {
    if (g < NG / 2) {
#pragma unroll
      for (int q = 0; q < PER; ++q) {
        const int r = g * PER + q;
        if (r < 16) {
          const float z = acc[r] + bj[r];
          acc[r] = z;
          if (SZ)
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(z), zrs, zlane,
                                                  ((r & 3) + 8 * (r >> 2)) * zrow4 + cc * 128, 0);
          const bool gt = z > em;
          em = gt ? z : em;
          ea = gt ? jw + acc32_row(r, half) : ea;
        }
      }
    } else if (WS) {
      const float m2 = em * L2E;
#pragma unroll
      for (int q = 0; q < PER; ++q) {
        const int r = (g - NG / 2) * PER + q;
        if (r < 16) es += __builtin_amdgcn_exp2f(fmaf(acc[r], L2E, -m2));
      }
    }
  };
  auto epi_finish = [&](int cc) __attribute__((always_inline)) {
    stat_merge(em, es, ea, __shfl_xor(em, 32), __shfl_xor(es, 32), __shfl_xor(ea, 32));
    if (half == 0) {
      pm[cc * 32] = em;
      if (WS) ps[cc * 32] = es;
      pa[cc * 32] = ea;
    }
    em = NEG_INF;
    es = 0.f;
    ea = INT32_MAX;
  };
  // MFMAs of chunk c into acc; group g consumes ring[g % PD] and refills it
  // with group g + PD (possibly of chunk c + 1; clamped past the end)
  auto chunk = [&](int c, f16v& acc, f16v& prev, int cprev, bool epi) __attribute__((always_inline)) {
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      const f4 hv = ring[g % PD];
      {
        const int gg = g + PD;
        const int cn = gg < NG ? c : (c + 1 < nch ? c + 1 : c);
        const int gl = gg < NG ? gg : gg - NG;
        ring[g % PD] = *reinterpret_cast<const f4*>(hl + (int64_t)cn * 32 * HF + 4 * gl);
      }
      acc = mfma32(Wreg[4 * g], hv.x, acc);
      if (epi) epi_slice(prev, cprev, g);
      acc = mfma32(Wreg[4 * g + 1], hv.y, acc);
      acc = mfma32(Wreg[4 * g + 2], hv.z, acc);
      acc = mfma32(Wreg[4 * g + 3], hv.w, acc);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  f16v accA = {}, accB = {};
  chunk(0, accA, accB, 0, false);
  int c = 1;
  for (; c + 1 < nch; c += 2) {
    accB = f16v{};
    chunk(c, accB, accA, c - 1, true);
    epi_finish(c - 1);
    accA = f16v{};
    chunk(c + 1, accA, accB, c, true);
    epi_finish(c);
  }
  if (c < nch) {  // one chunk left: its MFMAs carry the epilogue of chunk c−1
    accB = f16v{};
    chunk(c, accB, accA, c - 1, true);
    epi_finish(c - 1);
#pragma unroll
    for (int g = 0; g < NG; ++g) epi_slice(accB, c, g);
    epi_finish(c);
  } else {
#pragma unroll
    for (int g = 0; g < NG; ++g) epi_slice(accA, c - 1, g);
    epi_finish(c - 1);
  }
}

extern "C" int rg_head_fwd(const float* h, const float* W, const float* bias, int B, int A, int HF, float* ZT,
                           int64_t ldz, float* pmax, float* psum, int32_t* parg, int want_sum, hipStream_t stream) {
  if (B <= 0 || A <= 0) return RG_ERR_ARG;
  if (ZT && ldz < B) return RG_ERR_ARG;
  if (HF != 16 && HF != 32 && HF != 64 && HF != 128 && HF != 256) return RG_ERR_SHAPE;
  // whole 32-item blocks through the single-wave kernel when every 32-row
  // chunk is full; the remainder items (and ragged B) through the generic one
  const bool fast = (B % 32) == 0 && (want_sum ? psum != nullptr : true);
  const int nfull = fast ? A / RG_PBLK : 0;
  const int j0 = nfull * RG_PBLK;
  if (nfull > 0) {
#define PL(HFV, SZV, WSV)                                                                                        \
  hipLaunchKernelGGL((k_head_fwd_w1<HFV, SZV, WSV>), dim3(nfull), dim3(64), 0, stream, h, W, bias, B, ZT, ldz, \
                     pmax, psum, parg)
#define PH(HFV)                            \
  if (ZT && want_sum) PL(HFV, true, true); \
  else if (ZT) PL(HFV, true, false);       \
  else if (want_sum) PL(HFV, false, true); \
  else PL(HFV, false, false);
    switch (HF) {
      case 16: PH(16); break;
      case 32: PH(32); break;
      case 64: PH(64); break;
      case 128: PH(128); break;
      case 256: PH(256); break;
    }
#undef PH
#undef PL
  }
  if (j0 < A) {
    const int ntail = (A - j0 + 127) / 128;
#define HL(HFV)                                                                                                 \
  hipLaunchKernelGGL(k_head_fwd<HFV>, dim3(ntail), dim3(256), 0, stream, h, W, bias, B, A, ZT, ldz, pmax, psum, \
                     parg, want_sum, j0)
    switch (HF) {
      case 16: HL(16); break;
      case 32: HL(32); break;
      case 64: HL(64); break;
      case 128: HL(128); break;
      case 256: HL(256); break;
    }
#undef HL
  }
  RG_LAUNCH_CHECK();
  return RG_OK;
}

// --------------------------------------------------------- lse combine ----
// stage 1: split the nJ partials of each row into S groups.  Four partials
// per iteration are loaded before any is merged (the merge chain is serial).
__global__ void k_lse_stage1(const float* __restrict__ pmax, const float* __restrict__ psum,
                             const int32_t* __restrict__ parg, int B, int nJ, int jchunk, float* __restrict__ omax,
                             float* __restrict__ osum, int32_t* __restrict__ oarg) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const int z = blockIdx.y;
  const int j0 = z * jchunk, j1 = min(nJ, j0 + jchunk);
  float m = NEG_INF, s = 0.f;
  int a = INT32_MAX;
  int j = j0;
  for (; j + 4 <= j1; j += 4) {
    float mv[4], sv[4];
    int av[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int64_t o = (int64_t)(j + q) * B + b;
      mv[q] = pmax[o];
      sv[q] = psum ? psum[o] : 0.f;
      av[q] = parg[o];
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) stat_merge(m, s, a, mv[q], sv[q], av[q]);
  }
  for (; j < j1; ++j) {
    const int64_t o = (int64_t)j * B + b;
    stat_merge(m, s, a, pmax[o], psum ? psum[o] : 0.f, parg[o]);
  }
  const int64_t o = (int64_t)z * B + b;
  omax[o] = m;
  osum[o] = s;
  oarg[o] = a;
}

// stage 2: lse[b], argmax[b], and (when ZT/tgt are given) loss_b = lse_b − Zᵀ[a_b][b].
__global__ void k_lse_final(const float* __restrict__ omax, const float* __restrict__ osum,
                            const int32_t* __restrict__ oarg, int B, int S, const float* __restrict__ ZT,
                            int64_t ldz, const int64_t* __restrict__ tgt, int A, float* __restrict__ lse,
                            int32_t* __restrict__ amax, float* __restrict__ loss_row, float* __restrict__ mx) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  float m = NEG_INF, s = 0.f;
  int a = INT32_MAX;
  for (int z = 0; z < S; ++z) {
    const int64_t o = (int64_t)z * B + b;
    stat_merge(m, s, a, omax[o], osum[o], oarg[o]);
  }
  const float l = m + logf(s);
  if (lse) lse[b] = l;
  if (amax) amax[b] = a;
  if (mx) mx[b] = m;  // the row maximum itself (exact logit value)
  if (loss_row && ZT && tgt) {
    const int64_t t = tgt[b];  // CrossEntropyLoss raises on out-of-range targets
    loss_row[b] = (t >= 0 && t < A) ? l - ZT[t * ldz + b] : __builtin_nanf("");
  }
}

extern "C" int rg_lse_combine(const float* pmax, const float* psum, const int32_t* parg, int B, int nJ,
                              float* work, const float* ZT, int64_t ldz, const int64_t* tgt, int A, float* lse,
                              int32_t* amax, float* loss_row, float* mx, hipStream_t stream) {
  if (B <= 0 || nJ <= 0) return RG_ERR_ARG;
  int S = 128;
  if (S > nJ) S = nJ;
  int jchunk = (nJ + S - 1) / S;
  S = (nJ + jchunk - 1) / jchunk;
  float* omax = work;
  float* osum = work + (int64_t)S * B;
  int32_t* oarg = reinterpret_cast<int32_t*>(work + 2 * (int64_t)S * B);
  hipLaunchKernelGGL(k_lse_stage1, dim3((B + 255) / 256, S), dim3(256), 0, stream, pmax, psum, parg, B, nJ, jchunk,
                     omax, osum, oarg);
  hipLaunchKernelGGL(k_lse_final, dim3((B + 255) / 256), dim3(256), 0, stream, omax, osum, oarg, B, S, ZT, ldz,
                     tgt, A, lse, amax, loss_row, mx);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

// out[0] = (Σ x[i]) · scale  (one workgroup, fixed tree: deterministic)
__global__ __launch_bounds__(1024) void k_sum_scale(const float* __restrict__ x, int n, float scale,
                                                    float* __restrict__ out, double* __restrict__ out64) {
  __shared__ double red[1024];
  double s = 0.0;
  for (int i = threadIdx.x; i < n; i += 1024) s += (double)x[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int d = 512; d > 0; d >>= 1) {
    if ((int)threadIdx.x < d) red[threadIdx.x] += red[threadIdx.x + d];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    if (out) out[0] = (float)(red[0] * (double)scale);
    if (out64) out64[0] = red[0] * (double)scale;
  }
}

extern "C" int rg_sum_scale(const float* x, int n, float scale, float* out, double* out64, hipStream_t stream) {
  if (n <= 0) return RG_ERR_ARG;
  hipLaunchKernelGGL(k_sum_scale, dim3(1), dim3(1024), 0, stream, x, n, scale, out, out64);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

// ------------------------------------------------------------ dh ----------
// dh_slab[z][b][c] = Σ_{j in split z} dZᵀ[j][b] · W[j][c]
template <int HF>
__global__ __launch_bounds__(256) void k_head_dh(const float* __restrict__ ZT, int64_t ldz,
                                                 const float* __restrict__ lse, const int64_t* __restrict__ tgt,
                                                 float gscale, const float* __restrict__ W, int B, int A,
                                                 int jsplit, float* __restrict__ slabs) {
  constexpr int NCT = HF / 32 > 0 ? HF / 32 : 1;
  constexpr int JC = 32;
  constexpr int LDW = (HF < 32 ? 32 : HF) + 4;
  constexpr int NW4 = JC * HF / 4;            // float4 of W per chunk
  constexpr int NWL = (NW4 + 255) / 256;
  __shared__ __attribute__((aligned(16))) float zt[2][JC][128 + 4];
  __shared__ __attribute__((aligned(16))) float wt[2][JC][LDW];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, half = lane >> 5, l32 = lane & 31;
  const int b0 = blockIdx.x * 128;
  const int jb = blockIdx.y * jsplit;
  const int je = min(A, jb + jsplit);
  // this thread's 4 batch columns of every Zᵀ chunk
  const int c4 = tid & 31;
  const int bq = b0 + 4 * c4;
  float l4[4];
  int64_t t4[4];
  bool v4[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    v4[q] = (bq + q) < B;
    l4[q] = v4[q] ? lse[bq + q] * 1.4426950408889634f : 0.f;  // lse in log2 units
    t4[q] = v4[q] ? tgt[bq + q] : -1;
  }
  f4 zp[4];
  f4 wp[NWL];
  auto load = [&](int j0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int jj = (tid >> 5) + 8 * i;
      const int j = j0 + jj;
      f4 z = {0.f, 0.f, 0.f, 0.f};
      if (j < je && bq < B) z = *reinterpret_cast<const f4*>(ZT + (int64_t)j * ldz + bq);
      zp[i] = z;
    }
#pragma unroll
    for (int i = 0; i < NWL; ++i) {
      const int e = tid + 256 * i;
      const int jj = e / (HF / 4), cc = e % (HF / 4);
      const int j = j0 + jj;
      f4 v = {0.f, 0.f, 0.f, 0.f};
      if (e < NW4 && j < je) v = *reinterpret_cast<const f4*>(W + (int64_t)j * HF + 4 * cc);
      wp[i] = v;
    }
  };
  auto store = [&](int buf, int j0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int jj = (tid >> 5) + 8 * i;
      const int j = j0 + jj;
      f4 d;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float p = __builtin_amdgcn_exp2f(fmaf(zp[i][q], 1.4426950408889634f, -l4[q])) -
                  ((int64_t)j == t4[q] ? 1.0f : 0.0f);
        d[q] = (v4[q] && j < je) ? p * gscale : 0.0f;
      }
      *reinterpret_cast<f4*>(&zt[buf][jj][4 * c4]) = d;
    }
#pragma unroll
    for (int i = 0; i < NWL; ++i) {
      const int e = tid + 256 * i;
      if (e < NW4) {
        const int jj = e / (HF / 4), cc = e % (HF / 4);
        *reinterpret_cast<f4*>(&wt[buf][jj][4 * cc]) = wp[i];
      }
    }
  };
  f16v acc[NCT];
#pragma unroll
  for (int ct = 0; ct < NCT; ++ct) acc[ct] = f16v{};
  if (jb < je) {
    load(jb);
    store(0, jb);
  }
  __syncthreads();
  int cur = 0;
  for (int j0 = jb; j0 < je; j0 += JC) {
    const bool more = j0 + JC < je;
    if (more) load(j0 + JC);
#pragma unroll 4
    for (int s = 0; s < JC / 2; ++s) {
      const float a = zt[cur][2 * s + half][32 * w + l32];
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) {
        const float bb = (HF >= 32 || l32 < HF) ? wt[cur][2 * s + half][ct * 32 + l32] : 0.f;
        acc[ct] = mfma32(a, bb, acc[ct]);
      }
    }
    if (more) store(cur ^ 1, j0 + JC);
    __syncthreads();
    cur ^= 1;
  }
  float* out = slabs + (int64_t)blockIdx.y * B * HF;
#pragma unroll
  for (int ct = 0; ct < NCT; ++ct) {
    const int c = ct * 32 + l32;
    if (c >= HF) continue;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int b = b0 + 32 * w + acc32_row(r, half);
      if (b < B) out[(int64_t)b * HF + c] = acc[ct][r];
    }
  }
}

extern "C" int rg_head_dh(const float* ZT, int64_t ldz, const float* lse, const int64_t* tgt, float gscale,
                          const float* W, int B, int A, int HF, int splits, float* slabs, hipStream_t stream) {
  if (B <= 0 || A <= 0 || splits <= 0) return RG_ERR_ARG;
  if (ldz < ((B + 3) / 4) * 4) return RG_ERR_ARG;
  int jsplit = (A + splits - 1) / splits;
  jsplit = (jsplit + 31) / 32 * 32;
  splits = (A + jsplit - 1) / jsplit;
  dim3 grid((B + 127) / 128, splits);
#define DL(HFV)                                                                                              \
  hipLaunchKernelGGL(k_head_dh<HFV>, grid, dim3(256), 0, stream, ZT, ldz, lse, tgt, gscale, W, B, A, jsplit, \
                     slabs)
  switch (HF) {
    case 16: DL(16); break;
    case 32: DL(32); break;
    case 64: DL(64); break;
    case 128: DL(128); break;
    case 256: DL(256); break;
    default: return RG_ERR_SHAPE;
  }
#undef DL
  RG_LAUNCH_CHECK();
  return splits;  // number of slabs written (>0)
}

// ------------------------------------------------------ dW + Adam ---------
template <int HF>
__global__ __launch_bounds__(256) void k_head_dw_adam(const float* __restrict__ ZT, int64_t ldz,
                                                      const float* __restrict__ lse,
                                                      const int64_t* __restrict__ tgt, float gscale,
                                                      const float* __restrict__ h, int B, int A,
                                                      float* __restrict__ W, float* __restrict__ mW,
                                                      float* __restrict__ vW, float* __restrict__ bias,
                                                      float* __restrict__ mb, float* __restrict__ vb, AdamArgs args,
                                                      float* __restrict__ dW_out, float* __restrict__ db_out) {
  constexpr int NCT = HF / 32 > 0 ? HF / 32 : 1;
  constexpr int BC = 32;
  constexpr int LDZ = BC + 4;
  constexpr int LDH = (HF < 32 ? 32 : HF) + 4;
  constexpr int NH4 = BC * HF / 4;
  constexpr int NHL = (NH4 + 255) / 256;
  __shared__ __attribute__((aligned(16))) float zt[2][128][LDZ];
  __shared__ __attribute__((aligned(16))) float hs[2][BC][LDH];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, half = lane >> 5, l32 = lane & 31;
  const int j0 = blockIdx.x * 128;
  const int c4 = tid & 7;     // this thread's 4 batch columns within a chunk
  const int jr0 = tid >> 3;   // rows jr0 + 32 i, i < 4
  float dbp[4] = {0.f, 0.f, 0.f, 0.f};
  f4 zp[4];
  f4 hp[NHL];
  float l4[4];
  int64_t t4[4];
  auto load = [&](int b0) {
    const int bq = b0 + 4 * c4;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const bool v = (bq + q) < B;
      l4[q] = v ? lse[bq + q] * 1.4426950408889634f : 0.f;  // lse in log2 units
      t4[q] = v ? tgt[bq + q] : -2;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int j = j0 + jr0 + 32 * i;
      f4 z = {0.f, 0.f, 0.f, 0.f};
      if (j < A && bq < B) z = *reinterpret_cast<const f4*>(ZT + (int64_t)j * ldz + bq);
      zp[i] = z;
    }
#pragma unroll
    for (int i = 0; i < NHL; ++i) {
      const int e = tid + 256 * i;
      const int rr = e / (HF / 4), cc = e % (HF / 4);
      f4 v = {0.f, 0.f, 0.f, 0.f};
      if (e < NH4 && b0 + rr < B) v = *reinterpret_cast<const f4*>(h + (int64_t)(b0 + rr) * HF + 4 * cc);
      hp[i] = v;
    }
  };
  auto store = [&](int buf, int b0) {
    const int bq = b0 + 4 * c4;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int jj = jr0 + 32 * i;
      const int j = j0 + jj;
      f4 d;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float p = __builtin_amdgcn_exp2f(fmaf(zp[i][q], 1.4426950408889634f, -l4[q])) -
                  ((int64_t)j == t4[q] ? 1.0f : 0.0f);
        d[q] = ((bq + q) < B && j < A) ? p * gscale : 0.0f;
      }
      dbp[i] += (d[0] + d[1]) + (d[2] + d[3]);
      *reinterpret_cast<f4*>(&zt[buf][jj][4 * c4]) = d;
    }
#pragma unroll
    for (int i = 0; i < NHL; ++i) {
      const int e = tid + 256 * i;
      if (e < NH4) {
        const int rr = e / (HF / 4), cc = e % (HF / 4);
        *reinterpret_cast<f4*>(&hs[buf][rr][4 * cc]) = hp[i];
      }
    }
  };
  f16v acc[NCT];
#pragma unroll
  for (int ct = 0; ct < NCT; ++ct) acc[ct] = f16v{};
  const int nch = (B + BC - 1) / BC;
  load(0);
  store(0, 0);
  __syncthreads();
  int cur = 0;
  for (int c = 0; c < nch; ++c) {
    const bool more = c + 1 < nch;
    if (more) load((c + 1) * BC);
    const float* za = &zt[cur][32 * w + l32][half * (BC / 2)];
#pragma unroll
    for (int s = 0; s < BC / 2; s += 4) {
      f4 av = *reinterpret_cast<const f4*>(za + s);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int bb = half * (BC / 2) + s + q;
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct) {
          const float hv = (HF >= 32 || l32 < HF) ? hs[cur][bb][ct * 32 + l32] : 0.f;
          acc[ct] = mfma32(av[q], hv, acc[ct]);
        }
      }
    }
    if (more) store(cur ^ 1, (c + 1) * BC);
    __syncthreads();
    cur ^= 1;
  }
  // db: the 8 lanes sharing a row (consecutive tid) reduce their partials
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float v = dbp[i];
    v += __shfl_xor(v, 1);
    v += __shfl_xor(v, 2);
    v += __shfl_xor(v, 4);
    dbp[i] = v;
  }
  if (c4 == 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int j = j0 + jr0 + 32 * i;
      if (j >= A) continue;
      if (db_out) {
        db_out[j] = dbp[i];
      } else {
        float p = bias[j], m = mb[j], v = vb[j];
        adam_elem(p, m, v, dbp[i], args);
        bias[j] = p;
        mb[j] = m;
        vb[j] = v;
      }
    }
  }
#pragma unroll
  for (int ct = 0; ct < NCT; ++ct) {
    const int cc = ct * 32 + l32;
    if (cc >= HF) continue;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int j = j0 + 32 * w + acc32_row(r, half);
      if (j >= A) continue;
      const int64_t o = (int64_t)j * HF + cc;
      if (dW_out) {
        dW_out[o] = acc[ct][r];
      } else {
        float p = W[o], m = mW[o], v = vW[o];
        adam_elem(p, m, v, acc[ct][r], args);
        W[o] = p;
        mW[o] = m;
        vW[o] = v;
      }
    }
  }
}

extern "C" int rg_head_dw_adam(const float* ZT, int64_t ldz, const float* lse, const int64_t* tgt, float gscale,
                               const float* h, int B, int A, int HF, float* W, float* mW, float* vW, float* bias,
                               float* mb, float* vb, const float* adam6, float* dW_out, float* db_out,
                               hipStream_t stream) {
  if (B <= 0 || A <= 0) return RG_ERR_ARG;
  if (ldz < ((B + 3) / 4) * 4) return RG_ERR_ARG;
  if (!dW_out && !adam6) return RG_ERR_ARG;
  AdamArgs a{};
  if (adam6) a = AdamArgs{adam6[0], adam6[1], adam6[2], adam6[3], adam6[4], adam6[5]};
  dim3 grid((A + 127) / 128);
#define WL(HFV)                                                                                                 \
  hipLaunchKernelGGL(k_head_dw_adam<HFV>, grid, dim3(256), 0, stream, ZT, ldz, lse, tgt, gscale, h, B, A, W, mW, \
                     vW, bias, mb, vb, a, dW_out, db_out)
  switch (HF) {
    case 16: WL(16); break;
    case 32: WL(32); break;
    case 64: WL(64); break;
    case 128: WL(128); break;
    case 256: WL(256); break;
    default: return RG_ERR_SHAPE;
  }
#undef WL
  RG_LAUNCH_CHECK();
  return RG_OK;
}

// ---------------------------------------------------- item-sharded head ----
// Multi-GPU: rank r owns items [lo, hi).  lse over all items of row b =
// logsumexp over ranks of the per-rank lse (nr × B, rank-major).
__global__ void k_lse_merge_ranks(const float* __restrict__ lse_r, int nr, int B, float* __restrict__ lse) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  float m = -__builtin_inff();
  for (int q = 0; q < nr; ++q) m = fmaxf(m, lse_r[(int64_t)q * B + b]);
  float s = 0.f;
  for (int q = 0; q < nr; ++q) s += expf(lse_r[(int64_t)q * B + b] - m);
  lse[b] = m + logf(s);
}

extern "C" int rg_lse_merge_ranks(const float* lse_r, int nr, int B, float* lse, hipStream_t stream) {
  if (B <= 0 || nr <= 0) return RG_ERR_ARG;
  hipLaunchKernelGGL(k_lse_merge_ranks, dim3((B + 255) / 256), dim3(256), 0, stream, lse_r, nr, B, lse);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

// zt[b] = Zᵀ[a_b − lo][b] when lo ≤ a_b < hi else 0 (summed over ranks
// afterwards); tgt_loc[b] = a_b − lo (out-of-shard targets never match a
// local item in the backward kernels).
__global__ void k_shard_targets(const float* __restrict__ ZT, int64_t ldz, const int64_t* __restrict__ tgt, int64_t lo,
                                int64_t hi, int B, float* __restrict__ zt, int64_t* __restrict__ tgt_loc) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const int64_t t = tgt[b];
  const bool own = t >= lo && t < hi;
  zt[b] = own ? ZT[(t - lo) * ldz + b] : 0.0f;
  tgt_loc[b] = t - lo;
}

extern "C" int rg_shard_targets(const float* ZT, int64_t ldz, const int64_t* tgt, int64_t lo, int64_t hi, int B,
                                float* zt, int64_t* tgt_loc, hipStream_t stream) {
  if (B <= 0 || hi <= lo) return RG_ERR_ARG;
  hipLaunchKernelGGL(k_shard_targets, dim3((B + 255) / 256), dim3(256), 0, stream, ZT, ldz, tgt, lo, hi, B, zt,
                     tgt_loc);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

// loss_row[b] = lse[b] − zt[b]
__global__ void k_sub(const float* __restrict__ a, const float* __restrict__ b, int n, float* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = a[i] - b[i];
}

extern "C" int rg_sub(const float* a, const float* b, int n, float* out, hipStream_t stream) {
  if (n <= 0) return RG_ERR_ARG;
  hipLaunchKernelGGL(k_sub, dim3((n + 255) / 256), dim3(256), 0, stream, a, b, n, out);
  RG_LAUNCH_CHECK();
  return RG_OK;
}
