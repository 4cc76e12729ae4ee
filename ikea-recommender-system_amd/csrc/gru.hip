// Persistent GRU recurrence, forward and BPTT.
//
// Reference semantics (nn.GRU, gate order [r, z, n]; GRU4Rec/model.py:49-55,76-77):
//   r  = σ(gi_r + W_hr h + b_hr)
//   z  = σ(gi_z + W_hz h + b_hz)
//   n  = tanh(gi_n + r ⊙ (W_hn h + b_hn))
//   h' = (h − n) ⊙ z + n            (ATen's GRU cell form of (1−z)n + zh)
// gi = W_ih x + b_ih comes precomputed for every packed token (one MFMA GEMM,
// gemm.hip).  The final hidden is taken at each row's own length (packed
// sequence semantics); rows of a workgroup are length-sorted descending.
//
// Mapping: one workgroup = 16 batch rows × all H units; wave w owns units
// [16w, 16w+16).  W_hh stays in VGPRs for the whole sequence (the recurrent
// matrix, 3H×H fp32 = 192 KB at H=128, does not fit one CU's LDS): each wave
// holds the r/z/n rows of its 16 units (3 × H/4 registers per lane).  Per step
// the 16×H hidden tile is shared through LDS and every wave runs 3·H/4
// v_mfma_f32_16x16x4_f32 (exact f32).  The C/D layout of that MFMA puts
// (batch row = lane&15, units 4·(lane>>4)+0..3) in one lane, so the gate
// nonlinearity is lane-local and h stays in registers between steps.
//
// Saved for BPTT per token (planar, plane stride = T_max·H): h_prev, r, z, n,
// ghn = W_hn h + b_hn.
#include "common.h"

// Per-direction operands: BidirGRU4Rec runs both directions in one launch
// (blockIdx.y = direction), sharing the packing (perm / lsort / offs).
struct GruDirs {
  const float* Gi[2];
  const float* Whh[2];
  const float* bhh[2];
  float* saved[2];
};
struct GruBwdDirs {
  const float* saved[2];
  const float* Whh[2];
  float* dGi[2];
  float* dGh[2];
};

// hk (optional): the final h also leaves as the bf16 K-planes of the whole
// (B × ldh) hidden matrix (csrc/head_flash.hip layout: [row/32][k slice][plane]
// [lane], 16-B entries of 8 consecutive units) for the sampled head's logits
// (csrc/sampled.hip k_sampled_logits, HKP) — split here, once, where h is made.
template <int H>
__global__ __launch_bounds__(H * 4) void k_gru_fwd(GruDirs dirs, const int32_t* __restrict__ perm,
                                                   const int32_t* __restrict__ lsort,
                                                   const int32_t* __restrict__ offs, int B, float* __restrict__ hout,
                                                   int ldh, int hoff0, int64_t plane, bf16x8* __restrict__ hk) {
  // raised wave priority: the recurrence is the step's serial chain, and the
  // catch-up replay (VALU-bound, side stream) shares its CUs — this wave wins
  // issue on the SIMD (C3 +3 %, C2 +0.4 %, same box, profiles/r07/ab_gru_setprio.txt)
  __builtin_amdgcn_s_setprio(3);
  const int dir = blockIdx.y;
  const float* __restrict__ Gi = dirs.Gi[dir];
  const float* __restrict__ Whh = dirs.Whh[dir];
  const float* __restrict__ bhh = dirs.bhh[dir];
  float* __restrict__ saved = dirs.saved[dir];
  const int hoff = hoff0 + dir * H;
  constexpr int KQ = H / 4;  // reduction quarter owned by lane>>4
  constexpr int LDH = H + 4;
  __shared__ __attribute__((aligned(16))) float hbuf[2][16][LDH];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int bl = lane & 15;
  const int kq = lane >> 4;
  const int u0 = 16 * w + 4 * kq;  // first of this lane's 4 output units
  const int r0 = blockIdx.x * 16;
  const int row = r0 + bl;
  const bool valid = row < B;
  const int len = valid ? lsort[row] : 0;
  const int tokb = valid ? offs[row] : 0;
  const int tmax = lsort[r0];

  float Wr[KQ], Wz[KQ], Wn[KQ];
  {
    const int gi = 16 * w + bl;  // A row (gate row within tile) for this lane
#pragma unroll
    for (int s = 0; s < KQ; s += 4) {
      f4 a = *reinterpret_cast<const f4*>(Whh + (int64_t)(0 * H + gi) * H + kq * KQ + s);
      f4 b = *reinterpret_cast<const f4*>(Whh + (int64_t)(1 * H + gi) * H + kq * KQ + s);
      f4 c = *reinterpret_cast<const f4*>(Whh + (int64_t)(2 * H + gi) * H + kq * KQ + s);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        Wr[s + j] = a[j];
        Wz[s + j] = b[j];
        Wn[s + j] = c[j];
      }
    }
  }
  const f4 br = *reinterpret_cast<const f4*>(bhh + 0 * H + u0);
  const f4 bz = *reinterpret_cast<const f4*>(bhh + 1 * H + u0);
  const f4 bn = *reinterpret_cast<const f4*>(bhh + 2 * H + u0);

  f4 h = {0.f, 0.f, 0.f, 0.f};
  *reinterpret_cast<f4*>(&hbuf[0][bl][u0]) = h;
  __syncthreads();
  int cur = 0;
  for (int t = 0; t < tmax; ++t) {
    const bool act = t < len;
    f4 gr = {}, gz = {}, gn = {};
    if (act) {
      const float* g = Gi + (int64_t)(tokb + t) * (3 * H);
      gr = *reinterpret_cast<const f4*>(g + 0 * H + u0);
      gz = *reinterpret_cast<const f4*>(g + 1 * H + u0);
      gn = *reinterpret_cast<const f4*>(g + 2 * H + u0);
    }
    f4 ar = br, az = bz, an = bn;
    const float* hb = &hbuf[cur][bl][kq * KQ];
#pragma unroll
    for (int s = 0; s < KQ; s += 4) {
      f4 hv = *reinterpret_cast<const f4*>(hb + s);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        ar = mfma16(Wr[s + j], hv[j], ar);
        az = mfma16(Wz[s + j], hv[j], az);
        an = mfma16(Wn[s + j], hv[j], an);
      }
    }
    f4 hn = h;
    if (act) {
      f4 rr, zz, nn;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        rr[j] = sigmoidf_ref(gr[j] + ar[j]);
        zz[j] = sigmoidf_ref(gz[j] + az[j]);
        nn[j] = tanhf(gn[j] + rr[j] * an[j]);
        hn[j] = (h[j] - nn[j]) * zz[j] + nn[j];
      }
      if (saved) {
        const int64_t o = (int64_t)(tokb + t) * H + u0;
        *reinterpret_cast<f4*>(saved + 0 * plane + o) = h;
        *reinterpret_cast<f4*>(saved + 1 * plane + o) = rr;
        *reinterpret_cast<f4*>(saved + 2 * plane + o) = zz;
        *reinterpret_cast<f4*>(saved + 3 * plane + o) = nn;
        *reinterpret_cast<f4*>(saved + 4 * plane + o) = an;
      }
    }
    h = hn;
    *reinterpret_cast<f4*>(&hbuf[cur ^ 1][bl][u0]) = h;
    __syncthreads();
    cur ^= 1;
  }
  if (valid) *reinterpret_cast<f4*>(hout + (int64_t)perm[row] * ldh + hoff + u0) = h;
  if (hk != nullptr) {   // hbuf[cur] holds the 16 rows' final h (the loop ended on a barrier)
    constexpr int G = H / 8;   // 8-unit groups of this direction
    for (int i = threadIdx.x; i < 16 * G; i += H * 4) {
      const int rr = i / G, g = i % G;
      if (r0 + rr >= B) continue;
      const f4 lo = *reinterpret_cast<const f4*>(&hbuf[cur][rr][8 * g]);
      const f4 hi = *reinterpret_cast<const f4*>(&hbuf[cur][rr][8 * g + 4]);
      bf16x8 p0, p1, p2;
      split3x8(lo, hi, p0, p1, p2);
      const int x = perm[r0 + rr];
      const int gg = hoff / 8 + g;
      const int64_t e = kplane16(x, gg, ldh);
      hk[e] = p0;
      hk[e + 64] = p1;
      hk[e + 128] = p2;
    }
  }
}

// BPTT.  dh_final (original row order) -> dGi = [da_r, da_z, da_n],
// dGh = [da_r, da_z, da_n ⊙ r] per token; dh_prev = dh ⊙ z + W_hhᵀ dGh.
// Wave w again owns units [16w, 16w+16) of dh; the recurrent product reduces
// over all 3H gate rows, so W_hhᵀ for those units is held in VGPRs
// (3H/4 registers per lane) and the 16 × 3H dGh tile is shared through LDS.
template <int H>
__global__ __launch_bounds__(H * 4) void k_gru_bwd(GruBwdDirs dirs, int64_t plane, const int32_t* __restrict__ perm,
                                                   const int32_t* __restrict__ lsort,
                                                   const int32_t* __restrict__ offs, int B,
                                                   const float* __restrict__ dhout, int lddh, int dhoff0) {
  __builtin_amdgcn_s_setprio(3);   // as in k_gru_fwd
  const int dir = blockIdx.y;
  const float* __restrict__ saved = dirs.saved[dir];
  const float* __restrict__ Whh = dirs.Whh[dir];
  float* __restrict__ dGi = dirs.dGi[dir];
  float* __restrict__ dGh = dirs.dGh[dir];
  const int dhoff = dhoff0 + dir * H;
  constexpr int G = 3 * H;
  constexpr int KQ = G / 4;
  constexpr int LDG = G + 4;
  __shared__ __attribute__((aligned(16))) float gbuf[2][16][LDG];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int bl = lane & 15;
  const int kq = lane >> 4;
  const int u0 = 16 * w + 4 * kq;
  const int r0 = blockIdx.x * 16;
  const int row = r0 + bl;
  const bool valid = row < B;
  const int len = valid ? lsort[row] : 0;
  const int tokb = valid ? offs[row] : 0;
  const int tmax = lsort[r0];

  float WT[KQ];
  {
    const int col = 16 * w + bl;  // unit (A row) held by this lane
#pragma unroll
    for (int s = 0; s < KQ; ++s) WT[s] = Whh[(int64_t)(kq * KQ + s) * H + col];
  }
  f4 dh = {0.f, 0.f, 0.f, 0.f};
  if (valid) dh = *reinterpret_cast<const f4*>(dhout + (int64_t)perm[row] * lddh + dhoff + u0);
  int cur = 0;
  for (int t = tmax - 1; t >= 0; --t) {
    const bool act = t < len;
    f4 dar = {}, daz = {}, dan = {}, dghn = {}, dhd = dh;
    if (act) {
      const int64_t o = (int64_t)(tokb + t) * H + u0;
      const f4 hp = *reinterpret_cast<const f4*>(saved + 0 * plane + o);
      const f4 rr = *reinterpret_cast<const f4*>(saved + 1 * plane + o);
      const f4 zz = *reinterpret_cast<const f4*>(saved + 2 * plane + o);
      const f4 nn = *reinterpret_cast<const f4*>(saved + 3 * plane + o);
      const f4 gh = *reinterpret_cast<const f4*>(saved + 4 * plane + o);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float dn = dh[j] * (1.0f - zz[j]);
        const float dz = dh[j] * (hp[j] - nn[j]);
        dhd[j] = dh[j] * zz[j];
        dan[j] = dn * (1.0f - nn[j] * nn[j]);
        daz[j] = dz * (zz[j] * (1.0f - zz[j]));
        const float dr = dan[j] * gh[j];
        dar[j] = dr * (rr[j] * (1.0f - rr[j]));
        dghn[j] = dan[j] * rr[j];
      }
      float* gi = dGi + (int64_t)(tokb + t) * G;
      float* gh2 = dGh + (int64_t)(tokb + t) * G;
      *reinterpret_cast<f4*>(gi + 0 * H + u0) = dar;
      *reinterpret_cast<f4*>(gi + 1 * H + u0) = daz;
      *reinterpret_cast<f4*>(gi + 2 * H + u0) = dan;
      *reinterpret_cast<f4*>(gh2 + 0 * H + u0) = dar;
      *reinterpret_cast<f4*>(gh2 + 1 * H + u0) = daz;
      *reinterpret_cast<f4*>(gh2 + 2 * H + u0) = dghn;
    }
    *reinterpret_cast<f4*>(&gbuf[cur][bl][0 * H + u0]) = dar;
    *reinterpret_cast<f4*>(&gbuf[cur][bl][1 * H + u0]) = daz;
    *reinterpret_cast<f4*>(&gbuf[cur][bl][2 * H + u0]) = dghn;
    __syncthreads();
    f4 acc = {0.f, 0.f, 0.f, 0.f};
    const float* gb = &gbuf[cur][bl][kq * KQ];
#pragma unroll
    for (int s = 0; s < KQ; s += 4) {
      f4 gv = *reinterpret_cast<const f4*>(gb + s);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc = mfma16(WT[s + j], gv[j], acc);
    }
    if (act) {
#pragma unroll
      for (int j = 0; j < 4; ++j) dh[j] = dhd[j] + acc[j];
    }
    cur ^= 1;
  }
}

template <int H>
static void launch_fwd(const GruDirs& d, int ndir, const int32_t* perm, const int32_t* lsort, const int32_t* offs,
                       int B, float* hout, int ldh, int hoff, int64_t plane, bf16x8* hk, hipStream_t stream) {
  hipLaunchKernelGGL(k_gru_fwd<H>, dim3((B + 15) / 16, ndir), dim3(H * 4), 0, stream, d, perm, lsort, offs, B, hout,
                     ldh, hoff, plane, hk);
}

template <int H>
static void launch_bwd(const GruBwdDirs& d, int ndir, int64_t plane, const int32_t* perm, const int32_t* lsort,
                       const int32_t* offs, int B, const float* dhout, int lddh, int dhoff, hipStream_t stream) {
  hipLaunchKernelGGL(k_gru_bwd<H>, dim3((B + 15) / 16, ndir), dim3(H * 4), 0, stream, d, plane, perm, lsort, offs,
                     B, dhout, lddh, dhoff);
}

static int gru_fwd_dirs(const GruDirs& d, int ndir, const int32_t* perm, const int32_t* lsort, const int32_t* offs,
                        int B, int H, float* hout, int ldh, int hoff, int64_t plane, hipStream_t stream,
                        void* h_planes = nullptr) {
  if (B <= 0 || ndir < 1 || ndir > 2) return RG_ERR_ARG;
  if (h_planes && (!(ldh == 32 || ldh == 64 || ldh == 128 || ldh == 256) || (hoff % 8) || hoff + ndir * H > ldh))
    return RG_ERR_ARG;
  bf16x8* hk = (bf16x8*)h_planes;
  switch (H) {
    case 16: launch_fwd<16>(d, ndir, perm, lsort, offs, B, hout, ldh, hoff, plane, hk, stream); break;
    case 32: launch_fwd<32>(d, ndir, perm, lsort, offs, B, hout, ldh, hoff, plane, hk, stream); break;
    case 64: launch_fwd<64>(d, ndir, perm, lsort, offs, B, hout, ldh, hoff, plane, hk, stream); break;
    case 128: launch_fwd<128>(d, ndir, perm, lsort, offs, B, hout, ldh, hoff, plane, hk, stream); break;
    default: return RG_ERR_SHAPE;
  }
  RG_LAUNCH_CHECK();
  return RG_OK;
}

static int gru_bwd_dirs(const GruBwdDirs& d, int ndir, int64_t plane, const int32_t* perm, const int32_t* lsort,
                        const int32_t* offs, int B, int H, const float* dhout, int lddh, int dhoff,
                        hipStream_t stream) {
  if (B <= 0 || ndir < 1 || ndir > 2) return RG_ERR_ARG;
  switch (H) {
    case 16: launch_bwd<16>(d, ndir, plane, perm, lsort, offs, B, dhout, lddh, dhoff, stream); break;
    case 32: launch_bwd<32>(d, ndir, plane, perm, lsort, offs, B, dhout, lddh, dhoff, stream); break;
    case 64: launch_bwd<64>(d, ndir, plane, perm, lsort, offs, B, dhout, lddh, dhoff, stream); break;
    case 128: launch_bwd<128>(d, ndir, plane, perm, lsort, offs, B, dhout, lddh, dhoff, stream); break;
    default: return RG_ERR_SHAPE;
  }
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_gru_fwd(const float* Gi, const float* Whh, const float* bhh, const int32_t* perm,
                          const int32_t* lsort, const int32_t* offs, int B, int H, float* hout, int ldh, int hoff,
                          float* saved, int64_t plane, hipStream_t stream) {
  const GruDirs d{{Gi, Gi}, {Whh, Whh}, {bhh, bhh}, {saved, saved}};
  return gru_fwd_dirs(d, 1, perm, lsort, offs, B, H, hout, ldh, hoff, plane, stream);
}

extern "C" int rg_gru_bwd(const float* saved, int64_t plane, const float* Whh, const int32_t* perm,
                          const int32_t* lsort, const int32_t* offs, int B, int H, const float* dhout, int lddh,
                          int dhoff, float* dGi, float* dGh, hipStream_t stream) {
  const GruBwdDirs d{{saved, saved}, {Whh, Whh}, {dGi, dGi}, {dGh, dGh}};
  return gru_bwd_dirs(d, 1, plane, perm, lsort, offs, B, H, dhout, lddh, dhoff, stream);
}

// Both directions of a bidirectional layer in one launch (host arrays of
// ndir pointers; direction d writes / reads columns hoff + d·H of hout / dhout).
extern "C" int rg_gru_fwd_dirs(const float* const* Gi, const float* const* Whh, const float* const* bhh,
                               float* const* saved, int ndir, const int32_t* perm, const int32_t* lsort,
                               const int32_t* offs, int B, int H, float* hout, int ldh, int hoff, int64_t plane,
                               hipStream_t stream) {
  if (!Gi || !Whh || !bhh || !saved || ndir < 1 || ndir > 2) return RG_ERR_ARG;
  GruDirs d{};
  for (int i = 0; i < 2; ++i) {
    const int j = i < ndir ? i : 0;
    d.Gi[i] = Gi[j];
    d.Whh[i] = Whh[j];
    d.bhh[i] = bhh[j];
    d.saved[i] = saved[j];
  }
  return gru_fwd_dirs(d, ndir, perm, lsort, offs, B, H, hout, ldh, hoff, plane, stream);
}

// rg_gru_fwd_dirs that also writes the final h as bf16 K-planes (rows padded
// to 32: rg_head_plane_bytes(B, ldh) bytes; ldh in {32, 64, 128, 256}).
// Rows past B in the last 32-row block are left as they are.
extern "C" int rg_gru_fwd_dirs_planes(const float* const* Gi, const float* const* Whh, const float* const* bhh,
                                      float* const* saved, int ndir, const int32_t* perm, const int32_t* lsort,
                                      const int32_t* offs, int B, int H, float* hout, int ldh, int hoff,
                                      int64_t plane, void* h_planes, hipStream_t stream) {
  if (!Gi || !Whh || !bhh || !saved || !h_planes || ndir < 1 || ndir > 2) return RG_ERR_ARG;
  GruDirs d{};
  for (int i = 0; i < 2; ++i) {
    const int j = i < ndir ? i : 0;
    d.Gi[i] = Gi[j];
    d.Whh[i] = Whh[j];
    d.bhh[i] = bhh[j];
    d.saved[i] = saved[j];
  }
  return gru_fwd_dirs(d, ndir, perm, lsort, offs, B, H, hout, ldh, hoff, plane, stream, h_planes);
}

extern "C" int rg_gru_bwd_dirs(float* const* saved, const float* const* Whh, float* const* dGi, float* const* dGh,
                               int ndir, int64_t plane, const int32_t* perm, const int32_t* lsort,
                               const int32_t* offs, int B, int H, const float* dhout, int lddh, int dhoff,
                               hipStream_t stream) {
  if (!saved || !Whh || !dGi || !dGh || ndir < 1 || ndir > 2) return RG_ERR_ARG;
  GruBwdDirs d{};
  for (int i = 0; i < 2; ++i) {
    const int j = i < ndir ? i : 0;
    d.saved[i] = saved[j];
    d.Whh[i] = Whh[j];
    d.dGi[i] = dGi[j];
    d.dGh[i] = dGh[j];
  }
  return gru_bwd_dirs(d, ndir, plane, perm, lsort, offs, B, H, dhout, lddh, dhoff, stream);
}

// ------------------------------------------- persistent wide path (H 256) --
// One launch for the whole sequence at H = 256 (config C5), where W_hh
// (768 KB fp32) fits neither one CU's VGPRs nor its LDS: each workgroup owns
// 32 length-sorted batch rows for all timesteps and streams W_hh from L2
// (which holds it: 768 KB of each XCD's 4 MB) every step, as MFMA-fragment
// ordered 16-B loads; h (fwd) / dG (BPTT) of the 32 rows is the A operand
// from LDS.  v_mfma_f32_32x32x2_f32 (exact fp32): lane l feeds A[l%32][k] /
// B[k][l%32] with k = 2q + l/32 of each 8-wide k block, and holds
// C[acc32_row(r, l/32)][l%32] — one unit (column) × 16 rows per lane, so the
// gate math stays lane-local.  Per step and wave: 3 gates × H/2 MFMAs.
//
// Fragment layout (k_gru_wfrag): frag[(nb·K/8 + kk)·64 + lane] (16 B) holds
// M[kk·8 + 2q + lane/32][nb·32 + lane%32], q = 0..3, for the K × N operand
// M[k][n] = src[k·sk + n·sn].  LDS rows store k at position
// (k & ~7) + (k & 1)·4 + ((k >> 1) & 3), so a lane's four k values of one
// block are one ds_read_b128.
__device__ __forceinline__ int wide_pos(int k) { return (k & ~7) + (k & 1) * 4 + ((k >> 1) & 3); }

__global__ void k_gru_wfrag(const float* __restrict__ src, int64_t sk, int64_t sn, int K, int N, f4* __restrict__ frag) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int KK = K / 8;
  if (e >= (int64_t)(N / 32) * KK * 64) return;
  const int lane = (int)(e & 63);
  const int64_t blk = e >> 6;
  const int kk = (int)(blk % KK), nb = (int)(blk / KK);
  const int n = nb * 32 + (lane & 31), k0 = kk * 8 + (lane >> 5);
  f4 v;
#pragma unroll
  for (int q = 0; q < 4; ++q) v[q] = src[(int64_t)(k0 + 2 * q) * sk + (int64_t)n * sn];
  frag[e] = v;
}

template <int H>
__global__ __launch_bounds__(2 * H) void k_gru_fwd_wide(const float* __restrict__ Gi, const f4* __restrict__ WF,
                                                        const float* __restrict__ bhh, const int32_t* __restrict__ perm,
                                                        const int32_t* __restrict__ lsort,
                                                        const int32_t* __restrict__ offs, int B,
                                                        float* __restrict__ hout, int ldh, int hoff,
                                                        float* __restrict__ saved, int64_t plane) {
  constexpr int NW = H / 32, KK = H / 8, LDX = H + 4;
  __shared__ __attribute__((aligned(16))) float xs[2][32][LDX];
  __shared__ int len_s[32], tok_s[32];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, hh = lane >> 5, j = lane & 31;
  const int u = 32 * w + j;  // this lane's unit
  const int r0 = blockIdx.x * 32;
  if (tid < 32) {
    const bool v = r0 + tid < B;
    len_s[tid] = v ? lsort[r0 + tid] : 0;
    tok_s[tid] = v ? offs[r0 + tid] : 0;
  }
  for (int e = tid; e < 32 * LDX; e += 2 * H) xs[0][e / LDX][e % LDX] = 0.f;
  const float br = bhh[u], bz = bhh[H + u], bn = bhh[2 * H + u];
  const int tmax = lsort[r0];
  const int pu = wide_pos(u);
  const f4* wr_p = WF + (int64_t)(0 * NW + w) * KK * 64 + lane;
  const f4* wz_p = WF + (int64_t)(1 * NW + w) * KK * 64 + lane;
  const f4* wn_p = WF + (int64_t)(2 * NW + w) * KK * 64 + lane;
  float h[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) h[i] = 0.f;
  __syncthreads();
  int cur = 0;
  for (int t = 0; t < tmax; ++t) {
    // this step's input-gate terms (issued ahead of the MFMAs)
    float gr[16], gz[16], gn[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int row = acc32_row(i, hh);
      gr[i] = gz[i] = gn[i] = 0.f;
      if (t < len_s[row]) {
        const float* g = Gi + (int64_t)(tok_s[row] + t) * (3 * H);
        gr[i] = g[u];
        gz[i] = g[H + u];
        gn[i] = g[2 * H + u];
      }
    }
    f16v ar, az, an;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      ar[i] = br;
      az[i] = bz;
      an[i] = bn;
    }
    const float* xa = &xs[cur][j][hh * 4];
#pragma unroll 4
    for (int kk = 0; kk < KK; ++kk) {
      const f4 a = *reinterpret_cast<const f4*>(xa + kk * 8);
      const f4 vr = wr_p[kk * 64], vz = wz_p[kk * 64], vn = wn_p[kk * 64];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        ar = mfma32(a[q], vr[q], ar);
        az = mfma32(a[q], vz[q], az);
        an = mfma32(a[q], vn[q], an);
      }
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int row = acc32_row(i, hh);
      if (t < len_s[row]) {
        const float rr = sigmoidf_ref(gr[i] + ar[i]);
        const float zz = sigmoidf_ref(gz[i] + az[i]);
        const float nn = tanhf(gn[i] + rr * an[i]);
        const float hn = (h[i] - nn) * zz + nn;
        if (saved) {
          const int64_t o = (int64_t)(tok_s[row] + t) * H + u;
          saved[0 * plane + o] = h[i];
          saved[1 * plane + o] = rr;
          saved[2 * plane + o] = zz;
          saved[3 * plane + o] = nn;
          saved[4 * plane + o] = an[i];
        }
        h[i] = hn;
      }
      xs[cur ^ 1][row][pu] = h[i];
    }
    __syncthreads();
    cur ^= 1;
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int row = r0 + acc32_row(i, hh);
    if (row < B) hout[(int64_t)perm[row] * ldh + hoff + u] = h[i];
  }
}

template <int H>
__global__ __launch_bounds__(2 * H) void k_gru_bwd_wide(const float* __restrict__ saved, int64_t plane,
                                                        const f4* __restrict__ WB, const int32_t* __restrict__ perm,
                                                        const int32_t* __restrict__ lsort,
                                                        const int32_t* __restrict__ offs, int B,
                                                        const float* __restrict__ dhout, int lddh, int dhoff,
                                                        float* __restrict__ dGi, float* __restrict__ dGh) {
  constexpr int G = 3 * H, KK = G / 8, LDG = G + 4;
  __shared__ __attribute__((aligned(16))) float gs[32][LDG];
  __shared__ int len_s[32], tok_s[32];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, hh = lane >> 5, j = lane & 31;
  const int u = 32 * w + j;
  const int r0 = blockIdx.x * 32;
  if (tid < 32) {
    const bool v = r0 + tid < B;
    len_s[tid] = v ? lsort[r0 + tid] : 0;
    tok_s[tid] = v ? offs[r0 + tid] : 0;
  }
  const int tmax = lsort[r0];
  const int p0 = wide_pos(u), p1 = wide_pos(H + u), p2 = wide_pos(2 * H + u);
  const f4* wb_p = WB + (int64_t)w * KK * 64 + lane;
  float dh[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int row = r0 + acc32_row(i, hh);
    dh[i] = row < B ? dhout[(int64_t)perm[row] * lddh + dhoff + u] : 0.f;
  }
  __syncthreads();
  for (int t = tmax - 1; t >= 0; --t) {
    float dhd[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int row = acc32_row(i, hh);
      float dar = 0.f, daz = 0.f, dghn = 0.f;
      dhd[i] = dh[i];
      if (t < len_s[row]) {
        const int64_t tok = tok_s[row] + t;
        const int64_t o = tok * H + u;
        const float hp = saved[0 * plane + o], rr = saved[1 * plane + o], zz = saved[2 * plane + o];
        const float nn = saved[3 * plane + o], gh = saved[4 * plane + o];
        const float dn = dh[i] * (1.0f - zz);
        const float dz = dh[i] * (hp - nn);
        dhd[i] = dh[i] * zz;
        const float dan = dn * (1.0f - nn * nn);
        daz = dz * (zz * (1.0f - zz));
        dar = (dan * gh) * (rr * (1.0f - rr));
        dghn = dan * rr;
        float* gi = dGi + tok * G;
        float* g2 = dGh + tok * G;
        gi[u] = dar;
        gi[H + u] = daz;
        gi[2 * H + u] = dan;
        g2[u] = dar;
        g2[H + u] = daz;
        g2[2 * H + u] = dghn;
      }
      gs[row][p0] = dar;
      gs[row][p1] = daz;
      gs[row][p2] = dghn;
    }
    __syncthreads();
    if (t > 0) {  // recurrent term of step t-1: W_hhᵀ · dG
      f16v acc = {};
      const float* ga = &gs[j][hh * 4];
#pragma unroll 4
      for (int kk = 0; kk < KK; ++kk) {
        const f4 a = *reinterpret_cast<const f4*>(ga + kk * 8);
        const f4 v = wb_p[kk * 64];
#pragma unroll
        for (int q = 0; q < 4; ++q) acc = mfma32(a[q], v[q], acc);
      }
#pragma unroll
      for (int i = 0; i < 16; ++i)
        if (t < len_s[acc32_row(i, hh)]) dh[i] = dhd[i] + acc[i];
    }
    __syncthreads();
  }
}

extern "C" int64_t rg_gru_wide_work_bytes(int H) { return H == 256 ? (int64_t)3 * H * H * 4 : RG_ERR_SHAPE; }

extern "C" int rg_gru_fwd_wide(const float* Gi, const float* Whh, const float* bhh, const int32_t* perm,
                               const int32_t* lsort, const int32_t* offs, int B, int H, float* hout, int ldh, int hoff,
                               float* saved, int64_t plane, void* wfrag, hipStream_t stream) {
  if (B <= 0 || !Gi || !Whh || !bhh || !perm || !lsort || !offs || !hout || !wfrag) return RG_ERR_ARG;
  if (H != 256) return RG_ERR_SHAPE;
  const int64_t nf = (int64_t)3 * H / 32 * (H / 8) * 64;
  // operand M[k][n] = W_hh[n][k]: K = H, N = 3H
  hipLaunchKernelGGL(k_gru_wfrag, dim3((unsigned)((nf + 255) / 256)), dim3(256), 0, stream, Whh, (int64_t)1,
                     (int64_t)H, H, 3 * H, (f4*)wfrag);
  hipLaunchKernelGGL(k_gru_fwd_wide<256>, dim3((B + 31) / 32), dim3(2 * 256), 0, stream, Gi, (const f4*)wfrag, bhh,
                     perm, lsort, offs, B, hout, ldh, hoff, saved, plane);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_gru_bwd_wide(const float* saved, int64_t plane, const float* Whh, const int32_t* perm,
                               const int32_t* lsort, const int32_t* offs, int B, int H, const float* dhout, int lddh,
                               int dhoff, float* dGi, float* dGh, void* wfrag, hipStream_t stream) {
  if (B <= 0 || !saved || !Whh || !perm || !lsort || !offs || !dhout || !dGi || !dGh || !wfrag) return RG_ERR_ARG;
  if (H != 256) return RG_ERR_SHAPE;
  const int64_t nf = (int64_t)H / 32 * (3 * H / 8) * 64;
  // operand M[k][n] = W_hh[k][n]: K = 3H, N = H
  hipLaunchKernelGGL(k_gru_wfrag, dim3((unsigned)((nf + 255) / 256)), dim3(256), 0, stream, Whh, (int64_t)H,
                     (int64_t)1, 3 * H, H, (f4*)wfrag);
  hipLaunchKernelGGL(k_gru_bwd_wide<256>, dim3((B + 31) / 32), dim3(2 * 256), 0, stream, saved, plane,
                     (const f4*)wfrag, perm, lsort, offs, B, dhout, lddh, dhoff, dGi, dGh);
  RG_LAUNCH_CHECK();
  return RG_OK;
}
