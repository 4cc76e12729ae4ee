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

template <int H>
__global__ __launch_bounds__(H * 4) void k_gru_fwd(const float* __restrict__ Gi, const float* __restrict__ Whh,
                                                   const float* __restrict__ bhh, const int32_t* __restrict__ perm,
                                                   const int32_t* __restrict__ lsort,
                                                   const int32_t* __restrict__ offs, int B, float* __restrict__ hout,
                                                   int ldh, int hoff, float* __restrict__ saved, int64_t plane) {
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
}

// BPTT.  dh_final (original row order) -> dGi = [da_r, da_z, da_n],
// dGh = [da_r, da_z, da_n ⊙ r] per token; dh_prev = dh ⊙ z + W_hhᵀ dGh.
// Wave w again owns units [16w, 16w+16) of dh; the recurrent product reduces
// over all 3H gate rows, so W_hhᵀ for those units is held in VGPRs
// (3H/4 registers per lane) and the 16 × 3H dGh tile is shared through LDS.
template <int H>
__global__ __launch_bounds__(H * 4) void k_gru_bwd(const float* __restrict__ saved, int64_t plane,
                                                   const float* __restrict__ Whh, const int32_t* __restrict__ perm,
                                                   const int32_t* __restrict__ lsort,
                                                   const int32_t* __restrict__ offs, int B,
                                                   const float* __restrict__ dhout, int lddh, int dhoff,
                                                   float* __restrict__ dGi, float* __restrict__ dGh) {
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
static int launch_fwd(const float* Gi, const float* Whh, const float* bhh, const int32_t* perm,
                      const int32_t* lsort, const int32_t* offs, int B, float* hout, int ldh, int hoff,
                      float* saved, int64_t plane, hipStream_t stream) {
  hipLaunchKernelGGL(k_gru_fwd<H>, dim3((B + 15) / 16), dim3(H * 4), 0, stream, Gi, Whh, bhh, perm, lsort, offs,
                     B, hout, ldh, hoff, saved, plane);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

template <int H>
static int launch_bwd(const float* saved, int64_t plane, const float* Whh, const int32_t* perm,
                      const int32_t* lsort, const int32_t* offs, int B, const float* dhout, int lddh, int dhoff,
                      float* dGi, float* dGh, hipStream_t stream) {
  hipLaunchKernelGGL(k_gru_bwd<H>, dim3((B + 15) / 16), dim3(H * 4), 0, stream, saved, plane, Whh, perm, lsort,
                     offs, B, dhout, lddh, dhoff, dGi, dGh);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_gru_fwd(const float* Gi, const float* Whh, const float* bhh, const int32_t* perm,
                          const int32_t* lsort, const int32_t* offs, int B, int H, float* hout, int ldh, int hoff,
                          float* saved, int64_t plane, hipStream_t stream) {
  if (B <= 0) return RG_ERR_ARG;
  switch (H) {
    case 16: return launch_fwd<16>(Gi, Whh, bhh, perm, lsort, offs, B, hout, ldh, hoff, saved, plane, stream);
    case 32: return launch_fwd<32>(Gi, Whh, bhh, perm, lsort, offs, B, hout, ldh, hoff, saved, plane, stream);
    case 64: return launch_fwd<64>(Gi, Whh, bhh, perm, lsort, offs, B, hout, ldh, hoff, saved, plane, stream);
    case 128: return launch_fwd<128>(Gi, Whh, bhh, perm, lsort, offs, B, hout, ldh, hoff, saved, plane, stream);
    default: return RG_ERR_SHAPE;
  }
}

extern "C" int rg_gru_bwd(const float* saved, int64_t plane, const float* Whh, const int32_t* perm,
                          const int32_t* lsort, const int32_t* offs, int B, int H, const float* dhout, int lddh,
                          int dhoff, float* dGi, float* dGh, hipStream_t stream) {
  if (B <= 0) return RG_ERR_ARG;
  switch (H) {
    case 16: return launch_bwd<16>(saved, plane, Whh, perm, lsort, offs, B, dhout, lddh, dhoff, dGi, dGh, stream);
    case 32: return launch_bwd<32>(saved, plane, Whh, perm, lsort, offs, B, dhout, lddh, dhoff, dGi, dGh, stream);
    case 64: return launch_bwd<64>(saved, plane, Whh, perm, lsort, offs, B, dhout, lddh, dhoff, dGi, dGh, stream);
    case 128:
      return launch_bwd<128>(saved, plane, Whh, perm, lsort, offs, B, dhout, lddh, dhoff, dGi, dGh, stream);
    default: return RG_ERR_SHAPE;
  }
}

// ------------------------------------------------ time-stepped path -------
// For hidden sizes whose recurrent matrix cannot stay register-resident
// (H = 256, config C5: W_hh is 768 KB), the recurrence runs one timestep per
// pair of launches from a native loop: Gh = h·W_hhᵀ + b_hh for the rows still
// active at step t (an MFMA GEMM, rg_gemm_f32, whose row count nact[t] is read
// on the device), then one fused gate kernel.  Rows are length-sorted
// descending, so the rows active at t are the prefix [0, nact[t]).  Same
// formulas, token layout and saved planes as k_gru_fwd / k_gru_bwd.
extern "C" int rg_gemm_f32(const float* A, int64_t sam, int64_t sak, const float* B, int64_t sbk, int64_t sbn,
                           float* C, int64_t ldc, const float* bias, int M, const int32_t* Mptr, int N, int K,
                           const int32_t* Kptr, int splits, hipStream_t stream);

// nact[t] = #rows with length > t, t ≤ tmax (nact[tmax] = 0)
__global__ void k_gru_counts(const int32_t* __restrict__ lsort, int B, int tmax, int32_t* __restrict__ nact) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t > tmax) return;
  int lo = 0, hi = B;  // first row with lsort <= t (lsort descending)
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (lsort[mid] > t) lo = mid + 1;
    else hi = mid;
  }
  nact[t] = lo;
}

__global__ void k_gru_step_fwd(int t, const float* __restrict__ Gi, const float* __restrict__ Gh,
                               const int32_t* __restrict__ nact, const int32_t* __restrict__ offs, int H,
                               float* __restrict__ hs, float* __restrict__ saved, int64_t plane) {
  const int r = blockIdx.x;
  if (r >= nact[t]) return;
  const int64_t tok = offs[r] + t;
  const float* gi = Gi + tok * 3 * H;
  const float* gh = Gh + (int64_t)r * 3 * H;
  for (int u = threadIdx.x; u < H; u += blockDim.x) {
    const float hp = hs[(int64_t)r * H + u];
    const float rr = sigmoidf_ref(gi[u] + gh[u]);
    const float zz = sigmoidf_ref(gi[H + u] + gh[H + u]);
    const float an = gh[2 * H + u];
    const float nn = tanhf(gi[2 * H + u] + rr * an);
    hs[(int64_t)r * H + u] = (hp - nn) * zz + nn;
    if (saved) {
      const int64_t o = tok * H + u;
      saved[0 * plane + o] = hp;
      saved[1 * plane + o] = rr;
      saved[2 * plane + o] = zz;
      saved[3 * plane + o] = nn;
      saved[4 * plane + o] = an;
    }
  }
}

__global__ void k_gru_rows_out(const float* __restrict__ hs, const int32_t* __restrict__ perm, int B, int H,
                               float* __restrict__ hout, int ldh, int hoff) {
  const int r = blockIdx.x;
  for (int u = threadIdx.x; u < H; u += blockDim.x) hout[(int64_t)perm[r] * ldh + hoff + u] = hs[(int64_t)r * H + u];
}

// dh entering step t: rows continuing from t+1 sum the direct and recurrent
// terms left by step t+1; rows whose last token is t start from dh_final.
__global__ void k_gru_step_bwd(int t, const float* __restrict__ saved, int64_t plane,
                               const int32_t* __restrict__ nact, const int32_t* __restrict__ offs,
                               const int32_t* __restrict__ perm, int H, const float* __restrict__ dhout, int lddh,
                               int dhoff, float* __restrict__ dh_dir, const float* __restrict__ dh_mat,
                               float* __restrict__ dGi, float* __restrict__ dGh, float* __restrict__ dGs) {
  const int r = blockIdx.x;
  if (r >= nact[t]) return;
  const bool cont = r < nact[t + 1];
  const int64_t tok = offs[r] + t;
  const int G = 3 * H;
  for (int u = threadIdx.x; u < H; u += blockDim.x) {
    const int64_t ri = (int64_t)r * H + u;
    const float dh = cont ? dh_dir[ri] + dh_mat[ri] : dhout[(int64_t)perm[r] * lddh + dhoff + u];
    const int64_t o = tok * H + u;
    const float hp = saved[0 * plane + o], rr = saved[1 * plane + o], zz = saved[2 * plane + o];
    const float nn = saved[3 * plane + o], gh = saved[4 * plane + o];
    const float dn = dh * (1.0f - zz);
    const float dz = dh * (hp - nn);
    const float dan = dn * (1.0f - nn * nn);
    const float daz = dz * (zz * (1.0f - zz));
    const float dar = (dan * gh) * (rr * (1.0f - rr));
    const float dghn = dan * rr;
    dh_dir[ri] = dh * zz;
    float* gi = dGi + tok * G;
    float* g2 = dGh + tok * G;
    float* gs = dGs + (int64_t)r * G;
    gi[u] = dar;
    gi[H + u] = daz;
    gi[2 * H + u] = dan;
    g2[u] = dar;
    g2[H + u] = daz;
    g2[2 * H + u] = dghn;
    gs[u] = dar;
    gs[H + u] = daz;
    gs[2 * H + u] = dghn;
  }
}

extern "C" int rg_gru_fwd_steps(const float* Gi, const float* Whh, const float* bhh, const int32_t* perm,
                                const int32_t* lsort, const int32_t* offs, int B, int H, int tmax, float* hout,
                                int ldh, int hoff, float* saved, int64_t plane, float* work, hipStream_t stream) {
  if (B <= 0 || H <= 0 || H % 4 || tmax <= 0) return RG_ERR_ARG;
  float* hs = work;                                               // B × H
  float* Gh = hs + (int64_t)B * H;                                // B × 3H
  int32_t* nact = reinterpret_cast<int32_t*>(Gh + (int64_t)B * 3 * H);  // tmax + 1
  hipLaunchKernelGGL(k_gru_counts, dim3((tmax + 256) / 256), dim3(256), 0, stream, lsort, B, tmax, nact);
  if (hipMemsetAsync(hs, 0, sizeof(float) * (size_t)B * H, stream) != hipSuccess) return RG_ERR_LAUNCH;
  const int thr = H < 256 ? H : 256;
  for (int t = 0; t < tmax; ++t) {
    int rc = rg_gemm_f32(hs, H, 1, Whh, 1, H, Gh, 3 * H, bhh, B, nact + t, 3 * H, H, nullptr, 1, stream);
    if (rc != RG_OK) return rc;
    hipLaunchKernelGGL(k_gru_step_fwd, dim3(B), dim3(thr), 0, stream, t, Gi, Gh, nact, offs, H, hs, saved, plane);
  }
  hipLaunchKernelGGL(k_gru_rows_out, dim3(B), dim3(thr), 0, stream, hs, perm, B, H, hout, ldh, hoff);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_gru_bwd_steps(const float* saved, int64_t plane, const float* Whh, const int32_t* perm,
                                const int32_t* lsort, const int32_t* offs, int B, int H, int tmax,
                                const float* dhout, int lddh, int dhoff, float* dGi, float* dGh, float* work,
                                hipStream_t stream) {
  if (B <= 0 || H <= 0 || H % 4 || tmax <= 0) return RG_ERR_ARG;
  float* dh_dir = work;                                            // B × H
  float* dh_mat = dh_dir + (int64_t)B * H;                         // B × H
  float* dGs = dh_mat + (int64_t)B * H;                            // B × 3H
  int32_t* nact = reinterpret_cast<int32_t*>(dGs + (int64_t)B * 3 * H);  // tmax + 1
  hipLaunchKernelGGL(k_gru_counts, dim3((tmax + 256) / 256), dim3(256), 0, stream, lsort, B, tmax, nact);
  const int thr = H < 256 ? H : 256;
  for (int t = tmax - 1; t >= 0; --t) {
    hipLaunchKernelGGL(k_gru_step_bwd, dim3(B), dim3(thr), 0, stream, t, saved, plane, nact, offs, perm, H, dhout,
                       lddh, dhoff, dh_dir, dh_mat, dGi, dGh, dGs);
    if (t > 0) {  // recurrent term for step t−1: dGs · W_hh over the active rows
      int rc = rg_gemm_f32(dGs, 3 * H, 1, Whh, H, 1, dh_mat, H, nullptr, B, nact + t, H, 3 * H, nullptr, 1, stream);
      if (rc != RG_OK) return rc;
    }
  }
  RG_LAUNCH_CHECK();
  return RG_OK;
}
