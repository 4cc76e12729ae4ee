// Ragged packing and item-embedding gather / scatter (A3).
//
// Reference: recommenders/models/GRU4Rec/model.py:68-74 —
//   emb = nn.Embedding(s); pack_padded_sequence(emb, lengths, enforce_sorted=False)
// The reference sorts on the host and materialises (B, L, E) embeddings incl.
// pads.  Here: one device pass sorts rows by length (descending, stable), writes
// CSR offsets over the sorted rows, and the gather writes only the T valid
// tokens as a packed (T, E) fp32 matrix plus their int32 item ids.
#include "common.h"
#include <hip/hip_fp16.h>

// ---------------------------------------------------------------- pack -----
// One workgroup of 1024 threads.  lens (int64, B) are clamped to [1, L] (the
// host shim validates CPU lengths like pack_padded_sequence does).  With
// unpacked=1 every row runs all L steps (GRU4Rec/model.py:73-74: the
// unpacked GRU consumes pads and returns the state after step L).
// Outputs: perm[r] = original row of sorted row r, lsort[r], offs[r] (r<=B).
#define PACK_THREADS 1024
#define PACK_MAXL 512
__global__ __launch_bounds__(PACK_THREADS) void k_pack(const int64_t* __restrict__ lens, int B, int L,
                                                       int unpacked, int32_t* __restrict__ perm,
                                                       int32_t* __restrict__ lsort,
                                                       int32_t* __restrict__ offs) {
  __shared__ int cnt[PACK_MAXL + 1];
  __shared__ int start[PACK_MAXL + 2];
  __shared__ int chunk_len[PACK_THREADS];
  __shared__ int scan[PACK_THREADS];
  __shared__ int carry;
  const int tid = threadIdx.x;
  for (int v = tid; v <= PACK_MAXL; v += PACK_THREADS) cnt[v] = 0;
  __syncthreads();
  for (int b = tid; b < B; b += PACK_THREADS) {
    int l = unpacked ? L : (int)lens[b];
    l = l < 1 ? 1 : (l > L ? L : l);
    atomicAdd(&cnt[l], 1);
  }
  __syncthreads();
  if (tid == 0) {
    int acc = 0;
    for (int v = L; v >= 1; --v) {  // descending length order
      start[v] = acc;
      acc += cnt[v];
    }
  }
  __syncthreads();
  // stable rank within each length bin, chunk by chunk
  for (int c0 = 0; c0 < B; c0 += PACK_THREADS) {
    int b = c0 + tid;
    int l = 0;
    if (b < B) {
      l = unpacked ? L : (int)lens[b];
      l = l < 1 ? 1 : (l > L ? L : l);
    }
    chunk_len[tid] = (b < B) ? l : -1;
    __syncthreads();
    if (b < B) {
      int before = 0;
      for (int j = 0; j < tid; ++j) before += (chunk_len[j] == l);
      int r = start[l] + before;
      perm[r] = b;
      lsort[r] = l;
    }
    __syncthreads();
    // advance bin starts by this chunk's counts
    if (tid <= L && tid >= 1) {
      int add = 0;
      int n = min(PACK_THREADS, B - c0);
      for (int j = 0; j < n; ++j) add += (chunk_len[j] == tid);
      start[tid] += add;
    }
    __syncthreads();
  }
  // exclusive scan of lsort -> offs (offs[B] = T)
  if (tid == 0) carry = 0;
  __syncthreads();
  for (int c0 = 0; c0 < B; c0 += PACK_THREADS) {
    int r = c0 + tid;
    int v = (r < B) ? lsort[r] : 0;
    scan[tid] = v;
    __syncthreads();
    for (int d = 1; d < PACK_THREADS; d <<= 1) {
      int x = (tid >= d) ? scan[tid - d] : 0;
      __syncthreads();
      scan[tid] += x;
      __syncthreads();
    }
    if (r < B) offs[r] = carry + scan[tid] - v;
    __syncthreads();
    if (tid == PACK_THREADS - 1) carry += scan[tid];
    __syncthreads();
  }
  if (tid == 0) offs[B] = carry;
}

#define PACK_SORT_MAX 8192

// B <= PACK_SORT_MAX (the step's pack): a stable counting sort by length in
// one workgroup, no comparison network.  Wave w takes rows w·64·per .. +64·per,
// round q of it rows q·64 + lane (so (wave, round, lane) order is row order);
// bin = L − len (ascending bin = descending length).  Per-wave bin counts in
// LDS -> per bin the waves' exclusive prefix and total -> bin starts and token
// offsets by one scan over the L bins (every row of a bin has the same
// length: offs[r] = binoff[b] + (r − binstart[b])·len) -> each round's rows
// ranked by a match loop over the wave's distinct bins (one ballot per value
// and round).  The bitonic sort it replaces ran 78 barrier-separated stages,
// 40 us at B 4096.
__device__ __forceinline__ int pack_block_exscan(int v, int* wsum, int& total) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  int inc = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int y = __shfl_up(inc, d);
    if (lane >= d) inc += y;
  }
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  int base = 0, all = 0;
  for (int q = 0; q < PACK_THREADS / 64; ++q) {
    base += q < w ? wsum[q] : 0;
    all += wsum[q];
  }
  __syncthreads();   // wsum reusable
  total = all;
  return base + inc - v;
}

__global__ __launch_bounds__(PACK_THREADS) void k_pack_count(const int64_t* __restrict__ lens, int B, int L,
                                                             int unpacked, int per, int32_t* __restrict__ perm,
                                                             int32_t* __restrict__ lsort, int32_t* __restrict__ offs) {
  constexpr int NWV = PACK_THREADS / 64, PMAX = PACK_SORT_MAX / PACK_THREADS;
  __shared__ int cnt[NWV][PACK_MAXL];   // wave w's rows in bin b -> the earlier waves' rows in bin b
  __shared__ int bstart[PACK_MAXL], boff[PACK_MAXL];
  __shared__ int wsum[NWV];
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  for (int i = tid; i < NWV * PACK_MAXL; i += PACK_THREADS) (&cnt[0][0])[i] = 0;
  __syncthreads();
  const int rw = w * 64 * per + lane;   // row of round 0
  int bins[PMAX];
#pragma unroll
  for (int q = 0; q < PMAX; ++q) {
    const int r = rw + 64 * q;
    bins[q] = -1;
    if (q < per && r < B) {
      int l = unpacked ? L : (int)lens[r];
      l = l < 1 ? 1 : (l > L ? L : l);
      bins[q] = L - l;
      atomicAdd(&cnt[w][L - l], 1);
    }
  }
  __syncthreads();
  int tot = 0;
  if (tid < L) {
    for (int q = 0; q < NWV; ++q) {
      const int c = cnt[q][tid];
      cnt[q][tid] = tot;
      tot += c;
    }
  }
  int T = 0, nb = 0;
  const int bs = pack_block_exscan(tid < L ? tot : 0, wsum, nb);
  const int bo = pack_block_exscan(tid < L ? tot * (L - tid) : 0, wsum, T);
  if (tid < L) {
    bstart[tid] = bs;
    boff[tid] = bo;
  }
  __syncthreads();
  // ranks inside the wave: one match step per distinct bin of its rows (the
  // leader value's ballot in every round; no LDS traffic in the loop)
  const uint64_t lt = (1ull << lane) - 1ull;
  uint64_t pend[PMAX];
  int rk[PMAX];
#pragma unroll
  for (int q = 0; q < PMAX; ++q) {
    pend[q] = q < per ? __ballot(bins[q] >= 0) : 0ull;
    rk[q] = 0;
  }
  for (;;) {
    int v = -1;
#pragma unroll
    for (int q = 0; q < PMAX; ++q)
      if (v < 0 && pend[q] != 0ull) v = __builtin_amdgcn_readlane(bins[q], __builtin_ctzll(pend[q]));
    if (v < 0) break;
    int acc = 0;   // rows of bin v in the wave's earlier rounds
#pragma unroll
    for (int q = 0; q < PMAX; ++q) {
      if (q < per) {
        const uint64_t m = __ballot(bins[q] == v);
        if (bins[q] == v) rk[q] = acc + __popcll(m & lt);
        acc += __popcll(m);
        pend[q] &= ~m;
      }
    }
  }
#pragma unroll
  for (int q = 0; q < PMAX; ++q) {
    const int b = bins[q];
    if (q < per && b >= 0) {
      const int pos = bstart[b] + cnt[w][b] + rk[q];
      perm[pos] = rw + 64 * q;
      lsort[pos] = L - b;
      offs[pos] = boff[b] + (pos - bstart[b]) * (L - b);
    }
  }
  if (tid == 0) offs[B] = T;
}

extern "C" int rg_pack(const int64_t* lens, int B, int L, int unpacked, int32_t* perm, int32_t* lsort,
                       int32_t* offs, hipStream_t stream) {
  if (B <= 0 || L <= 0 || L > PACK_MAXL) return RG_ERR_ARG;
  if (B <= PACK_SORT_MAX) {
    const int per = (B + PACK_THREADS - 1) / PACK_THREADS;
    hipLaunchKernelGGL(k_pack_count, dim3(1), dim3(PACK_THREADS), 0, stream, lens, B, L, unpacked, per, perm, lsort,
                       offs);
  } else {
    hipLaunchKernelGGL(k_pack, dim3(1), dim3(PACK_THREADS), 0, stream, lens, B, L, unpacked, perm, lsort, offs);
  }
  RG_LAUNCH_CHECK();
  return RG_OK;
}

// -------------------------------------------------------------- gather -----
// One workgroup per sorted row r; token (r, t) lives at offs[r] + t.
// reverse=1 stores the row's tokens in reverse time order (the backward
// direction of the bidirectional GRU reads its valid prefix back to front).
// E is a multiple of 4: one float4 per lane, a 512-B row per 32 lanes (E=128).
// 4 consecutive table values as fp32 (fp32 table: one 16-B load; fp16 table:
// one 8-B load + exact widening)
__device__ __forceinline__ f4 load4(const float* row, int c) { return reinterpret_cast<const f4*>(row)[c]; }
__device__ __forceinline__ f4 load4(const __half* row, int c) {
  const uint2 u = reinterpret_cast<const uint2*>(row)[c];
  const __half2 a = *reinterpret_cast<const __half2*>(&u.x);
  const __half2 b = *reinterpret_cast<const __half2*>(&u.y);
  const float2 fa = __half22float2(a), fb = __half22float2(b);
  return f4{fa.x, fa.y, fb.x, fb.y};
}

template <typename TE>
__global__ __launch_bounds__(256) void k_gather(const int64_t* __restrict__ s, int L,
                                                const int32_t* __restrict__ perm,
                                                const int32_t* __restrict__ lsort,
                                                const int32_t* __restrict__ offs,
                                                const TE* __restrict__ emb, int64_t n_rows, int E,
                                                int reverse, int32_t* __restrict__ tok_id,
                                                float* __restrict__ X, int32_t* __restrict__ err) {
  const int r = blockIdx.x;
  const int b = perm[r];
  const int len = lsort[r];
  const int base = offs[r];
  const int v4 = E >> 2;
  const int total = len * v4;
  for (int e = threadIdx.x; e < total; e += blockDim.x) {
    int t = e / v4;
    int c = e - t * v4;
    int64_t id = s[(int64_t)b * L + (reverse ? len - 1 - t : t)];
    int tok = base + t;
    f4 val = {0.f, 0.f, 0.f, 0.f};
    const bool ok = id >= 0 && id < n_rows;  // nn.Embedding raises on such ids
    if (ok) val = load4(emb + id * E, c);
    reinterpret_cast<f4*>(X + (int64_t)tok * E)[c] = val;
    if (c == 0) {
      tok_id[tok] = ok ? (int32_t)id : -1;
      if (!ok && err) atomicOr(err, 1);
    }
  }
}

// Compile-time-E variant (E ∈ {32, 64, 128, 256}, L <= GW_MAXL): a workgroup
// takes GW_ROWS sorted rows (two long, two short when B % 4 == 0; else
// consecutive ones), each row's tokens at its own packed range.  Three dependent memory steps
// per workgroup: the rows' (perm, length, offset), their item ids (into LDS),
// then every table row of the range — a lane issues all of its (up to U) row
// loads before any store, so up to GW_FLIGHT random 512-B rows are in flight
// per workgroup (the table rows are random: latency, not bandwidth, is what a
// lane waits on; 128 in flight measured 0.3 µs faster than 64 at C2, the next
// group's loads issued under this group's stores no faster; 8 rows per
// workgroup 12.5 -> 16 µs, 2 rows slower too).  V4 = E/4 lanes
// per token row.
//
// Sampled steps (rg_gather_neg) put the negatives' row gather in the same
// launch: the first np.nwg workgroups draw the S negatives and write their
// ids, biases, fp32 rows and fragment-order bf16 planes (common.h NegPrep)
// while the rest gather the embedding rows.
constexpr int GW_ROWS = 4;
constexpr int GW_FLIGHT = 128;
constexpr int GW_MAXL = 64;

// one thread per (negative, 8-value group): a wave covers 32 negatives × 2
// groups = one 16-deep slice, so each of its three plane stores is one
// contiguous 1 KB fragment (S % 32 == 0)
__device__ __forceinline__ void neg_prep(const NegPrep& np, int bid) {
  const int G = np.HF >> 3, NS = np.HF >> 4;
  const int64_t i = (int64_t)bid * 256 + threadIdx.x;
  if (i >= (int64_t)np.S * G) return;
  const int blk = (int)(i / (32 * G));
  const int rem = (int)(i - (int64_t)blk * 32 * G);
  const int x = blk * 32 + (rem & 31), g = rem >> 5;
  const int id = draw_id(np.seed, np.counter, np.S, x, np.A);
  const float* src = np.W + (int64_t)id * np.HF + 8 * g;
  const f4 lo = *reinterpret_cast<const f4*>(src);
  const f4 hi = *reinterpret_cast<const f4*>(src + 4);
  float* dst = np.Wg + (int64_t)x * np.HF + 8 * g;
  *reinterpret_cast<f4*>(dst) = lo;
  *reinterpret_cast<f4*>(dst + 4) = hi;
  const int lane = (g & 1) * 32 + (x & 31);
  if (np.wfmt) {
    f4* wf = reinterpret_cast<f4*>(np.Wp);
    wf[frag_idx(blk, g >> 1, 0, lane, NS)] = lo;
    wf[frag_idx(blk, g >> 1, 1, lane, NS)] = hi;
    if (g == 0) {
      np.ids[x] = id;
      np.bg[x] = np.bias[id];
    }
    return;
  }
  bf16x8 p0, p1, p2;
  split3x8(lo, hi, p0, p1, p2);
  np.Wp[plane_idx(blk, g >> 1, 0, lane, NS)] = p0;
  np.Wp[plane_idx(blk, g >> 1, 1, lane, NS)] = p1;
  np.Wp[plane_idx(blk, g >> 1, 2, lane, NS)] = p2;
  if (g == 0) {
    np.ids[x] = id;
    np.bg[x] = np.bias[id];
  }
}

template <typename TE, int E>
__global__ __launch_bounds__(256) void k_gather_e(const int64_t* __restrict__ s, int B, int L,
                                                  const int32_t* __restrict__ perm,
                                                  const int32_t* __restrict__ lsort,
                                                  const int32_t* __restrict__ offs,
                                                  const TE* __restrict__ emb, int64_t n_rows, int reverse,
                                                  int32_t* __restrict__ tok_id, float* __restrict__ X,
                                                  int32_t* __restrict__ err, NegPrep np) {
  constexpr int V4 = E / 4;
  constexpr int TPP = 256 / V4;                       // tokens per pass of the workgroup
  constexpr int FLT = E >= 256 ? GW_FLIGHT / 2 : GW_FLIGHT;   // rows in flight (64 VGPRs of f4 per lane)
  constexpr int U = FLT / TPP;                        // passes whose loads issue together
  __shared__ int ids[GW_ROWS * GW_MAXL], dsts[GW_ROWS * GW_MAXL];
  __shared__ int rb[GW_ROWS], rl[GW_ROWS], ro[GW_ROWS];
  if ((int)blockIdx.x < np.nwg) {
    neg_prep(np, blockIdx.x);
    return;
  }
  const int tid = threadIdx.x;
  // B % 4 == 0: workgroup k takes sorted rows 2k, 2k + 1 (long) and B − 2 − 2k,
  // B − 1 − 2k (short), so every workgroup gathers about the mean token count
  // (four consecutive sorted rows: 4 to 4·L tokens); the longest pairs still
  // dispatch first
  constexpr int GH = GW_ROWS / 2;
  const int k = (int)blockIdx.x - np.nwg;
  const bool pair = B % GW_ROWS == 0;
  const int r0 = k * GW_ROWS;
  const int nr = pair ? GW_ROWS : min(GW_ROWS, B - r0);
  if (tid < nr) {
    const int r = !pair ? r0 + tid : tid < GH ? GH * k + tid : B - GH * (k + 1) + tid - GH;
    rb[tid] = perm[r];
    rl[tid] = lsort[r];
    ro[tid] = offs[r];   // packed position of the row's token 0
  }
  __syncthreads();
  int pre[GW_ROWS];   // workgroup token index where row j starts
  int ntok = 0;
#pragma unroll
  for (int q = 0; q < GW_ROWS; ++q) {
    pre[q] = q < nr ? ntok : INT32_MAX;
    ntok += q < nr ? rl[q] : 0;
  }
  // item ids of every (row, t) and its packed position
  for (int i = tid; i < ntok; i += 256) {
    int j = 0;
#pragma unroll
    for (int q = 1; q < GW_ROWS; ++q) j += i >= pre[q];
    const int t = i - pre[j], len = rl[j];
    const int64_t id = s[(int64_t)rb[j] * L + (reverse ? len - 1 - t : t)];
    ids[i] = (id >= 0 && id < n_rows) ? (int32_t)id : -1;   // nn.Embedding raises on such ids
    dsts[i] = ro[j] + t;
  }
  __syncthreads();
  const int c = tid % V4, t0 = tid / V4;
  for (int i0 = t0; i0 < ntok; i0 += FLT) {
    f4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + TPP * u;
      v[u] = f4{0.f, 0.f, 0.f, 0.f};
      if (i < ntok && ids[i] >= 0) v[u] = load4(emb + (int64_t)ids[i] * E, c);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + TPP * u;
      if (i < ntok) {
        const int d = dsts[i];
        reinterpret_cast<f4*>(X + (int64_t)d * E)[c] = v[u];
        if (c == 0) {
          tok_id[d] = ids[i];
          if (ids[i] < 0 && err) atomicOr(err, 1);
        }
      }
    }
  }
}

template <typename TE>
static bool launch_gather_e(const int64_t* s, int B, int L, const int32_t* perm, const int32_t* lsort,
                            const int32_t* offs, const TE* emb, int64_t n_rows, int E, int reverse,
                            int32_t* tok_id, float* X, int32_t* err, const NegPrep& np, hipStream_t stream) {
  if (L > GW_MAXL) return false;
  const dim3 grid((unsigned)(np.nwg + (B + GW_ROWS - 1) / GW_ROWS));
#define GE(EV)                                                                                              \
  RG_TLAUNCH((k_gather_e<TE, EV>), grid, dim3(256), 0, stream, s, B, L, perm, lsort, offs, emb, n_rows,       \
             reverse, tok_id, X, err, np)
  switch (E) {
    case 32: GE(32); return true;
    case 64: GE(64); return true;
    case 128: GE(128); return true;
    case 256: GE(256); return true;
    default: return false;
  }
#undef GE
}

extern "C" int rg_gather(const int64_t* s, int B, int L, const int32_t* perm, const int32_t* lsort,
                         const int32_t* offs, const float* emb, int64_t n_rows, int E, int reverse,
                         int32_t* tok_id, float* X, int32_t* err, hipStream_t stream) {
  if (B <= 0 || (E & 3)) return RG_ERR_ARG;
  if (launch_gather_e(s, B, L, perm, lsort, offs, emb, n_rows, E, reverse, tok_id, X, err, NegPrep{}, stream)) {
    RG_LAUNCH_CHECK();
    return RG_OK;
  }
  hipLaunchKernelGGL(k_gather<float>, dim3(B), dim3(256), 0, stream, s, L, perm, lsort, offs, emb, n_rows, E,
                     reverse, tok_id, X, err);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

// Same gather from an fp16 copy of the table (config C5: fp16 embedding
// storage, fp32 master/Adam; rows widened exactly to fp32 on load).
extern "C" int rg_gather_h(const int64_t* s, int B, int L, const int32_t* perm, const int32_t* lsort,
                           const int32_t* offs, const uint16_t* emb16, int64_t n_rows, int E, int reverse,
                           int32_t* tok_id, float* X, int32_t* err, hipStream_t stream) {
  if (B <= 0 || (E & 3)) return RG_ERR_ARG;
  if (launch_gather_e(s, B, L, perm, lsort, offs, reinterpret_cast<const __half*>(emb16), n_rows, E, reverse, tok_id,
                      X, err, NegPrep{}, stream)) {
    RG_LAUNCH_CHECK();
    return RG_OK;
  }
  hipLaunchKernelGGL(k_gather<__half>, dim3(B), dim3(256), 0, stream, s, L, perm, lsort, offs,
                     reinterpret_cast<const __half*>(emb16), n_rows, E, reverse, tok_id, X, err);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

// The embedding gather of a sampled step with the negatives' row gather in the
// same launch (common.h NegPrep): draw `counter` of the counter-based stream
// (seed, S, A) -> ids[S], bg[S] = bias[ids], Wg[S][HF] = W[ids] and the rows'
// bf16 planes Wp (S·HF·6 bytes, fragment order) that rg_sampled_logits reads
// with draw = 2 — or, wfmt 1 (HF <= 128), the rows as fp32 fragments
// (S·HF·4 bytes, common.h frag_idx) for draw = 3.  emb16 != 0: the table is fp16 (rg_gather_h).  Needs the
// compile-time gather (E ∈ {32, 64, 128, 256}, L <= 64), S % 32 == 0,
// HF ∈ {32, 64, 128, 256}.
extern "C" int rg_gather_neg(const int64_t* s, int B, int L, const int32_t* perm, const int32_t* lsort,
                             const int32_t* offs, const void* emb, int emb16, int64_t n_rows, int E, int reverse,
                             int32_t* tok_id, float* X, int32_t* err, const float* W, const float* bias,
                             uint64_t seed, uint64_t counter, int64_t A, int S, int HF, int32_t* ids, float* Wg,
                             float* bg, void* Wp, int wfmt, hipStream_t stream) {
  if (B <= 0 || (E & 3) || L > GW_MAXL || !W || !bias || !ids || !Wg || !bg || !Wp) return RG_ERR_ARG;
  if (wfmt < 0 || wfmt > 1 || (wfmt == 1 && HF > 128)) return RG_ERR_ARG;
  if (S <= 0 || S % 32 || A <= 0 || A > INT32_MAX) return RG_ERR_ARG;
  if (E != 32 && E != 64 && E != 128 && E != 256) return RG_ERR_SHAPE;
  if (HF != 32 && HF != 64 && HF != 128 && HF != 256) return RG_ERR_SHAPE;
  NegPrep np{W, bias, ids, Wg, bg, reinterpret_cast<bf16x8*>(Wp), seed, counter, (uint64_t)A, S, HF,
             (int)(((int64_t)S * (HF / 8) + 255) / 256), wfmt};
  const bool ok = emb16 ? launch_gather_e(s, B, L, perm, lsort, offs, reinterpret_cast<const __half*>(emb), n_rows,
                                          E, reverse, tok_id, X, err, np, stream)
                        : launch_gather_e(s, B, L, perm, lsort, offs, reinterpret_cast<const float*>(emb), n_rows,
                                          E, reverse, tok_id, X, err, np, stream);
  if (!ok) return RG_ERR_SHAPE;
  RG_LAUNCH_CHECK();
  return RG_OK;
}
