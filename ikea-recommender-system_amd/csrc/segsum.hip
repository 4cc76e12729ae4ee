// Deterministic, atomic-free row scatter-add: G[id[i]] += src[i] (row i at
// src + i·lds, E floats) over the
// rows i < *n_ptr whose id is valid and not skip_id, and tags[id] = tag for
// every touched row.  It replaces atomic float adds (whose result depends on
// the arrival order as soon as a row gets three or more contributions — the
// Zipf-popular items get thousands per step) for
//   * the embedding gradient (nn.Embedding backward: index_add of the token
//     gradients, GRU4Rec/model.py:75, 146),
//   * the sampled head's row gradients (targets and negatives).
//
// 1. keys: id, or a sentinel above every id for skipped / invalid / padding
//    rows; values: the row index.
// 2. stable sort of (key, row) — hipCUB's radix sort over rocPRIM (below 1M
//    items it runs rocPRIM's block sort + merge passes; forcing the onesweep
//    radix passes measured slower at these sizes) — so equal ids are
//    consecutive and in row order.  With reuse_sort the previous call's sorted
//    order (same ids, same n_max) is used again: the sampled head scatters its
//    row gradients and its bias gradients over one sort.
// 3. one wave per 64-position block of the sorted array walks its block in
//    order, summing each maximal run of one id; a run wholly inside the block
//    is added to G here, the (at most two) runs crossing a block edge leave
//    their block-local sums as partials (first / last run of the block).
// 4. one wave per block that starts a crossing run adds that run's partials
//    block by block in order and writes G.
// Every row's sum is taken in one fixed order, so repeated runs are bitwise
// identical (checkpoint resume, parity across runs).
#include <hipcub/hipcub.hpp>

#include "common.h"

namespace {

constexpr uint32_t SENT = 0xFFFFFFFFu;
constexpr int SB = 64;   // sorted positions per block

int key_bits(int64_t n_rows) {
  int b = 1;
  while (b < 32 && ((int64_t)1 << b) <= n_rows) ++b;   // 2^b > n_rows: the sentinel's low bits sort last
  return b;
}

__global__ void k_seg_keys(const int32_t* __restrict__ ids, const int32_t* __restrict__ n_ptr, int n_max,
                           int64_t n_rows, int skip_id, uint32_t* __restrict__ keys, int32_t* __restrict__ vals) {
  rg_main_prio();
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_max) return;
  const int n = *n_ptr;
  uint32_t k = SENT;
  if (i < n) {
    const int32_t id = ids[i];
    if (id >= 0 && id < n_rows && id != skip_id) k = (uint32_t)id;
  }
  keys[i] = k;
  vals[i] = i;
}

// One wave per 64-position block of the sorted array, lane q = position q:
// each lane streams its own row in V-float chunks and a segmented inclusive
// scan across the lanes (fixed shuffle tree, so a fixed summation order) sums
// every run of equal ids at once; the lane ending a run adds the sum into G
// (all run ends of the block in parallel).  A run crossing a block edge
// leaves its block-local sum as a partial (first / last run of the block).
template <int V>
struct vec_t;
template <>
struct vec_t<1> {
  using T = float;
};
template <>
struct vec_t<4> {
  using T = f4;
};

// ASSIGN (the dedup exchange's per-unique-id sums, rg_shard_dedup_grads): G
// is a fresh buffer and every run is written exactly once — by the lane that
// closes it or, for a run crossing blocks, by k_seg_cross — so the sums are
// stored, not added; tags may be null
template <int V, bool ASSIGN = false>
__global__ __launch_bounds__(256) void k_seg_blocks(const uint32_t* __restrict__ keys, const int32_t* __restrict__ rows,
                                                    int n_max, const float* __restrict__ src, int E, int lds,
                                                    float* __restrict__ G, int32_t* __restrict__ tags, int32_t tag,
                                                    float* __restrict__ part_first, float* __restrict__ part_last) {
  rg_main_prio();
  using T = typename vec_t<V>::T;
  const int lane = threadIdx.x & 63;
  const int blk = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int p0 = blk * SB;
  if (p0 >= n_max) return;
  const int pos = p0 + lane;
  const uint32_t key = pos < n_max ? keys[pos] : SENT;
  const int row = pos < n_max ? rows[pos] : 0;
  const uint32_t before = p0 > 0 ? keys[p0 - 1] : SENT - 1;          // != keys[p0] when p0 == 0
  const uint32_t after = p0 + SB < n_max ? keys[p0 + SB] : SENT;
  uint32_t prev = __shfl_up(key, 1);
  if (lane == 0) prev = before;
  uint32_t next = __shfl_down(key, 1);
  if (lane == 63) next = after;
  const bool valid = key != SENT;
  const bool start = valid && key != prev;
  const bool end = valid && (key != next || lane == 63);
  const int first_end = __builtin_ctzll(__ballot(end) | (1ull << 63));
  const bool open_left = valid && key == before && lane <= first_end;  // run continued from the previous block
  const bool open_right = valid && lane == 63 && key == after;          // run continues into the next block
  const bool closed = end && !open_right && !(open_left && lane == first_end);
  if (__ballot(valid) == 0) return;   // a block of skipped rows only
  const T* r = reinterpret_cast<const T*>(src + (int64_t)row * lds);
  T* g = reinterpret_cast<T*>(G + (int64_t)key * E);
  const int nv = E / V;
  // the lane's row is read SU chunks at a time, all in flight before the
  // first is summed (one chunk per iteration waited for each load in turn:
  // C3's scatters 0.238 → 0.227 ms, profiles/r07/ab_seg_blocks_batched_loads.txt)
  constexpr int SU = 8;
  for (int c0 = 0; c0 < nv; c0 += SU) {
    T xs[SU];
#pragma unroll
    for (int u = 0; u < SU; ++u) xs[u] = (valid && c0 + u < nv) ? r[c0 + u] : T{};
#pragma unroll
    for (int u = 0; u < SU; ++u) {
      const int c = c0 + u;
      if (c >= nv) break;
      T x = xs[u];
      bool hd = start || lane == 0;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        T y;
        if constexpr (V == 4) {
          y = f4{__shfl_up(x[0], d), __shfl_up(x[1], d), __shfl_up(x[2], d), __shfl_up(x[3], d)};
        } else {
          y = __shfl_up(x, d);
        }
        const bool hy = __shfl_up((int)hd, d);
        if (lane >= d && !hd) x += y;
        if (lane >= d) hd = hd || hy;
      }
      if (closed) {
        if constexpr (ASSIGN) g[c] = x;
        else g[c] += x;
      }
      if (end && open_left && lane == first_end) reinterpret_cast<T*>(part_first + (int64_t)blk * E)[c] = x;
      if (open_right) reinterpret_cast<T*>(part_last + (int64_t)blk * E)[c] = x;
    }
  }
  if (closed && tags) tags[key] = tag;
}

// A run crossing block edges: the block where it starts adds its last-run
// partial and the first-run partials of the following blocks that continue
// it (their first keys equal the run's id), in block order.
template <int EPL, bool ASSIGN = false>
__global__ __launch_bounds__(256) void k_seg_cross(const uint32_t* __restrict__ keys, int n_max, int E,
                                                   float* __restrict__ G, int32_t* __restrict__ tags, int32_t tag,
                                                   const float* __restrict__ part_first,
                                                   const float* __restrict__ part_last) {
  rg_main_prio();
  const int lane = threadIdx.x & 63;
  const int blk = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int p0 = blk * SB, p1 = p0 + SB;
  if (p1 >= n_max) return;                 // no next block: nothing crosses
  const uint32_t k = keys[p1 - 1];
  if (k == SENT || keys[p1] != k) return;  // the block's last run does not cross
  // the run starts in this block unless it covers the whole block and continues from before
  if (p0 > 0 && keys[p0] == k && keys[p0 - 1] == k) return;
  float acc[EPL];
#pragma unroll
  for (int x = 0; x < EPL; ++x) {
    const int c = lane + 64 * x;
    acc[x] = c < E ? part_last[(int64_t)blk * E + c] : 0.f;
  }
  const int nb = (n_max + SB - 1) / SB;
  for (int b0 = blk + 1; b0 < nb; b0 += 64) {
    // blocks b0 .. b0+63 that continue the run form a prefix (the keys are sorted)
    const int b = b0 + lane;
    const uint64_t cont = __ballot(b < nb && keys[(int64_t)b * SB] == k);
    const int cnt = (~cont) ? __builtin_ctzll(~cont) : 64;
    for (int i = 0; i < cnt; i += 8) {
      float v[8][EPL];
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int x = 0; x < EPL; ++x) {
          const int c = lane + 64 * x;
          v[u][x] = (i + u < cnt && c < E) ? part_first[(int64_t)(b0 + i + u) * E + c] : 0.f;
        }
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int x = 0; x < EPL; ++x)
          if (i + u < cnt) acc[x] += v[u][x];
    }
    if (cnt < 64) break;
  }
  float* g = G + (int64_t)k * E;
#pragma unroll
  for (int x = 0; x < EPL; ++x) {
    const int c = lane + 64 * x;
    if (c < E) {
      if constexpr (ASSIGN) g[c] = acc[x];
      else g[c] += acc[x];
    }
  }
  if (lane == 0 && tags) tags[k] = tag;
}

struct SegLayout {
  size_t keys_in, keys_out, vals_in, vals_out, part_first, part_last, sort_tmp, total, sort_bytes;
};

// layouts are cached per (n_max, E, key bits): the hipCUB size query costs
// host time every call
struct SegKey {
  int n_max, E, bits;
};
constexpr int SEG_CACHE = 16;
thread_local SegKey seg_keys_[SEG_CACHE];
thread_local SegLayout seg_vals_[SEG_CACHE];
thread_local int seg_n_ = 0;

SegLayout seg_layout_uncached(int n_max, int E, int64_t n_rows);

SegLayout seg_layout(int n_max, int E, int64_t n_rows) {
  const int bits = key_bits(n_rows);
  for (int i = 0; i < seg_n_; ++i)
    if (seg_keys_[i].n_max == n_max && seg_keys_[i].E == E && seg_keys_[i].bits == bits) return seg_vals_[i];
  const SegLayout L = seg_layout_uncached(n_max, E, n_rows);
  const int slot = seg_n_ < SEG_CACHE ? seg_n_++ : (n_max + E) % SEG_CACHE;
  seg_keys_[slot] = SegKey{n_max, E, bits};
  seg_vals_[slot] = L;
  return L;
}

SegLayout seg_layout_uncached(int n_max, int E, int64_t n_rows) {
  SegLayout L{};
  const size_t nb = (size_t)(n_max + SB - 1) / SB;
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  size_t off = 0;
  L.keys_in = off; off += al(sizeof(uint32_t) * n_max);
  L.keys_out = off; off += al(sizeof(uint32_t) * n_max);
  L.vals_in = off; off += al(sizeof(int32_t) * n_max);
  L.vals_out = off; off += al(sizeof(int32_t) * n_max);
  L.part_first = off; off += al(sizeof(float) * nb * E);
  L.part_last = off; off += al(sizeof(float) * nb * E);
  size_t tmp = 0;
  hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                     (const int32_t*)nullptr, (int32_t*)nullptr, n_max, 0, key_bits(n_rows));
  L.sort_bytes = tmp;
  L.sort_tmp = off; off += al(tmp);
  L.total = off;
  return L;
}

}  // namespace

extern "C" int64_t rg_scatter_rows_work_bytes(int n_max, int E, int64_t n_rows) {
  if (n_max <= 0 || E <= 0 || n_rows <= 0) return RG_ERR_ARG;
  return (int64_t)seg_layout(n_max, E, n_rows).total;
}

extern "C" int rg_scatter_rows(const int32_t* ids, const float* src, int E, int lds, const int32_t* n_ptr, int n_max,
                               int skip_id, float* G, int64_t n_rows, int32_t* tags, int32_t tag, int reuse_sort,
                               void* work, int64_t work_bytes, hipStream_t stream) {
  if (n_max <= 0 || E <= 0 || E > 512 || lds < E || n_rows <= 0 || !ids || !src || !n_ptr || !G || !tags || !work)
    return RG_ERR_ARG;
  if (E % 4 == 0 && (lds % 4 || (reinterpret_cast<uintptr_t>(src) & 15))) return RG_ERR_ARG;   // f4 rows
  const SegLayout L = seg_layout(n_max, E, n_rows);
  if (work_bytes < (int64_t)L.total) return RG_ERR_ARG;
  char* w = static_cast<char*>(work);
  uint32_t* kin = (uint32_t*)(w + L.keys_in);
  uint32_t* kout = (uint32_t*)(w + L.keys_out);
  int32_t* vin = (int32_t*)(w + L.vals_in);
  int32_t* vout = (int32_t*)(w + L.vals_out);
  float* pf = (float*)(w + L.part_first);
  float* pl = (float*)(w + L.part_last);
  size_t tmp = L.sort_bytes;
  if (!reuse_sort) {
    hipLaunchKernelGGL(k_seg_keys, dim3((n_max + 255) / 256), dim3(256), 0, stream, ids, n_ptr, n_max, n_rows,
                       skip_id, kin, vin);
    if (hipcub::DeviceRadixSort::SortPairs(w + L.sort_tmp, tmp, kin, kout, vin, vout, n_max, 0, key_bits(n_rows),
                                           stream) != hipSuccess)
      return RG_ERR_LAUNCH;
  }
  const int nb = (n_max + SB - 1) / SB;
  const dim3 grid((unsigned)((nb + 3) / 4));
  if (E % 4 == 0)
    hipLaunchKernelGGL(k_seg_blocks<4>, grid, dim3(256), 0, stream, kout, vout, n_max, src, E, lds, G, tags, tag, pf,
                       pl);
  else
    hipLaunchKernelGGL(k_seg_blocks<1>, grid, dim3(256), 0, stream, kout, vout, n_max, src, E, lds, G, tags, tag, pf,
                       pl);
#define SEG(EPLV) \
  hipLaunchKernelGGL(k_seg_cross<EPLV>, grid, dim3(256), 0, stream, kout, n_max, E, G, tags, tag, pf, pl)
  if (E <= 64) {
    SEG(1);
  } else if (E <= 128) {
    SEG(2);
  } else if (E <= 256) {
    SEG(4);
  } else {
    SEG(8);
  }
#undef SEG
  RG_LAUNCH_CHECK();
  return RG_OK;
}

// ------------------------------------------------------ dedup exchange ----
// Row-sharded item table (csrc/emb_shard.hip): a trunk pass
// requests each DISTINCT id once.  A C2 batch's ~88K packed tokens carry
// ~1.7K distinct (Zipf) items, so the ids sent, the rows returned and the
// row-gradients sent back shrink ~50× against one per token.
//
// rg_shard_dedup (the forward, on the gather's critical path): no sort.  A
// mark byte per table row — byte id + 1 set to 1 for every token's id (an
// invalid id −1 is byte 0, so it comes first and goes with rank 0's group;
// plain byte stores: every token of an id writes the same value, where
// atomic bit-ORs serialised on the Zipf-hot words, 134 µs at C2) — and one
// exclusive scan of the popcounts of the marks' 32-bit words (a word holds
// four 0/1 bytes) rank the marked ids: u = rank(id + 1) in increasing id
// order.  The ids of one owner are a contiguous range, so that order is
// grouped by owner and
//   uslot[t]  = u of token t (rg_place_rows reads rows_in[uslot[t]]),
//   uids[u]   = the distinct ids in increasing order (−1 first, if any),
//   counts[o] = distinct ids owned by rank o (owner ⌈(id+1)·W/N1⌉ − 1):
//               rank past the owner's last byte minus rank of its first,
//   *nuniq    = U = rank(N1 + 1);
// five short launches (clear, mark, scan init + scan, write) over N1 bytes
// of marks and N1 of prefix instead of a multi-pass sort of the tokens.
// The write also leaves (u, t) key / value pairs in the work buffer for the
// backward.
// rg_shard_dedup_grads (the backward): a stable radix sort of those pairs
// by u (token order within one u) and gsend[u] = Σ of the token rows of u,
// summed in token order (k_seg_blocks / k_seg_cross over the sorted runs: a
// fixed order, so the step stays bitwise repeatable), stored once per u.
namespace {

// mark index of a token's id: id + 1, 0 for an invalid id (outside [0, N1))
__device__ __forceinline__ int dd_index(int32_t id, int64_t N1) { return id >= 0 && id < N1 ? id + 1 : 0; }

__global__ void k_dd_mark(const int32_t* __restrict__ tok_id, const int32_t* __restrict__ n_ptr, int n_max,
                          int64_t N1, uint8_t* __restrict__ marks) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_max || i >= *n_ptr) return;
  marks[dd_index(tok_id[i], N1)] = 1;   // (same value from every token of an id)
}

struct Popc {
  __host__ __device__ int operator()(uint32_t x) const {
#ifdef __HIP_DEVICE_COMPILE__
    return __popc(x);
#else
    return __builtin_popcount(x);
#endif
  }
};

// marked indices below k (k <= N1 + 1; pos = exclusive prefix over the mark words)
__device__ __forceinline__ int dd_rank(const uint32_t* words, const int32_t* pos, int64_t k, int64_t nwords) {
  const int64_t w = k >> 2;
  if (w >= nwords) return pos[nwords - 1] + __popc(words[nwords - 1]);
  const int sh = 8 * (int)(k & 3);
  return pos[w] + (sh ? __popc(words[w] & ((1u << sh) - 1u)) : 0);
}

__global__ void k_dd_write(const int32_t* __restrict__ tok_id, const uint32_t* __restrict__ words,
                           const int32_t* __restrict__ pos, int64_t nwords, const int32_t* __restrict__ n_ptr,
                           int n_max, int64_t N1, int W, int32_t* __restrict__ uslot, int32_t* __restrict__ uids,
                           uint32_t* __restrict__ keys, int32_t* __restrict__ vals, int32_t* __restrict__ counts,
                           int32_t* __restrict__ nuniq) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (blockIdx.x == 0) {
    if (threadIdx.x < W) {   // owner o: ids [o·N1/W, (o+1)·N1/W) = mark indices (o·N1/W, (o+1)·N1/W]
      const int o = threadIdx.x;
      const int64_t hi = ((int64_t)(o + 1) * N1) / W, lo = ((int64_t)o * N1) / W;
      counts[o] = dd_rank(words, pos, hi + 1, nwords) - (o == 0 ? 0 : dd_rank(words, pos, lo + 1, nwords));
    }
    if (threadIdx.x == 0) *nuniq = dd_rank(words, pos, N1 + 1, nwords);
  }
  if (i >= n_max) return;
  vals[i] = i;
  if (i >= *n_ptr) {
    keys[i] = SENT;
    return;
  }
  const int k = dd_index(tok_id[i], N1);
  const int u = dd_rank(words, pos, k, nwords);
  uslot[i] = u;
  keys[i] = (uint32_t)u;
  uids[u] = k - 1;   // (same value from every token of an id)
}

// Host-routed dedup (rg_shard_dedup_ids): the batch's distinct ids come with
// it from the host (dist.distinct_ids, which the exchange's splits are counted
// from anyway), sorted, −1 first — the order k_dd_write gives.  map[k] = u for
// the U distinct mark indices k (only entries of this batch's ids are read
// afterwards, so the map is never cleared); the tail [T, n_max) of the
// backward's sort pairs gets the sentinel key.
__global__ void k_dd_map(const int32_t* __restrict__ uids, int U, int64_t N1, int32_t* __restrict__ map,
                         const int32_t* __restrict__ n_ptr, int n_max, uint32_t* __restrict__ keys,
                         int32_t* __restrict__ vals) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < U) map[dd_index(uids[i], N1)] = i;
  if (i < n_max && i >= *n_ptr) {
    keys[i] = SENT;
    vals[i] = i;
  }
}

// one workgroup per sorted row r (k_token_ids' layout, csrc/emb_shard.hip):
// packed token t = offs[r] + τ of s[perm[r]][τ]: tok_id[t] (−1 outside
// [0, N1), err), uslot[t] = its distinct index, and the backward's sort pair
// (keys[t], vals[t]) = (uslot[t], t)
__global__ __launch_bounds__(64) void k_dd_tokens(const int64_t* __restrict__ s, int L,
                                                  const int32_t* __restrict__ perm, const int32_t* __restrict__ lsort,
                                                  const int32_t* __restrict__ offs, int64_t N1,
                                                  const int32_t* __restrict__ map, int32_t* __restrict__ tok_id,
                                                  int32_t* __restrict__ uslot, uint32_t* __restrict__ keys,
                                                  int32_t* __restrict__ vals, int32_t* __restrict__ err) {
  const int r = blockIdx.x;
  const int b = perm[r], len = lsort[r], base = offs[r];
  for (int t = threadIdx.x; t < len; t += blockDim.x) {
    const int64_t id = s[(int64_t)b * L + t];
    const bool ok = id >= 0 && id < N1;
    const int u = map[ok ? id + 1 : 0];
    tok_id[base + t] = ok ? (int32_t)id : -1;
    uslot[base + t] = u;
    keys[base + t] = (uint32_t)u;
    vals[base + t] = base + t;
    if (!ok && err) atomicOr(err, 1);
  }
}

struct DedupLayout {
  size_t keys_in, keys_out, vals_in, vals_out, marks, pos, part_first, part_last, tmp, total, sort_bytes,
      scan_bytes;
  int64_t nwords;
  int bits;
};

DedupLayout dedup_layout(int n_max, int E, int64_t N1) {
  DedupLayout L{};
  const size_t nb = (size_t)(n_max + SB - 1) / SB;
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  size_t off = 0;
  L.keys_in = off; off += al(sizeof(uint32_t) * n_max);
  L.keys_out = off; off += al(sizeof(uint32_t) * n_max);
  L.vals_in = off; off += al(sizeof(int32_t) * n_max);
  L.vals_out = off; off += al(sizeof(int32_t) * n_max);
  L.nwords = (N1 + 1 + 3) / 4;   // mark bytes, four per word
  L.marks = off; off += al(sizeof(uint32_t) * L.nwords);
  L.pos = off; off += al(sizeof(int32_t) * L.nwords);
  L.part_first = off; off += al(sizeof(float) * nb * E);
  L.part_last = off; off += al(sizeof(float) * nb * E);
  L.bits = key_bits(n_max);   // keys u < U <= n_max, the sentinel's low bits above them
  size_t ts = 0, tc = 0;
  hipcub::DeviceRadixSort::SortPairs(nullptr, ts, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                     (const int32_t*)nullptr, (int32_t*)nullptr, n_max, 0, L.bits);
  hipcub::TransformInputIterator<int, Popc, const uint32_t*> pc((const uint32_t*)nullptr, Popc());
  hipcub::DeviceScan::ExclusiveSum(nullptr, tc, pc, (int32_t*)nullptr, (int)L.nwords);
  L.sort_bytes = ts;
  L.scan_bytes = tc;
  L.tmp = off; off += al(ts > tc ? ts : tc);
  L.total = off;
  return L;
}

}  // namespace

extern "C" int64_t rg_shard_dedup_work_bytes(int n_max, int E, int64_t N1) {
  if (n_max <= 0 || E <= 0 || N1 <= 0 || N1 >= INT32_MAX) return RG_ERR_ARG;
  return (int64_t)dedup_layout(n_max, E, N1).total;
}

extern "C" int rg_shard_dedup(const int32_t* tok_id, const int32_t* n_ptr, int n_max, int64_t N1, int W, int E,
                              int32_t* uslot, int32_t* uids, int32_t* counts, int32_t* nuniq, void* work,
                              int64_t work_bytes, hipStream_t stream) {
  if (n_max <= 0 || N1 <= 0 || N1 >= INT32_MAX || W <= 0 || W > N1 || W > 256 || E <= 0 || !tok_id || !n_ptr ||
      !uslot || !uids || !counts || !nuniq || !work)
    return RG_ERR_ARG;
  const DedupLayout L = dedup_layout(n_max, E, N1);
  if (work_bytes < (int64_t)L.total) return RG_ERR_ARG;
  char* w = static_cast<char*>(work);
  uint32_t* bits = (uint32_t*)(w + L.marks);
  int32_t* pos = (int32_t*)(w + L.pos);
  const dim3 g((unsigned)((n_max + 255) / 256));
  if (hipMemsetAsync(bits, 0, sizeof(uint32_t) * L.nwords, stream) != hipSuccess) return RG_ERR_LAUNCH;
  hipLaunchKernelGGL(k_dd_mark, g, dim3(256), 0, stream, tok_id, n_ptr, n_max, N1, (uint8_t*)bits);
  size_t tc = L.scan_bytes;
  hipcub::TransformInputIterator<int, Popc, const uint32_t*> pc(bits, Popc());
  if (hipcub::DeviceScan::ExclusiveSum(w + L.tmp, tc, pc, pos, (int)L.nwords, stream) != hipSuccess)
    return RG_ERR_LAUNCH;
  hipLaunchKernelGGL(k_dd_write, g, dim3(256), 0, stream, tok_id, bits, pos, L.nwords, n_ptr, n_max, N1, W, uslot,
                     uids, (uint32_t*)(w + L.keys_in), (int32_t*)(w + L.vals_in), counts, nuniq);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

// rg_shard_dedup with the distinct ids given (sorted, −1 first: uids[0, U))
// and k_token_ids fused in: two launches instead of six (memset, mark, scan
// init + scan, write, token ids).  Same uslot / tok_id / sort pairs; the
// counts and U are the host's.  map: N1 + 1 int32 (one per pass in flight).
extern "C" int rg_shard_dedup_ids(const int64_t* s, int B, int L, const int32_t* perm, const int32_t* lsort,
                                  const int32_t* offs, const int32_t* n_ptr, int n_max, int64_t N1,
                                  const int32_t* uids, int U, int32_t* map, int32_t* tok_id, int32_t* uslot,
                                  int32_t* err, int E, void* work, int64_t work_bytes, hipStream_t stream) {
  if (B <= 0 || L <= 0 || n_max <= 0 || N1 <= 0 || N1 >= INT32_MAX || U < 0 || U > n_max + 1 || E <= 0 || !s ||
      !perm || !lsort || !offs || !n_ptr || !map || !tok_id || !uslot || !work || (U > 0 && !uids))
    return RG_ERR_ARG;
  const DedupLayout Ly = dedup_layout(n_max, E, N1);
  if (work_bytes < (int64_t)Ly.total) return RG_ERR_ARG;
  char* w = static_cast<char*>(work);
  uint32_t* keys = (uint32_t*)(w + Ly.keys_in);
  int32_t* vals = (int32_t*)(w + Ly.vals_in);
  const int nthr = U > n_max ? U : n_max;
  hipLaunchKernelGGL(k_dd_map, dim3((unsigned)((nthr + 255) / 256)), dim3(256), 0, stream, uids, U, N1, map, n_ptr,
                     n_max, keys, vals);
  hipLaunchKernelGGL(k_dd_tokens, dim3(B), dim3(64), 0, stream, s, L, perm, lsort, offs, N1, map, tok_id, uslot,
                     keys, vals, err);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_shard_dedup_grads(const float* src, int E, int n_max, int64_t N1, float* gsend, void* work,
                                    int64_t work_bytes, hipStream_t stream) {
  if (n_max <= 0 || E <= 0 || E > 512 || (E & 3) || N1 <= 0 || !src || !gsend || !work) return RG_ERR_ARG;
  const DedupLayout L = dedup_layout(n_max, E, N1);
  if (work_bytes < (int64_t)L.total) return RG_ERR_ARG;
  char* w = static_cast<char*>(work);
  uint32_t* ukeys = (uint32_t*)(w + L.keys_out);
  int32_t* vout = (int32_t*)(w + L.vals_out);
  size_t ts = L.sort_bytes;
  if (hipcub::DeviceRadixSort::SortPairs(w + L.tmp, ts, (const uint32_t*)(w + L.keys_in), ukeys,
                                         (const int32_t*)(w + L.vals_in), vout, n_max, 0, L.bits, stream) != hipSuccess)
    return RG_ERR_LAUNCH;
  float* pf = (float*)(w + L.part_first);
  float* pl = (float*)(w + L.part_last);
  const int nb = (n_max + SB - 1) / SB;
  const dim3 grid((unsigned)((nb + 3) / 4));
  hipLaunchKernelGGL((k_seg_blocks<4, true>), grid, dim3(256), 0, stream, ukeys, vout, n_max, src, E, E, gsend,
                     (int32_t*)nullptr, 0, pf, pl);
#define SEGA(EPLV)                                                                                                \
  hipLaunchKernelGGL((k_seg_cross<EPLV, true>), grid, dim3(256), 0, stream, ukeys, n_max, E, gsend, (int32_t*)nullptr, \
                     0, pf, pl)
  if (E <= 64) {
    SEGA(1);
  } else if (E <= 128) {
    SEGA(2);
  } else if (E <= 256) {
    SEGA(4);
  } else {
    SEGA(8);
  }
#undef SEGA
  RG_LAUNCH_CHECK();
  return RG_OK;
}
