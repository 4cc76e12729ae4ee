// Deterministic, atomic-free row scatter-add: G[id[i]] += src[i] over the
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
// 2. stable radix sort of (key, row) — hipCUB over rocPRIM — so equal ids
//    are consecutive and in row order.
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

// E / 64 (rounded up) floats per lane; lane c holds columns c, c + 64, ...
template <int EPL>
__global__ __launch_bounds__(256) void k_seg_blocks(const uint32_t* __restrict__ keys, const int32_t* __restrict__ rows,
                                                    int n_max, const float* __restrict__ src, int E,
                                                    float* __restrict__ G, int32_t* __restrict__ tags, int32_t tag,
                                                    float* __restrict__ part_first, float* __restrict__ part_last) {
  const int lane = threadIdx.x & 63;
  const int blk = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int p0 = blk * SB;
  if (p0 >= n_max) return;
  const int p1 = min(p0 + SB, n_max);
  const uint32_t before = p0 > 0 ? keys[p0 - 1] : SENT - 1;   // any value != keys[p0] when p0 == 0
  const uint32_t after = p1 < n_max ? keys[p1] : SENT;
  int p = p0;
  bool first = true;
  while (p < p1) {
    const uint32_t k = keys[p];
    if (k == SENT) break;   // sentinels sort last: the rest of the array is skipped rows
    int q = p + 1;
    while (q < p1 && keys[q] == k) ++q;
    // rows p .. q-1 in order, eight rows' loads in flight at a time
    float acc[EPL];
#pragma unroll
    for (int e = 0; e < EPL; ++e) acc[e] = 0.f;
    for (int r = p; r < q; r += 8) {
      float v[8][EPL];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const bool ok = r + u < q;
        const float* s = src + (int64_t)(ok ? rows[r + u] : 0) * E;
#pragma unroll
        for (int e = 0; e < EPL; ++e) {
          const int c = lane + 64 * e;
          v[u][e] = (ok && c < E) ? s[c] : 0.f;
        }
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int e = 0; e < EPL; ++e)
          if (r + u < q) acc[e] += v[u][e];
    }
    const bool open_left = first && k == before;   // run continues from the previous block
    const bool open_right = q == p1 && k == after;  // run continues into the next block
    if (!open_left && !open_right) {
      float* g = G + (int64_t)k * E;
#pragma unroll
      for (int e = 0; e < EPL; ++e) {
        const int c = lane + 64 * e;
        if (c < E) g[c] += acc[e];
      }
      if (lane == 0) tags[k] = tag;
    } else {
      // open_left: this is the block's first run; open_right: its last run
      // (both for a run covering the whole block)
#pragma unroll
      for (int e = 0; e < EPL; ++e) {
        const int c = lane + 64 * e;
        if (c < E) {
          if (open_left) part_first[(int64_t)blk * E + c] = acc[e];
          if (open_right) part_last[(int64_t)blk * E + c] = acc[e];
        }
      }
    }
    first = false;
    p = q;
  }
}

template <int EPL>
__global__ __launch_bounds__(256) void k_seg_cross(const uint32_t* __restrict__ keys, int n_max, int E,
                                                   float* __restrict__ G, int32_t* __restrict__ tags, int32_t tag,
                                                   const float* __restrict__ part_first,
                                                   const float* __restrict__ part_last) {
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
  for (int e = 0; e < EPL; ++e) {
    const int c = lane + 64 * e;
    acc[e] = c < E ? part_last[(int64_t)blk * E + c] : 0.f;
  }
  for (int b = blk + 1; b * SB < n_max && keys[b * SB] == k; ++b) {
#pragma unroll
    for (int e = 0; e < EPL; ++e) {
      const int c = lane + 64 * e;
      if (c < E) acc[e] += part_first[(int64_t)b * E + c];
    }
    const int q1 = min((b + 1) * SB, n_max);
    if (keys[q1 - 1] != k || (q1 < n_max && keys[q1] != k) || q1 == n_max) break;
  }
  float* g = G + (int64_t)k * E;
#pragma unroll
  for (int e = 0; e < EPL; ++e) {
    const int c = lane + 64 * e;
    if (c < E) g[c] += acc[e];
  }
  if (lane == 0) tags[k] = tag;
}

struct SegLayout {
  size_t keys_in, keys_out, vals_in, vals_out, part_first, part_last, sort_tmp, total, sort_bytes;
};

SegLayout seg_layout(int n_max, int E, int64_t n_rows) {
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

extern "C" int rg_scatter_rows(const int32_t* ids, const float* src, int E, const int32_t* n_ptr, int n_max,
                               int skip_id, float* G, int64_t n_rows, int32_t* tags, int32_t tag, void* work,
                               int64_t work_bytes, hipStream_t stream) {
  if (n_max <= 0 || E <= 0 || E > 512 || n_rows <= 0 || !ids || !src || !n_ptr || !G || !tags || !work)
    return RG_ERR_ARG;
  const SegLayout L = seg_layout(n_max, E, n_rows);
  if (work_bytes < (int64_t)L.total) return RG_ERR_ARG;
  char* w = static_cast<char*>(work);
  uint32_t* kin = (uint32_t*)(w + L.keys_in);
  uint32_t* kout = (uint32_t*)(w + L.keys_out);
  int32_t* vin = (int32_t*)(w + L.vals_in);
  int32_t* vout = (int32_t*)(w + L.vals_out);
  float* pf = (float*)(w + L.part_first);
  float* pl = (float*)(w + L.part_last);
  hipLaunchKernelGGL(k_seg_keys, dim3((n_max + 255) / 256), dim3(256), 0, stream, ids, n_ptr, n_max, n_rows, skip_id,
                     kin, vin);
  size_t tmp = L.sort_bytes;
  if (hipcub::DeviceRadixSort::SortPairs(w + L.sort_tmp, tmp, kin, kout, vin, vout, n_max, 0, key_bits(n_rows),
                                         stream) != hipSuccess)
    return RG_ERR_LAUNCH;
  const int nb = (n_max + SB - 1) / SB;
  const dim3 grid((unsigned)((nb + 3) / 4));
#define SEG(EPLV)                                                                                              \
  hipLaunchKernelGGL(k_seg_blocks<EPLV>, grid, dim3(256), 0, stream, kout, vout, n_max, src, E, G, tags, tag,  \
                     pf, pl);                                                                                  \
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
