// Shared helpers for the gfx950 (MI355X / CDNA4) kernels of the GRU4Rec /
// SQN / SMORL training path.  Wave64 everywhere; fp32 data; exact-f32 MFMA
// (v_mfma_f32_32x32x2_f32 / v_mfma_f32_16x16x4_f32, bitwise an fmaf chain).
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

// Kernel-exact timing (bench.py's single-kernel regions, rg_timing_events):
// when armed, the next RG_TLAUNCH launch records the two events at its
// dispatch packet's start / end (hipExtLaunchKernelGGL) and disarms them, so
// the measured duration excludes the event-record commands around it.
extern hipEvent_t rg_tev0, rg_tev1;
#define RG_TLAUNCH(K, G, BK, SH, ST, ...)                                                \
  do {                                                                                   \
    if (rg_tev0 != nullptr) {                                                            \
      hipExtLaunchKernelGGL(K, G, BK, SH, ST, rg_tev0, rg_tev1, 0u, __VA_ARGS__);        \
      rg_tev0 = rg_tev1 = nullptr;                                                       \
    } else {                                                                             \
      hipLaunchKernelGGL(K, G, BK, SH, ST, __VA_ARGS__);                                 \
    }                                                                                    \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));

#define RG_OK 0
// items per online-softmax (max, Σexp, argmax) partial of the head forward
#define RG_PBLK 32
#define RG_ERR_ARG (-1)
#define RG_ERR_LAUNCH (-2)
#define RG_ERR_SHAPE (-3)

#define RG_LAUNCH_CHECK()                                  \
  do {                                                     \
    hipError_t e_ = hipGetLastError();                     \
    if (e_ != hipSuccess) return RG_ERR_LAUNCH;            \
  } while (0)

__device__ __forceinline__ f4 mfma16(float a, float b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f16v mfma32(float a, float b, f16v c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// Row of a 32x32 MFMA accumulator register r held by lane half h (= lane>>5).
__device__ __forceinline__ int acc32_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

__device__ __forceinline__ float sigmoidf_ref(float x) {
  // torch CPU sigmoid: 1 / (1 + exp(-x))
  return 1.0f / (1.0f + expf(-x));
}

// online (max, sum-exp, argmax) merge; ties keep the smaller index
struct LseState {
  float m;
  float s;
  int arg;
};
__device__ __forceinline__ void lse_merge(float& m, float& s, int& arg, float m2, float s2, int arg2) {
  if (m2 > m || (m2 == m && arg2 < arg)) {
    float nm = m2;
    s = s * expf(m - nm) + s2;
    m = nm;
    arg = arg2;
  } else {
    s = s + s2 * expf(m2 - m);
  }
}

__device__ __forceinline__ int wave_lane() { return threadIdx.x & 63; }

// torch.optim.Adam (defaults: amsgrad=False, weight_decay=0, maximize=False),
// _single_tensor_adam op by op:
//   exp_avg.lerp_(grad, 1-β1)          -> m + w1*(g - m)         (weight < 0.5 branch)
//   exp_avg_sq.mul_(β2).addcmul_(g, g, value=1-β2)
//   denom = (exp_avg_sq.sqrt() / bias_correction2_sqrt).add_(eps)
//   param.addcdiv_(exp_avg, denom, value=-step_size)
// Scalars arrive already rounded to fp32 the way the CPU kernels see them.
struct AdamArgs {
  float w1;        // 1 - beta1
  float beta2;     // beta2
  float c2;        // 1 - beta2
  float bc2_sqrt;  // sqrt(1 - beta2^t)
  float eps;
  float neg_step;  // -lr / (1 - beta1^t)
};

// Every rounding is explicit (fp contraction off; lerp as ATen's vectorised
// fmadd), so the update is the same fp32 sequence in every kernel that inlines
// it — the eager sweeps, the fused head epilogues and the catch-up Adam's
// replays (csrc/optim.hip rg_lazy_*), which must agree bit for bit.
__device__ __forceinline__ void adam_elem(float& p, float& m, float& v, float g, const AdamArgs& a) {
#pragma clang fp contract(off)
  m = __builtin_fmaf(a.w1, g - m, m);
  v = v * a.beta2;
  v = v + a.c2 * g * g;
  const float denom = sqrtf(v) / a.bc2_sqrt + a.eps;
  p = p + a.neg_step * (m / denom);
}

// ---- split-bf16 fp32 GEMM (precision "f32x9" / "f32x6") ----
// x = x0 + x1 + x2 EXACTLY for a normal fp32 x: x0 = bf16(x) (RNE), x1 =
// bf16(x − x0), x2 = x − x0 − x1 (≤ 8 significant bits left, so it is a bf16).
// A product a·b is then Σ_{p,q} a_p·b_q, every a_p·b_q exact in the fp32
// accumulator of v_mfma_f32_32x32x16_bf16.  f32x9 keeps all nine terms (the
// products are exact; only the fp32 accumulation rounds, as in an fmaf
// chain); f32x6 drops the three with p+q ≥ 3 (|a1·b2|, |a2·b1| ≤ 2^-24·|ab|,
// |a2·b2| ≤ 2^-32·|ab|: below fp32's unit roundoff per product).
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// `terms` code of the fused head (rg_flash_*) beyond 6 / 9 (every
// contraction at that many plane products): precision "f32x6d3" — the logits
// (S = W·hᵀ, both passes) and dW at 6 products, pass 1's O = P·W (→ dh) at 3
#define RG_TERMS_X6D3 636

__device__ __forceinline__ f16v mfma32bf(bf16x8 a, bf16x8 b, f16v c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// raw buffer resource over `base` (SGPRs; num_records = 2^31 - 1 bytes) and
// a 16-byte buffer -> LDS DMA: lane reads base + voff + soff, LDS address =
// wave-uniform base + 16·lane
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rg_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ void rg_blds16(__amdgpu_buffer_rsrc_t r, void* lds_wave_base, int voff, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds_wave_base, 16, voff,
                                           soff, 0, 0);
}

// Issue priority of the launch stream's short serial kernels over the side
// streams' VALU work (the catch-up replay, the head's pass 2); s_setprio is a
// SOPP instruction, it only changes the wave's issue arbitration (DESIGN §4d;
// the segmented scatter, the Adam updates, the direction sum: C4 +1 %, C2 / C3
// unchanged, same box, profiles/r07/ab_main_setprio.txt)
#ifndef RG_MAIN_PRIO
#define RG_MAIN_PRIO 2
#endif
__device__ __forceinline__ void rg_main_prio() {
  if constexpr (RG_MAIN_PRIO > 0) __builtin_amdgcn_s_setprio(RG_MAIN_PRIO);
}

// 8 consecutive fp32 values -> their three bf16 planes
__device__ __forceinline__ void split3x8(const f4& lo, const f4& hi, bf16x8& p0, bf16x8& p1, bf16x8& p2) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const float x = i < 4 ? lo[i] : hi[i - 4];
    const __bf16 b0 = (__bf16)x;
    const float r1 = x - (float)b0;
    const __bf16 b1 = (__bf16)r1;
    const float r2 = r1 - (float)b1;
    p0[i] = b0;
    p1[i] = b1;
    p2[i] = (__bf16)r2;
  }
}

// split3x8 with the conversions paired explicitly (one v_cvt_pk_bf16_f32 per
// two values and plane) and the fp32 arithmetic scalar: the same RNE planes,
// bitwise.  For units built without SLP vectorisation (head_flash.hip), where
// the plain loop converts one value per instruction
__device__ __forceinline__ void split3x8_pair(const f4& lo, const f4& hi, bf16x8& p0, bf16x8& p1, bf16x8& p2) {
  typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
  typedef float fl2 __attribute__((ext_vector_type(2)));
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float xa = i < 2 ? lo[2 * i] : hi[2 * i - 4], xb = i < 2 ? lo[2 * i + 1] : hi[2 * i - 3];
    const bf2 b0 = __builtin_convertvector((fl2){xa, xb}, bf2);
    const uint32_t u0 = __builtin_bit_cast(uint32_t, b0);
    const float ra = xa - __uint_as_float(u0 << 16), rb = xb - __uint_as_float(u0 & 0xFFFF0000u);
    const bf2 b1 = __builtin_convertvector((fl2){ra, rb}, bf2);
    const uint32_t u1 = __builtin_bit_cast(uint32_t, b1);
    const float sa = ra - __uint_as_float(u1 << 16), sb = rb - __uint_as_float(u1 & 0xFFFF0000u);
    const bf2 b2 = __builtin_convertvector((fl2){sa, sb}, bf2);
    p0[2 * i] = b0.x; p0[2 * i + 1] = b0.y;
    p1[2 * i] = b1.x; p1[2 * i + 1] = b1.y;
    p2[2 * i] = b2.x; p2[2 * i + 1] = b2.y;
  }
}

// ---- sampled negatives (csrc/sampled.hip, csrc/pack_gather.hip) ----
// Counter-based uniform draw: negative s of draw `counter` is the high 64 bits
// of splitmix64(seed + φ·(counter·S + s + 1))·A — reproducible on the host.
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ int32_t draw_id(uint64_t seed, uint64_t counter, int S, int s, uint64_t A) {
  return (int32_t)__umul64hi(mix64(seed + 0x9E3779B97F4A7C15ull * (counter * (uint64_t)S + (uint64_t)s + 1ull)), A);
}
// Fragment-order plane buffer of 32-row blocks (the A operand of the sampled
// logits' v_mfma_f32_32x32x16_bf16): entry (block, 16-deep slice j, plane p,
// lane), lane (hh, n) = row n, k = 16j + 8hh .. +8, one 16-B bf16x8 each.
__device__ __forceinline__ int64_t plane_idx(int blk, int j, int p, int lane, int NS) {
  return (((int64_t)blk * NS + j) * 3 + p) * 64 + lane;
}
// The same blocks as fp32 fragments (rg_gather_neg wfmt 1, rg_sampled_logits
// draw 3): entry (block, slice j, half q, lane) = one f4, lane (hh, n) = row n,
// k = 16j + 8hh + 4q .. +4 — two thirds of the planes' bytes, split in the
// logits kernel right before each slice's MFMAs.
__device__ __forceinline__ int64_t frag_idx(int blk, int j, int q, int lane, int NS) {
  return (((int64_t)blk * NS + j) * 2 + q) * 64 + lane;
}
// The negatives' row gather of a sampled step, done by extra workgroups of the
// embedding-gather launch (rg_gather_neg): ids, biases, fp32 rows (the
// backward's operands) and the rows' bf16 planes in fragment order (the
// logits' A operand, so rg_sampled_logits reads them as whole 1 KB
// wave-instructions instead of gathering 512-B rows itself).
struct NegPrep {
  const float* W;
  const float* bias;
  int32_t* ids;
  float* Wg;
  float* bg;
  bf16x8* Wp;   // wfmt 0: bf16 planes (plane_idx); 1: fp32 fragments (frag_idx)
  uint64_t seed, counter, A;
  int S, HF, nwg, wfmt;
};

// acc += Σ_terms a_p · b_q over one 16-wide k slice (NT = 9, 6 or 3 terms),
// smallest terms first.  NT = 3 keeps a0·b0, a0·b1, a1·b0 (dropped terms
// ≤ 3·2^-18·|ab|); only the fused head's O = P·W contraction (→ dh) uses it
// (precision "f32x6d3", RG_TERMS_X6D3), never logits or dW.
template <int NT>
__device__ __forceinline__ f16v mfma_split(const bf16x8& a0, const bf16x8& a1, const bf16x8& a2, const bf16x8& b0,
                                           const bf16x8& b1, const bf16x8& b2, f16v acc) {
  if (NT == 3) {
    acc = mfma32bf(a0, b1, acc);
    acc = mfma32bf(a1, b0, acc);
    return mfma32bf(a0, b0, acc);
  }
  if (NT == 9) {
    acc = mfma32bf(a2, b2, acc);
    acc = mfma32bf(a1, b2, acc);
    acc = mfma32bf(a2, b1, acc);
  }
  acc = mfma32bf(a0, b2, acc);
  acc = mfma32bf(a1, b1, acc);
  acc = mfma32bf(a2, b0, acc);
  acc = mfma32bf(a0, b1, acc);
  acc = mfma32bf(a1, b0, acc);
  acc = mfma32bf(a0, b0, acc);
  return acc;
}

// The same plane products on v_mfma_f32_16x16x32_bf16 (16×16 tile, k 32
// deep: operand lane l carries row / col l%16, k group l/16 (8 values);
// accumulator register i of lane l is C[4(l/16) + i][l%16]).  The fused head
// runs on this shape: in an LDS-fed split-bf16 loop at two waves per SIMD it
// sustains 0.84 of the bf16 peak against 0.73 for 32x32x16 at equal FLOPs
// (tools/mfma_shape.hip: the chip holds a higher clock).
//
// Operand planes of a matrix X (rows × HF) in that shape, 16-B entries:
//   K-planes  [x/32][s < HF/32][blk < 2][p < 3][lane]: lane = 16·kg + n holds
//             X[32(x/32) + 16·blk + n][32s + 8kg + 0..7]        (k over features)
//   R-planes  [x/32][fb < HF/16][p < 3][lane]: lane = 16·kg + n holds
//             X[32(x/32) + kperm16(kg, e)][16fb + n], e = 0..7   (k over rows)
// kperm16: the k order in which an accumulator pair (rows 4kg + i of tile 0,
// 16 + 4kg + i of tile 1) feeds the next MFMA as its 32-deep operand.
__device__ __forceinline__ int kperm16(int kg, int e) { return (e & 3) + 4 * kg + 16 * (e >> 2); }
__device__ __forceinline__ int64_t kplane16(int64_t x, int g8, int HF) {   // entry of (row x, 8-value group g8), plane 0
  return ((((x >> 5) * (HF / 32) + (g8 >> 2)) * 2 + ((x >> 4) & 1)) * 3) * 64 + 16 * (g8 & 3) + (x & 15);
}
__device__ __forceinline__ f4 mfma16bf(bf16x8 a, bf16x8 b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
template <int NT>
__device__ __forceinline__ f4 mfma16_split(const bf16x8& a0, const bf16x8& a1, const bf16x8& a2, const bf16x8& b0,
                                          const bf16x8& b1, const bf16x8& b2, f4 acc) {
  if (NT == 1) return mfma16bf(a0, b0, acc);
  if (NT == 3) {
    acc = mfma16bf(a0, b1, acc);
    acc = mfma16bf(a1, b0, acc);
    return mfma16bf(a0, b0, acc);
  }
  if (NT == 9) {
    acc = mfma16bf(a2, b2, acc);
    acc = mfma16bf(a1, b2, acc);
    acc = mfma16bf(a2, b1, acc);
  }
  acc = mfma16bf(a0, b2, acc);
  acc = mfma16bf(a1, b1, acc);
  acc = mfma16bf(a2, b0, acc);
  acc = mfma16bf(a0, b1, acc);
  acc = mfma16bf(a1, b0, acc);
  acc = mfma16bf(a0, b0, acc);
  return acc;
}
