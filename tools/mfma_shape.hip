// Calibration: the split-bf16 inner loop of the fused head (A planes in
// VGPRs, B planes from LDS by ds_read_b128, 6 plane products per fp32
// product, two waves per SIMD) on v_mfma_f32_32x32x16_bf16 vs
// v_mfma_f32_16x16x32_bf16 at equal FLOPs, random operands, whole chip.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I ../ikea-recommender-system_amd/csrc mfma_shape.hip -o mfma_shape
#include <cstdio>
#include <cstdlib>
#include "common.h"

__device__ __forceinline__ float rnd(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return ((int)(x & 0xFFFFFF) - 0x800000) * (1.0f / 0x800000);
}

// 32x32x16: wave = 32 rows x 32 cols, 8 k-slices of 16 per iteration
__global__ __launch_bounds__(512) void k32(int iters, float* out) {
  __shared__ bf16x8 lds[8 * 192];
  const int tid = threadIdx.x, lane = tid & 63;
  for (int e = tid; e < 8 * 192; e += 512) {
    f4 lo, hi;
    for (int i = 0; i < 4; ++i) { lo[i] = rnd(e * 8 + i + 7 * blockIdx.x); hi[i] = rnd(e * 8 + 4 + i + 7 * blockIdx.x); }
    bf16x8 p0, p1, p2;
    split3x8(lo, hi, p0, p1, p2);
    lds[e] = p0;
  }
  bf16x8 a0[8], a1[8], a2[8];
  for (int j = 0; j < 8; ++j) {
    f4 lo, hi;
    for (int i = 0; i < 4; ++i) { lo[i] = rnd(tid * 97 + j * 8 + i); hi[i] = rnd(tid * 97 + j * 8 + 4 + i); }
    split3x8(lo, hi, a0[j], a1[j], a2[j]);
  }
  __syncthreads();
  f16v acc = {};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      acc = mfma_split<6>(a0[j], a1[j], a2[j], lds[j * 192 + lane], lds[j * 192 + 64 + lane], lds[j * 192 + 128 + lane],
                          acc);
  }
  float s = 0.f;
  for (int r = 0; r < 16; ++r) s += acc[r];
  out[blockIdx.x * 512 + tid] = s;
}

// 16x16x32: wave = 2 x 2 blocks of 16 x 16, 4 k-slices of 32 per iteration
__global__ __launch_bounds__(512) void k16(int iters, float* out) {
  __shared__ bf16x8 lds[8 * 192];
  const int tid = threadIdx.x, lane = tid & 63;
  for (int e = tid; e < 8 * 192; e += 512) {
    f4 lo, hi;
    for (int i = 0; i < 4; ++i) { lo[i] = rnd(e * 8 + i + 7 * blockIdx.x); hi[i] = rnd(e * 8 + 4 + i + 7 * blockIdx.x); }
    bf16x8 p0, p1, p2;
    split3x8(lo, hi, p0, p1, p2);
    lds[e] = p0;
  }
  bf16x8 a0[2][4], a1[2][4], a2[2][4];
  for (int nb = 0; nb < 2; ++nb)
    for (int s = 0; s < 4; ++s) {
      f4 lo, hi;
      for (int i = 0; i < 4; ++i) {
        lo[i] = rnd(tid * 97 + (nb * 4 + s) * 8 + i);
        hi[i] = rnd(tid * 97 + (nb * 4 + s) * 8 + 4 + i);
      }
      split3x8(lo, hi, a0[nb][s], a1[nb][s], a2[nb][s]);
    }
  __syncthreads();
  f4 acc[2][2] = {};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int rb = 0; rb < 2; ++rb) {
        const bf16x8* hb = lds + (s * 2 + rb) * 192 + lane;
        const bf16x8 b0 = hb[0], b1 = hb[64], b2 = hb[128];
#pragma unroll
        for (int nb = 0; nb < 2; ++nb)
          acc[nb][rb] = mfma16_split<6>(a0[nb][s], a1[nb][s], a2[nb][s], b0, b1, b2, acc[nb][rb]);
      }
  }
  float s = 0.f;
  for (int nb = 0; nb < 2; ++nb)
    for (int rb = 0; rb < 2; ++rb)
      for (int r = 0; r < 4; ++r) s += acc[nb][rb][r];
  out[blockIdx.x * 512 + tid] = s;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 4000;
  const int grid = 256;
  float* out;
  if (hipMalloc(&out, grid * 512 * sizeof(float)) != hipSuccess) return 1;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  // MACs per wave per iteration: 32 x 32 x 128 x 6 (both forms)
  const double flops = 2.0 * 32 * 32 * 128 * 6 * (double)iters * 8 * grid;
  for (int rep = 0; rep < 3; ++rep) {
    for (int form = 0; form < 2; ++form) {
      for (int w = 0; w < 2; ++w) {
        if (form == 0) hipLaunchKernelGGL(k32, dim3(grid), dim3(512), 0, 0, iters, out);
        else hipLaunchKernelGGL(k16, dim3(grid), dim3(512), 0, 0, iters, out);
      }
      hipEventRecord(e0, 0);
      const int n = 5;
      for (int i = 0; i < n; ++i) {
        if (form == 0) hipLaunchKernelGGL(k32, dim3(grid), dim3(512), 0, 0, iters, out);
        else hipLaunchKernelGGL(k16, dim3(grid), dim3(512), 0, 0, iters, out);
      }
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float ms = 0.f;
      hipEventElapsedTime(&ms, e0, e1);
      ms /= n;
      printf("%s  %.3f ms  %.1f TFLOP/s bf16 executed (%.3f of 2500)\n", form ? "16x16x32" : "32x32x16", ms,
             flops / ms / 1e9, flops / ms / 1e9 / 2500.0);
      fflush(stdout);
    }
  }
  hipFree(out);
  return 0;
}
