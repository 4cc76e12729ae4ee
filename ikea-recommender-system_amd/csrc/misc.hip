// Small elementwise helpers on the step path (dropout mask, SMORL head
// combination) and the ABI version probe.
#include "common.h"

__global__ void k_mask_scale(const float* __restrict__ x, const float* __restrict__ mask, float scale, int64_t n,
                             float* __restrict__ y) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    y[i] = x[i] * (mask[i] * scale);
}

extern "C" int rg_mask_scale(const float* x, const float* mask, float scale, int64_t n, float* y,
                             hipStream_t stream) {
  if (n <= 0) return RG_ERR_ARG;
  int blocks = (int)((n + 255) / 256);
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(k_mask_scale, dim3(blocks), dim3(256), 0, stream, x, mask, scale, n, y);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

struct Ptr4 {
  const float* p[4];
  float w[4];
};

__global__ void k_weighted_sum(Ptr4 in, int nh, int64_t n, float* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float s = in.p[0][i] * in.w[0];
    for (int k = 1; k < nh; ++k) s = s + in.p[k][i] * in.w[k];
    out[i] = s;
  }
}

// X: HOST array of nh device pointers; w: HOST array of nh weights.
extern "C" int rg_weighted_sum(const float* const* X, const float* w, int nh, int64_t n, float* out,
                               hipStream_t stream) {
  if (nh <= 0 || nh > 4 || n <= 0) return RG_ERR_ARG;
  Ptr4 in{};
  for (int k = 0; k < nh; ++k) {
    in.p[k] = X[k];
    in.w[k] = w[k];
  }
  int blocks = (int)((n + 255) / 256);
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL(k_weighted_sum, dim3(blocks), dim3(256), 0, stream, in, nh, n, out);
  RG_LAUNCH_CHECK();
  return RG_OK;
}

extern "C" int rg_abi_version(void) { return 1; }
