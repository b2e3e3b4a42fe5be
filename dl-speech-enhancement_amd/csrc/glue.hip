// Step glue kernels: on-device noise mixing (dataloader/data_utils.py:12-22).
#include <algorithm>
#include <cmath>

#include "sel_common.h"

namespace sel {
namespace glue {

constexpr int kBlocks = 1024;

__global__ __launch_bounds__(256) void k_sumsq2(const float* __restrict__ a, const float* __restrict__ b,
                                                int64_t n, double* __restrict__ part) {
  __shared__ double red[16];
  double sa = 0.0, sb = 0.0;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
    const float x = a[i], y = b[i];
    sa += double(x) * x;
    sb += double(y) * y;
  }
  sa = block_sum<double>(sa, red);
  sb = block_sum<double>(sb, red);
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = sa;
    part[2 * blockIdx.x + 1] = sb;
  }
}

__global__ __launch_bounds__(256) void k_mix(const float* __restrict__ a, const float* __restrict__ b,
                                             int64_t n, const double* __restrict__ part, int np, float snr,
                                             float* __restrict__ out) {
  __shared__ float scale;
  __shared__ double red[16];
  double sa = 0.0, sb = 0.0;
  for (int i = threadIdx.x; i < np; i += blockDim.x) {
    sa += part[2 * i];
    sb += part[2 * i + 1];
  }
  sa = block_sum<double>(sa, red);
  sb = block_sum<double>(sb, red);
  if (threadIdx.x == 0) {
    // fp32 like the reference: speech.norm(p=2), noise.norm(p=2), math.exp(snr/10)
    const float sp = sqrtf(float(sa)), npw = sqrtf(float(sb));
    scale = float(std::exp(double(snr) / 10.0)) * npw / sp;
  }
  __syncthreads();
  const float s = scale;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x)
    out[i] = (s * a[i] + b[i]) / 2.f;
}

}  // namespace glue
}  // namespace sel

using namespace sel;
using namespace sel::glue;

extern "C" {

size_t sel_add_noise_workspace(int64_t n) {
  (void)n;
  return size_t(kBlocks) * 2 * sizeof(double);
}

int sel_add_noise(const float* speech, const float* noise, int64_t n, float snr, float* out, void* ws,
                  size_t ws_bytes, sel_stream_t stream) {
  SEL_REQUIRE(n > 0, SEL_ERR_ARG, "empty batch");
  SEL_REQUIRE(ws_bytes >= sel_add_noise_workspace(n), SEL_ERR_WORKSPACE, "workspace too small");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int nb = int(std::min<int64_t>(kBlocks, (n + 255) / 256));
  double* part = static_cast<double*>(ws);
  hipLaunchKernelGGL(k_sumsq2, dim3(nb), dim3(256), 0, s, speech, noise, n, part);
  SEL_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_mix, dim3(nb), dim3(256), 0, s, speech, noise, n, part, nb, snr, out);
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

}  // extern "C"
