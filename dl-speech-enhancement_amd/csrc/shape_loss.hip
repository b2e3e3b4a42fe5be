// Waveform shape loss (losses/waveform_loss.py:15-74): per window length w,
// L1(maxpool_w(|y_hat|), maxpool_w(|y|)) with MaxPool1d(w) (stride w, no
// padding, floor: the T % w tail is dropped), averaged over the window lengths.
// Forward: one thread per (row, window) pair computes both maxima (the first
// maximum wins, like MaxPool1d's index), |difference| into deterministic
// per-block fp64 partials, and keeps the argmax and the sign of the difference
// for the backward.  Backward: each window scatters its gradient to its argmax
// (windows of one length are disjoint: no atomics); lengths accumulate.
#include <algorithm>
#include <cmath>

#include "sel_common.h"

namespace sel {
namespace shape {

__global__ __launch_bounds__(256) void k_shape_fwd(const float* __restrict__ yh, const float* __restrict__ y,
                                                   int64_t rows, int64_t T, int w, int64_t nwin,
                                                   int32_t* __restrict__ arg, float* __restrict__ sgn,
                                                   double* __restrict__ part) {
  __shared__ double red[16];
  double acc = 0.0;
  const int64_t total = rows * nwin;
  for (int64_t id = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; id < total;
       id += int64_t(gridDim.x) * blockDim.x) {
    const int64_t r = id / nwin, k = id - r * nwin;
    const float* ph = yh + r * T + k * w;
    const float* py = y + r * T + k * w;
    float mh = -1.f, my = -1.f;
    int am = 0;
    for (int i = 0; i < w; ++i) {
      const float a = fabsf(ph[i]), b = fabsf(py[i]);
      if (a > mh) {  // strictly greater: the first maximum is kept
        mh = a;
        am = i;
      }
      my = fmaxf(my, b);
    }
    const float d = mh - my;
    acc += double(fabsf(d));
    arg[id] = am;
    sgn[id] = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
  }
  const double s = block_sum<double>(acc, red);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

__global__ void k_shape_finish(const double* __restrict__ part, int np, double inv_n, float* __restrict__ out) {
  __shared__ double red[16];
  double s = 0.0;
  for (int i = threadIdx.x; i < np; i += blockDim.x) s += part[i];
  s = block_sum<double>(s, red);
  if (threadIdx.x == 0) out[0] = float(s * inv_n);
}

// g_yh[argmax] += g * sign(d) * sign(y_hat[argmax]) / (rows * nwin); g read on device
__global__ __launch_bounds__(256) void k_shape_bwd(const float* __restrict__ yh, int64_t rows, int64_t T, int w,
                                                   int64_t nwin, const int32_t* __restrict__ arg,
                                                   const float* __restrict__ sgn, const float* __restrict__ g_out,
                                                   float gmul, float* __restrict__ g_yh) {
  const int64_t total = rows * nwin;
  const float g = g_out[0] * gmul;
  for (int64_t id = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; id < total;
       id += int64_t(gridDim.x) * blockDim.x) {
    const int64_t r = id / nwin, k = id - r * nwin;
    const int64_t e = r * T + k * w + arg[id];
    const float v = yh[e];
    const float sv = v > 0.f ? 1.f : (v < 0.f ? -1.f : 0.f);  // d|v|/dv, 0 at 0
    g_yh[e] += g * sgn[id] * sv;
  }
}

constexpr int kBlocks = 1024;

}  // namespace shape
}  // namespace sel

using namespace sel;
using namespace sel::shape;

extern "C" {

size_t sel_shape_loss_workspace(int64_t rows, int64_t T, int win) {
  (void)rows;
  (void)T;
  (void)win;
  return size_t(kBlocks) * sizeof(double);
}

int sel_shape_loss_fwd(const float* y_hat, const float* y, int64_t rows, int64_t T, int win, int32_t* argidx,
                       float* dsign, float* out, void* ws, size_t ws_bytes, sel_stream_t stream) {
  SEL_REQUIRE(rows > 0 && T > 0 && win > 0 && T >= win, SEL_ERR_ARG, "bad shape loss input (%lld, %lld, w=%d)",
              (long long)rows, (long long)T, win);
  SEL_REQUIRE(ws_bytes >= sel_shape_loss_workspace(rows, T, win), SEL_ERR_WORKSPACE, "workspace too small");
  const int64_t nwin = T / win;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int nb = int(std::min<int64_t>(kBlocks, (rows * nwin + 255) / 256));
  double* part = static_cast<double*>(ws);
  hipLaunchKernelGGL(k_shape_fwd, dim3(nb), dim3(256), 0, s, y_hat, y, rows, T, win, nwin, argidx, dsign, part);
  SEL_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_shape_finish, dim3(1), dim3(256), 0, s, part, nb, 1.0 / double(rows * nwin), out);
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

int sel_shape_loss_bwd(const float* y_hat, int64_t rows, int64_t T, int win, const int32_t* argidx,
                       const float* dsign, const float* g_out, float g_mul, float* g_yhat, sel_stream_t stream) {
  SEL_REQUIRE(rows > 0 && T > 0 && win > 0 && T >= win, SEL_ERR_ARG, "bad shape loss input");
  const int64_t nwin = T / win;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int nb = int(std::min<int64_t>(4096, (rows * nwin + 255) / 256));
  hipLaunchKernelGGL(k_shape_bwd, dim3(nb), dim3(256), 0, s, y_hat, rows, T, win, nwin, argidx, dsign, g_out,
                     g_mul / float(rows * nwin), g_yhat);
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

}  // extern "C"
