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

__global__ __launch_bounds__(256) void k_finish2(const double* __restrict__ part, int np, double* __restrict__ sums2) {
  __shared__ double red[16];
  double sa = 0.0, sb = 0.0;
  for (int i = threadIdx.x; i < np; i += blockDim.x) {
    sa += part[2 * i];
    sb += part[2 * i + 1];
  }
  sa = block_sum<double>(sa, red);
  sb = block_sum<double>(sb, red);
  if (threadIdx.x == 0) {
    sums2[0] = sa;
    sums2[1] = sb;
  }
}

__global__ __launch_bounds__(256) void k_mix2(const float* __restrict__ a, const float* __restrict__ b, int64_t n,
                                              const double* __restrict__ sums2, float snr, float* __restrict__ out) {
  const float sp = sqrtf(float(sums2[0])), npw = sqrtf(float(sums2[1]));
  const float s = float(std::exp(double(snr) / 10.0)) * npw / sp;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x)
    out[i] = (s * a[i] + b[i]) / 2.f;
}

// SNR (torchmetrics SignalNoiseRatio, zero_mean=False): one block per sample.
__global__ __launch_bounds__(256) void k_snr_sums(const float* __restrict__ p, const float* __restrict__ t, int64_t T,
                                                  double* __restrict__ sums) {
  __shared__ double red[16];
  const int64_t b = blockIdx.x;
  double st = 0.0, sd = 0.0;
  for (int64_t i = threadIdx.x; i < T; i += blockDim.x) {
    const float tv = t[b * T + i], d = tv - p[b * T + i];
    st += double(tv) * tv;
    sd += double(d) * d;
  }
  st = block_sum<double>(st, red);
  sd = block_sum<double>(sd, red);
  if (threadIdx.x == 0) {
    sums[2 * b] = st;
    sums[2 * b + 1] = sd;
  }
}

__global__ __launch_bounds__(256) void k_snr_finish(const double* __restrict__ sums, int64_t B, float* __restrict__ out) {
  __shared__ float red[16];
  const float eps = 1.1920928955078125e-07f;  // torch.finfo(float32).eps
  float v = 0.f;
  for (int64_t b = threadIdx.x; b < B; b += blockDim.x)
    v += 10.f * log10f((float(sums[2 * b]) + eps) / (float(sums[2 * b + 1]) + eps));
  v = block_sum<float>(v, red);
  if (threadIdx.x == 0) out[0] = v / float(B);
}

__global__ __launch_bounds__(256) void k_snr_bwd(const float* __restrict__ p, const float* __restrict__ t, int64_t B,
                                                 int64_t T, const double* __restrict__ sums,
                                                 const float* __restrict__ g, float* __restrict__ gp) {
  const float eps = 1.1920928955078125e-07f;
  const float gv = g[0] * (20.f / 2.302585092994046f) / float(B);
  const int64_t n = B * T;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
    const int64_t b = i / T;
    const float den = float(sums[2 * b + 1]) + eps;
    gp[i] = gv * (t[i] - p[i]) / den;
  }
}


// Adam update of many fp32 tensors in one launch (torch.optim.Adam semantics,
// L2 weight decay, no amsgrad / maximize; the arithmetic of torch's fused
// kernel: m = b1 m + (1 - b1) g, v = b2 v + (1 - b2) g g, p -= step_size m /
// (sqrt(v) / bc2_sqrt + eps)).  Block b of the launch -> tensor j by the block
// ranges in the argument; four elements per thread (16-B accesses where the
// tensor allows them).
constexpr int ADAM_MAXT = 48;
constexpr int ADAM_EPB = 1024;  // elements per block
struct AdamJobs {
  float* p[ADAM_MAXT];
  const float* g[ADAM_MAXT];
  float* m[ADAM_MAXT];
  float* v[ADAM_MAXT];
  int64_t n[ADAM_MAXT];
  int bstart[ADAM_MAXT + 1];
  int nt;
};

struct AdamConst {
  float b1, omb1, b2, omb2, eps, wd, step_size, bc2_sqrt;  // omb = 1 - beta, rounded once from double
};

__device__ __forceinline__ void adam_one(float& p, float g, float& m, float& v, const AdamConst& c) {
  const float b1 = c.b1, omb1 = c.omb1, b2 = c.b2, omb2 = c.omb2, eps = c.eps, wd = c.wd,
              step_size = c.step_size, bc2_sqrt = c.bc2_sqrt;
  if (wd != 0.f) g = g + wd * p;
  m = b1 * m + omb1 * g;
  v = b2 * v + omb2 * g * g;
  const float denom = sqrtf(v) / bc2_sqrt + eps;
  p = p - step_size * m / denom;
}

// Capturable form (sel_adam_step_many_dev): the step count and the learning
// rate live on the device, so a captured update stays correct on every replay.
// One thread advances the count and writes (step_size, bc2_sqrt), rounded to
// float from double exactly as the host form's caller does; the update kernel
// then reads them (stream order: no reader sees a half-advanced count).
__global__ void k_adam_consts(const float* __restrict__ lr, float* __restrict__ step, double b1, double b2,
                              float* __restrict__ out) {
  const float t = step[0] + 1.f;
  step[0] = t;
  out[0] = float(double(lr[0]) / (1.0 - pow(b1, double(t))));
  out[1] = float(sqrt(1.0 - pow(b2, double(t))));
}

template <bool DEV>
__global__ __launch_bounds__(256) void k_adam_many(AdamJobs aj, AdamConst c, const float* __restrict__ dc) {
  if constexpr (DEV) {
    c.step_size = dc[0];
    c.bc2_sqrt = dc[1];
  }
  int j = 0;
  while (j + 1 < aj.nt && int(blockIdx.x) >= aj.bstart[j + 1]) ++j;  // block-uniform
  const int64_t n = aj.n[j];
  const int64_t i0 = int64_t(int(blockIdx.x) - aj.bstart[j]) * ADAM_EPB + 4 * threadIdx.x;
  float* __restrict__ P = aj.p[j];
  const float* __restrict__ G = aj.g[j];
  float* __restrict__ M = aj.m[j];
  float* __restrict__ V = aj.v[j];
  const bool vec = ((reinterpret_cast<uintptr_t>(P) | reinterpret_cast<uintptr_t>(G) | reinterpret_cast<uintptr_t>(M) |
                     reinterpret_cast<uintptr_t>(V)) & 15) == 0;
  if (vec && i0 + 4 <= n) {
    float4 p = *reinterpret_cast<const float4*>(P + i0), g = *reinterpret_cast<const float4*>(G + i0);
    float4 m = *reinterpret_cast<const float4*>(M + i0), v = *reinterpret_cast<const float4*>(V + i0);
    adam_one(p.x, g.x, m.x, v.x, c);
    adam_one(p.y, g.y, m.y, v.y, c);
    adam_one(p.z, g.z, m.z, v.z, c);
    adam_one(p.w, g.w, m.w, v.w, c);
    *reinterpret_cast<float4*>(P + i0) = p;
    *reinterpret_cast<float4*>(M + i0) = m;
    *reinterpret_cast<float4*>(V + i0) = v;
  } else {
    for (int64_t i = i0; i < i0 + 4 && i < n; ++i) adam_one(P[i], G[i], M[i], V[i], c);
  }
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

int sel_sumsq2(const float* speech, const float* noise, int64_t n, double* sums2, void* ws, size_t ws_bytes,
               sel_stream_t stream) {
  SEL_REQUIRE(n > 0, SEL_ERR_ARG, "empty batch");
  SEL_REQUIRE(ws_bytes >= sel_add_noise_workspace(n), SEL_ERR_WORKSPACE, "workspace too small");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int nb = int(std::min<int64_t>(kBlocks, (n + 255) / 256));
  double* part = static_cast<double*>(ws);
  hipLaunchKernelGGL(k_sumsq2, dim3(nb), dim3(256), 0, s, speech, noise, n, part);
  SEL_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_finish2, dim3(1), dim3(256), 0, s, part, nb, sums2);
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

int sel_mix_noise(const float* speech, const float* noise, int64_t n, const double* sums2, float snr, float* out,
                  sel_stream_t stream) {
  SEL_REQUIRE(n > 0, SEL_ERR_ARG, "empty batch");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int nb = int(std::min<int64_t>(4096, (n + 255) / 256));
  hipLaunchKernelGGL(k_mix2, dim3(nb), dim3(256), 0, s, speech, noise, n, sums2, snr, out);
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

int sel_snr_fwd(const float* pred, const float* target, int64_t B, int64_t T, double* sums, float* out,
                sel_stream_t stream) {
  SEL_REQUIRE(B > 0 && T > 0, SEL_ERR_ARG, "empty SNR input");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(k_snr_sums, dim3(unsigned(B)), dim3(256), 0, s, pred, target, T, sums);
  SEL_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_snr_finish, dim3(1), dim3(256), 0, s, sums, B, out);
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

int sel_snr_bwd(const float* pred, const float* target, int64_t B, int64_t T, const double* sums, const float* g_out,
                float* g_pred, sel_stream_t stream) {
  SEL_REQUIRE(B > 0 && T > 0, SEL_ERR_ARG, "empty SNR input");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int nb = int(std::min<int64_t>(4096, (B * T + 255) / 256));
  hipLaunchKernelGGL(k_snr_bwd, dim3(nb), dim3(256), 0, s, pred, target, B, T, sums, g_out, g_pred);
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

}  // extern "C"

namespace {
int adam_launch(const sel_adam_tensor* ts, int nt, const sel::glue::AdamConst& c, const float* dc, hipStream_t s) {
  using namespace sel::glue;
  for (int j = 0; j < nt; ++j)
    SEL_REQUIRE(ts[j].n >= 0 && (ts[j].n == 0 || (ts[j].p && ts[j].g && ts[j].m && ts[j].v)) &&
                    (ts[j].n + ADAM_EPB - 1) / ADAM_EPB < (int64_t(1) << 30),
                SEL_ERR_ARG, "bad Adam tensor %d", j);
  int j = 0;
  while (j < nt) {
    AdamJobs aj{};
    int64_t blocks = 0;
    int k = 0;
    for (; j < nt && k < ADAM_MAXT; ++j) {
      if (ts[j].n == 0) continue;
      const int64_t nb = (ts[j].n + ADAM_EPB - 1) / ADAM_EPB;
      if (k > 0 && blocks + nb >= (int64_t(1) << 31)) break;
      aj.p[k] = ts[j].p;
      aj.g[k] = ts[j].g;
      aj.m[k] = ts[j].m;
      aj.v[k] = ts[j].v;
      aj.n[k] = ts[j].n;
      aj.bstart[k] = int(blocks);
      blocks += nb;
      ++k;
    }
    aj.bstart[k] = int(blocks);
    aj.nt = k;
    if (blocks > 0) {
      if (dc)
        hipLaunchKernelGGL(k_adam_many<true>, dim3(unsigned(blocks)), dim3(256), 0, s, aj, c, dc);
      else
        hipLaunchKernelGGL(k_adam_many<false>, dim3(unsigned(blocks)), dim3(256), 0, s, aj, c, dc);
      SEL_LAUNCH_CHECK();
    }
  }
  return SEL_OK;
}

// (1 - beta) rounded once from the double, as torch's kernels receive it:
// 1 - float(0.999) is 1.3e-5 away from 0.001
sel::glue::AdamConst adam_const(double beta1, double beta2, double eps, double weight_decay, double step_size,
                                double bc2_sqrt) {
  return sel::glue::AdamConst{float(beta1), float(1.0 - beta1), float(beta2),        float(1.0 - beta2),
                              float(eps),   float(weight_decay), float(step_size), float(bc2_sqrt)};
}
}  // namespace

extern "C" {

int sel_adam_step_many(const sel_adam_tensor* ts, int nt, double beta1, double beta2, double eps, double weight_decay,
                       double step_size, double bc2_sqrt, sel_stream_t stream) {
  SEL_REQUIRE(nt >= 0 && (nt == 0 || ts), SEL_ERR_ARG, "bad Adam tensor list");
  SEL_REQUIRE(bc2_sqrt > 0.0 && eps >= 0.0, SEL_ERR_ARG, "bad Adam constants");
  return adam_launch(ts, nt, adam_const(beta1, beta2, eps, weight_decay, step_size, bc2_sqrt), nullptr,
                     reinterpret_cast<hipStream_t>(stream));
}

int sel_adam_step_many_dev(const sel_adam_tensor* ts, int nt, double beta1, double beta2, double eps,
                           double weight_decay, const float* lr, float* step, float* consts, sel_stream_t stream) {
  using namespace sel::glue;
  SEL_REQUIRE(nt >= 0 && (nt == 0 || ts), SEL_ERR_ARG, "bad Adam tensor list");
  SEL_REQUIRE(lr && step && consts, SEL_ERR_ARG, "null lr / step / consts");
  SEL_REQUIRE(beta2 < 1.0 && eps >= 0.0, SEL_ERR_ARG, "bad Adam constants");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(k_adam_consts, dim3(1), dim3(1), 0, s, lr, step, beta1, beta2, consts);
  SEL_LAUNCH_CHECK();
  return adam_launch(ts, nt, adam_const(beta1, beta2, eps, weight_decay, 0.0, 1.0), consts, s);
}

}  // extern "C"

// ---------------------------------------------------------------------------
// BatchNorm1d over channels-last rows (models/autoencoder/modules/projector.py
// :40-44, model='conv1d_bn': Conv1d then torch.nn.BatchNorm1d(code_dim)).
// x is (rows, C) fp32 with rows = B*T (the (B, C, T) tensor stored as (B, T, C)).
// Per-channel statistics: row chunks of kBnRows rows x 64-channel groups, each
// thread one channel of one row lane, fp64 sums; the chunk partials are summed
// in chunk order by one thread per channel (deterministic, no atomics).
// ---------------------------------------------------------------------------
namespace sel {
namespace glue {

constexpr int kBnRows = 256;   // rows per statistics chunk
constexpr int kBnLanes = 4;    // row lanes per 64-channel group (256 threads)

// mode 0: (sum x, sum x^2); mode 1: (sum gy, sum gy * (x - mean))
__global__ __launch_bounds__(256) void k_bn_partials(const float* __restrict__ x, const float* __restrict__ gy,
                                                     int64_t rows, int C, const float* __restrict__ mean, int mode,
                                                     double* __restrict__ part) {
  __shared__ double red[2][kBnLanes][64];
  const int cl = threadIdx.x & 63, lane = threadIdx.x >> 6;
  const int c = blockIdx.y * 64 + cl;
  const int64_t r0 = int64_t(blockIdx.x) * kBnRows;
  const int64_t r1 = r0 + kBnRows < rows ? r0 + kBnRows : rows;
  double a = 0.0, b = 0.0;
  if (c < C) {
    const float mu = mode ? mean[c] : 0.f;
    for (int64_t r = r0 + lane; r < r1; r += kBnLanes) {
      const float v = x[r * C + c];
      if (mode == 0) {
        a += double(v);
        b += double(v) * v;
      } else {
        const float g = gy[r * C + c];
        a += double(g);
        b += double(g) * double(v - mu);
      }
    }
  }
  red[0][lane][cl] = a;
  red[1][lane][cl] = b;
  __syncthreads();
  if (lane == 0 && c < C) {
    for (int l = 1; l < kBnLanes; ++l) {
      a += red[0][l][cl];
      b += red[1][l][cl];
    }
    part[(int64_t(blockIdx.x) * C + c) * 2] = a;
    part[(int64_t(blockIdx.x) * C + c) * 2 + 1] = b;
  }
}

// training statistics: mean, biased var -> invstd; running stats (torch's
// momentum update with the unbiased variance, batch_norm.cpp)
__global__ __launch_bounds__(256) void k_bn_stats(const double* __restrict__ part, int nchunk, int64_t rows, int C,
                                                  float eps, float momentum, float* __restrict__ running_mean,
                                                  float* __restrict__ running_var, float* __restrict__ save_mean,
                                                  float* __restrict__ save_invstd) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double s = 0.0, ss = 0.0;
  for (int k = 0; k < nchunk; ++k) {
    s += part[(int64_t(k) * C + c) * 2];
    ss += part[(int64_t(k) * C + c) * 2 + 1];
  }
  const double m = s / double(rows);
  double var = ss / double(rows) - m * m;
  var = var > 0.0 ? var : 0.0;
  save_mean[c] = float(m);
  save_invstd[c] = float(1.0 / sqrt(var + double(eps)));
  if (running_mean) {
    const double unb = rows > 1 ? var * double(rows) / double(rows - 1) : var;
    running_mean[c] = float((1.0 - momentum) * double(running_mean[c]) + momentum * m);
    running_var[c] = float((1.0 - momentum) * double(running_var[c]) + momentum * unb);
  }
}

// evaluation statistics from the running buffers
__global__ __launch_bounds__(256) void k_bn_eval_stats(const float* __restrict__ running_mean,
                                                       const float* __restrict__ running_var, int C, float eps,
                                                       float* __restrict__ save_mean, float* __restrict__ save_invstd) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  save_mean[c] = running_mean[c];
  save_invstd[c] = float(1.0 / sqrt(double(running_var[c]) + double(eps)));
}

// y = (x - mean) * invstd * gamma + beta
__global__ __launch_bounds__(256) void k_bn_apply(const float* __restrict__ x, int64_t n, int C,
                                                  const float* __restrict__ mean, const float* __restrict__ invstd,
                                                  const float* __restrict__ gamma, const float* __restrict__ beta,
                                                  float* __restrict__ y) {
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
    const int c = int(i % C);
    const float v = (x[i] - mean[c]) * invstd[c];
    y[i] = gamma ? fmaf(v, gamma[c], beta ? beta[c] : 0.f) : v;
  }
}

// gx = gamma invstd (gy - sum_gy / M - xhat sum(gy xhat) / M) (training), or
// gamma invstd gy (evaluation); also d gamma = sum(gy xhat), d beta = sum(gy)
__global__ __launch_bounds__(256) void k_bn_bwd(const float* __restrict__ x, const float* __restrict__ gy, int64_t n,
                                                int C, int64_t rows, const float* __restrict__ mean,
                                                const float* __restrict__ invstd, const float* __restrict__ gamma,
                                                const double* __restrict__ part, int nchunk, int training,
                                                float* __restrict__ gx) {
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
    const int c = int(i % C);
    const float is = invstd[c];
    const float w = gamma ? gamma[c] : 1.f;
    if (!training) {
      gx[i] = gy[i] * is * w;
      continue;
    }
    // the chunk sums were folded into part[0 .. 2C) by k_bn_gsum
    const float sg = float(part[2 * c] / double(rows));
    const float sgx = float(part[2 * c + 1] / double(rows)) * is * is;   // sum(gy (x - mu)) / M * invstd^2
    gx[i] = w * is * (gy[i] - sg - (x[i] - mean[c]) * sgx);
  }
}

// chunk partials -> per-channel totals (in place into chunk 0) and the affine gradients
__global__ __launch_bounds__(256) void k_bn_gsum(double* __restrict__ part, int nchunk, int C,
                                                 const float* __restrict__ invstd, float* __restrict__ ggamma,
                                                 float* __restrict__ gbeta) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double s = 0.0, sx = 0.0;
  for (int k = 0; k < nchunk; ++k) {
    s += part[(int64_t(k) * C + c) * 2];
    sx += part[(int64_t(k) * C + c) * 2 + 1];
  }
  part[2 * c] = s;
  part[2 * c + 1] = sx;
  if (ggamma) ggamma[c] = float(sx * double(invstd[c]));
  if (gbeta) gbeta[c] = float(s);
}

inline int bn_chunks(int64_t rows) { return int((rows + kBnRows - 1) / kBnRows); }
inline int bn_grid(int64_t n) { return int(std::min<int64_t>(4096, (n + 255) / 256)); }

}  // namespace glue
}  // namespace sel

extern "C" {

size_t sel_batchnorm_workspace(int64_t rows, int C) {
  return size_t(sel::glue::bn_chunks(rows)) * size_t(C) * 2 * sizeof(double);
}

int sel_batchnorm_fwd(const float* x, int64_t rows, int C, const float* gamma, const float* beta, int training,
                      float eps, float momentum, float* running_mean, float* running_var, float* save_mean,
                      float* save_invstd, float* y, void* ws, size_t ws_bytes, sel_stream_t stream) {
  using namespace sel::glue;
  SEL_REQUIRE(rows > 0 && C > 0 && x && y && save_mean && save_invstd, SEL_ERR_ARG, "bad batch-norm arguments");
  SEL_REQUIRE(training || (running_mean && running_var), SEL_ERR_ARG, "evaluation needs the running statistics");
  SEL_REQUIRE(!training || ws_bytes >= sel_batchnorm_workspace(rows, C), SEL_ERR_WORKSPACE, "workspace too small");
  SEL_REQUIRE(bn_chunks(rows) < 65536 * 16, SEL_ERR_ARG, "batch too large");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int cb = (C + 255) / 256;
  if (training) {
    double* part = static_cast<double*>(ws);
    hipLaunchKernelGGL(k_bn_partials, dim3(bn_chunks(rows), (C + 63) / 64), dim3(256), 0, s, x, nullptr, rows, C,
                       nullptr, 0, part);
    SEL_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_bn_stats, dim3(cb), dim3(256), 0, s, part, bn_chunks(rows), rows, C, eps, momentum,
                       running_mean, running_var, save_mean, save_invstd);
  } else {
    hipLaunchKernelGGL(k_bn_eval_stats, dim3(cb), dim3(256), 0, s, running_mean, running_var, C, eps, save_mean,
                       save_invstd);
  }
  SEL_LAUNCH_CHECK();
  const int64_t n = rows * C;
  hipLaunchKernelGGL(k_bn_apply, dim3(bn_grid(n)), dim3(256), 0, s, x, n, C, save_mean, save_invstd, gamma, beta, y);
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

int sel_batchnorm_bwd(const float* x, const float* gy, int64_t rows, int C, const float* gamma,
                      const float* save_mean, const float* save_invstd, int training, float* gx, float* ggamma,
                      float* gbeta, void* ws, size_t ws_bytes, sel_stream_t stream) {
  using namespace sel::glue;
  SEL_REQUIRE(rows > 0 && C > 0 && x && gy && save_mean && save_invstd, SEL_ERR_ARG, "bad batch-norm arguments");
  SEL_REQUIRE(ws_bytes >= sel_batchnorm_workspace(rows, C), SEL_ERR_WORKSPACE, "workspace too small");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  double* part = static_cast<double*>(ws);
  const int nc = bn_chunks(rows);
  hipLaunchKernelGGL(k_bn_partials, dim3(nc, (C + 63) / 64), dim3(256), 0, s, x, gy, rows, C, save_mean, 1, part);
  SEL_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_bn_gsum, dim3((C + 255) / 256), dim3(256), 0, s, part, nc, C, save_invstd, ggamma, gbeta);
  SEL_LAUNCH_CHECK();
  if (gx) {
    const int64_t n = rows * C;
    hipLaunchKernelGGL(k_bn_bwd, dim3(bn_grid(n)), dim3(256), 0, s, x, gy, n, C, rows, save_mean, save_invstd, gamma,
                       part, nc, training, gx);
    SEL_LAUNCH_CHECK();
  }
  return SEL_OK;
}

}  // extern "C"
