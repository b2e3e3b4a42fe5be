// Residual VQ (layers/vq_module.py:61-88 eval mode, ResidualVQ :119-134) on gfx950.
//
// Rows are independent through all stages, so one workgroup carries a block of
// 16 rows through every stage with the residual kept in LDS: per stage each
// lane scores 4 codes against the 16 rows (codebook streamed from L2,
// coalesced over k), a wavefront argmin with lowest-index tie-break picks the
// code, and the row update (straight-through value r + (q - r), next residual,
// running sum) is done in LDS.  Cross-row quantities (commitment SSE, code
// histogram for the perplexity) go to deterministic per-block partials and
// integer atomics.
#include <algorithm>

#include "sel_common.h"

namespace sel {
namespace vq {

constexpr int ROWS = 16;
constexpr int THREADS = 256;
constexpr int MAXD = 256;
constexpr int CPT = 4;  // codes per thread per pass

__device__ __forceinline__ bool better(float d, int k, float bd, int bk) {
  return d < bd || (d == bd && k < bk);
}

__global__ __launch_bounds__(THREADS) void k_rvq_fwd(const float* __restrict__ x, int64_t N, int D,
                                                     const float* __restrict__ embeds, int S, int K,
                                                     float* __restrict__ out, int64_t* __restrict__ idx,
                                                     int32_t* __restrict__ counts,
                                                     double* __restrict__ partials) {
  __shared__ float res[ROWS][MAXD + 1];
  __shared__ float acc_o[ROWS][MAXD + 1];
  __shared__ float xn[ROWS];
  __shared__ float red_d[4][ROWS];
  __shared__ int red_k[4][ROWS];
  __shared__ int sel_k[ROWS];
  __shared__ double red[16];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t r0 = int64_t(blockIdx.x) * ROWS;
  for (int i = tid; i < ROWS * D; i += THREADS) {
    const int r = i / D, d = i % D;
    const int64_t row = r0 + r;
    res[r][d] = row < N ? x[row * D + d] : 0.f;
    acc_o[r][d] = 0.f;
  }
  __syncthreads();

  for (int s = 0; s < S; ++s) {
    const float* __restrict__ E = embeds + int64_t(s) * D * K;
    // |r|^2 per row (one wave per 4 rows, lanes over d)
    for (int r = wave; r < ROWS; r += 4) {
      float v = 0.f;
      for (int d = lane; d < D; d += 64) v = fmaf(res[r][d], res[r][d], v);
      v = wave_sum(v);
      if (lane == 0) xn[r] = v;
    }
    __syncthreads();
    float bd[ROWS];
    int bk[ROWS];
#pragma unroll
    for (int r = 0; r < ROWS; ++r) {
      bd[r] = __builtin_inff();
      bk[r] = 0x7fffffff;
    }
    for (int kb = 0; kb < K; kb += THREADS * CPT) {
      float dot[ROWS][CPT];
      float en[CPT];
#pragma unroll
      for (int j = 0; j < CPT; ++j) {
        en[j] = 0.f;
#pragma unroll
        for (int r = 0; r < ROWS; ++r) dot[r][j] = 0.f;
      }
      for (int d = 0; d < D; ++d) {
        float e[CPT];
#pragma unroll
        for (int j = 0; j < CPT; ++j) {
          const int k = kb + tid + j * THREADS;
          e[j] = k < K ? E[int64_t(d) * K + k] : 0.f;
          en[j] = fmaf(e[j], e[j], en[j]);
        }
#pragma unroll
        for (int r = 0; r < ROWS; ++r) {
          const float xv = res[r][d];
#pragma unroll
          for (int j = 0; j < CPT; ++j) dot[r][j] = fmaf(xv, e[j], dot[r][j]);
        }
      }
#pragma unroll
      for (int j = 0; j < CPT; ++j) {
        const int k = kb + tid + j * THREADS;
        if (k >= K) continue;
#pragma unroll
        for (int r = 0; r < ROWS; ++r) {
          const float dist = (xn[r] - 2.f * dot[r][j]) + en[j];
          if (better(dist, k, bd[r], bk[r])) {
            bd[r] = dist;
            bk[r] = k;
          }
        }
      }
    }
    // wave argmin per row
#pragma unroll
    for (int r = 0; r < ROWS; ++r) {
      float d0 = bd[r];
      int k0 = bk[r];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const float d1 = __shfl_xor(d0, o, 64);
        const int k1 = __shfl_xor(k0, o, 64);
        if (better(d1, k1, d0, k0)) {
          d0 = d1;
          k0 = k1;
        }
      }
      if (lane == 0) {
        red_d[wave][r] = d0;
        red_k[wave][r] = k0;
      }
    }
    __syncthreads();
    if (tid < ROWS) {
      float d0 = red_d[0][tid];
      int k0 = red_k[0][tid];
      for (int w = 1; w < 4; ++w)
        if (better(red_d[w][tid], red_k[w][tid], d0, k0)) {
          d0 = red_d[w][tid];
          k0 = red_k[w][tid];
        }
      sel_k[tid] = k0;
      const int64_t row = r0 + tid;
      if (row < N) {
        idx[int64_t(s) * N + row] = k0;
        atomicAdd(&counts[int64_t(s) * K + k0], 1);
      }
    }
    __syncthreads();
    // row update: qst = r + (q - r); r <- r - qst; out += qst
    float sq = 0.f;
    for (int i = tid; i < ROWS * D; i += THREADS) {
      const int r = i / D, d = i % D;
      if (r0 + r >= N) continue;
      const float q = E[int64_t(d) * K + sel_k[r]];
      const float rv = res[r][d];
      const float diff = q - rv;
      sq = fmaf(diff, diff, sq);
      const float qst = rv + diff;
      res[r][d] = rv - qst;
      acc_o[r][d] += qst;
    }
    const double bs = block_sum<double>(double(sq), red);
    if (tid == 0) partials[int64_t(s) * gridDim.x + blockIdx.x] = bs;
    __syncthreads();
  }
  for (int i = tid; i < ROWS * D; i += THREADS) {
    const int r = i / D, d = i % D;
    const int64_t row = r0 + r;
    if (row < N) out[row * D + d] = acc_o[r][d];
  }
}

__global__ __launch_bounds__(256) void k_rvq_sqerr(const double* __restrict__ partials, int nb,
                                                   double* __restrict__ sqerr) {
  __shared__ double red[16];
  const int s = blockIdx.x;
  double v = 0.0;
  for (int i = threadIdx.x; i < nb; i += blockDim.x) v += partials[int64_t(s) * nb + i];
  v = block_sum<double>(v, red);
  if (threadIdx.x == 0) sqerr[s] = v;
}

__global__ __launch_bounds__(256) void k_rvq_finish(const int32_t* __restrict__ counts,
                                                    const double* __restrict__ sqerr, int64_t N, int D,
                                                    int K, float commitment, float* __restrict__ loss,
                                                    float* __restrict__ ppl) {
  __shared__ float red[16];
  const int s = blockIdx.x;
  float v = 0.f;
  const float invn = 1.f / float(N);
  for (int k = threadIdx.x; k < K; k += blockDim.x) {
    const float p = float(counts[int64_t(s) * K + k]) * invn;
    v += p * logf(p + 1e-10f);
  }
  v = block_sum<float>(v, red);
  if (threadIdx.x == 0) {
    ppl[s] = expf(-v);
    loss[s] = float(sqerr[s] / (double(N) * double(D))) * commitment;
  }
}

__global__ __launch_bounds__(256) void k_rvq_bwd(const float* __restrict__ x, int64_t N, int D,
                                                 const float* __restrict__ E0, int K,
                                                 const int64_t* __restrict__ idx0,
                                                 const float* __restrict__ g_out,
                                                 const float* __restrict__ g_loss, float commitment,
                                                 float* __restrict__ gx) {
  const float c = g_loss ? g_loss[0] * commitment * 2.f / float(double(N) * D) : 0.f;
  const int64_t total = N * D;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
       i += int64_t(gridDim.x) * blockDim.x) {
    const int64_t row = i / D;
    const int d = int(i % D);
    const float q = E0[int64_t(d) * K + idx0[row]];
    float g = g_out ? g_out[i] : 0.f;
    g += c * (x[i] - q);
    gx[i] = g;
  }
}

}  // namespace vq
}  // namespace sel

using namespace sel;
using namespace sel::vq;

extern "C" {

size_t sel_rvq_workspace(int64_t N, int S, int K) {
  (void)K;
  const int64_t nb = (N + ROWS - 1) / ROWS;
  return size_t(nb) * size_t(S) * sizeof(double) + 16;
}

int sel_rvq_fwd(const float* x, int64_t N, int D, const float* embeds, int S, int K, float* out, int64_t* idx,
                int32_t* counts, double* sqerr, void* ws, size_t ws_bytes, sel_stream_t stream) {
  SEL_REQUIRE(N >= 0 && D > 0 && D <= MAXD && S > 0 && K > 0, SEL_ERR_ARG,
              "bad rvq shape N=%lld D=%d S=%d K=%d", (long long)N, D, S, K);
  SEL_REQUIRE(ws_bytes >= sel_rvq_workspace(N, S, K), SEL_ERR_WORKSPACE, "workspace too small");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  SEL_HIP(hipMemsetAsync(counts, 0, size_t(S) * K * sizeof(int32_t), s));
  const int nb = int((N + ROWS - 1) / ROWS);
  double* part = static_cast<double*>(ws);
  if (nb > 0) {
    hipLaunchKernelGGL(k_rvq_fwd, dim3(nb), dim3(THREADS), 0, s, x, N, D, embeds, S, K, out, idx, counts, part);
    SEL_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(k_rvq_sqerr, dim3(S), dim3(256), 0, s, part, nb, sqerr);
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

int sel_rvq_finish(const int32_t* counts, const double* sqerr, int64_t N, int D, int S, int K, float commitment,
                   float* loss, float* ppl, sel_stream_t stream) {
  SEL_REQUIRE(N > 0, SEL_ERR_ARG, "empty VQ input");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(k_rvq_finish, dim3(S), dim3(256), 0, s, counts, sqerr, N, D, K, commitment, loss, ppl);
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

int sel_rvq_bwd(const float* x, int64_t N, int D, const float* embed0, int K, const int64_t* idx0,
                const float* g_out, const float* g_loss, float commitment, float* g_x, sel_stream_t stream) {
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int64_t total = N * D;
  if (total == 0) return SEL_OK;
  dim3 grid(unsigned(std::min<int64_t>(4096, (total + 255) / 256)));
  hipLaunchKernelGGL(k_rvq_bwd, grid, dim3(256), 0, s, x, N, D, embed0, K, idx0, g_out, g_loss, commitment, g_x);
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

}  // extern "C"
