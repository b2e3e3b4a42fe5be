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

// Staged-codebook variant (D % 8 == 0, K % 4 == 0): 20 rows per block (5120 rows
// -> 256 blocks, one per CU) and each stage's codebook streamed through LDS in
// 8-dim x 1024-code chunks (32 KB, double-buffered, prefetched one chunk ahead
// in registers) instead of dword loads from L2 inside the dot loop.  Thread t
// scores codes kb + 4t .. 4t+3 (one ds_read_b128) against the 20 rows (5
// broadcast ds_read_b128 of the transposed residual).  Per-(row, code)
// arithmetic is the k_rvq_fwd one exactly (fmaf over d ascending, same distance
// expression), so both kernels pick the same codes.
constexpr int R2 = 20;
constexpr int DC = 8;       // dims per staged chunk
constexpr int T2 = 512;     // 8 waves: 2 per SIMD
constexpr int C2 = 2;       // codes per thread per pass
constexpr int KP = T2 * C2; // codes per pass (1024)

__global__ __launch_bounds__(T2) void k_rvq_fwd2(const float* __restrict__ x, int64_t N, int D,
                                                      const float* __restrict__ embeds, int S, int K,
                                                      float* __restrict__ out, int64_t* __restrict__ idx,
                                                      int32_t* __restrict__ counts,
                                                      double* __restrict__ partials) {
  extern __shared__ __align__(16) unsigned char smem[];
  float* resT = reinterpret_cast<float*>(smem);       // [D][R2]
  float* acc_o = resT + MAXD * R2;                    // [R2][D]
  float* ebuf = acc_o + R2 * MAXD;                    // [2][DC][KP]
  __shared__ float xn[R2];
  __shared__ float red_d[T2 / 64][R2];
  __shared__ int red_k[T2 / 64][R2];
  __shared__ int sel_k[R2];
  __shared__ double red[16];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t r0 = int64_t(blockIdx.x) * R2;
  for (int i = tid; i < R2 * D; i += T2) {
    const int r = i / D, d = i % D;
    const int64_t row = r0 + r;
    resT[d * R2 + r] = row < N ? x[row * D + d] : 0.f;
    acc_o[r * D + d] = 0.f;
  }
  __syncthreads();

  const int nd = D / DC;
  const int npass = (K + KP - 1) / KP;
  const int nchunk = npass * nd;
  for (int s = 0; s < S; ++s) {
    const float* __restrict__ E = embeds + int64_t(s) * D * K;
    for (int r = wave; r < R2; r += T2 / 64) {
      float v = 0.f;
      for (int d = lane; d < D; d += 64) v = fmaf(resT[d * R2 + r], resT[d * R2 + r], v);
      v = wave_sum(v);
      if (lane == 0) xn[r] = v;
    }
    float4 pre[DC * KP / 4 / T2];  // 4 float4 per thread
    auto load = [&](int c) {
      const int kb = (c / nd) * KP, d0 = (c % nd) * DC;
#pragma unroll
      for (int i = 0; i < DC * KP / 4 / T2; ++i) {
        const int v = tid + i * T2;
        const int dd = v / (KP / 4), k = kb + (v % (KP / 4)) * 4;
        pre[i] = k < K ? *reinterpret_cast<const float4*>(E + int64_t(d0 + dd) * K + k)
                       : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    };
    auto store = [&](int buf) {
#pragma unroll
      for (int i = 0; i < DC * KP / 4 / T2; ++i) {
        const int v = tid + i * T2;
        reinterpret_cast<float4*>(ebuf + buf * DC * KP)[v] = pre[i];
      }
    };
    load(0);
    store(0);
    __syncthreads();

    float bd[R2];
    int bk[R2];
#pragma unroll
    for (int r = 0; r < R2; ++r) {
      bd[r] = __builtin_inff();
      bk[r] = 0x7fffffff;
    }
    for (int pass = 0; pass < npass; ++pass) {
      float dot[R2][C2], en[C2];
#pragma unroll
      for (int j = 0; j < C2; ++j) {
        en[j] = 0.f;
#pragma unroll
        for (int r = 0; r < R2; ++r) dot[r][j] = 0.f;
      }
      for (int dch = 0; dch < nd; ++dch) {
        const int c = pass * nd + dch;
        if (c + 1 < nchunk) load(c + 1);
        const float* eb = ebuf + (c & 1) * DC * KP + tid * C2;
        const float* xr = resT + dch * DC * R2;
#pragma unroll 2
        for (int dd = 0; dd < DC; ++dd) {
          const float2 e2 = *reinterpret_cast<const float2*>(eb + dd * KP);
          const float e[C2] = {e2.x, e2.y};
#pragma unroll
          for (int j = 0; j < C2; ++j) en[j] = fmaf(e[j], e[j], en[j]);
#pragma unroll
          for (int r4 = 0; r4 < R2 / 4; ++r4) {
            const float4 xv4 = *reinterpret_cast<const float4*>(xr + dd * R2 + 4 * r4);
            const float xv[4] = {xv4.x, xv4.y, xv4.z, xv4.w};
#pragma unroll
            for (int rr = 0; rr < 4; ++rr)
#pragma unroll
              for (int j = 0; j < C2; ++j) dot[4 * r4 + rr][j] = fmaf(xv[rr], e[j], dot[4 * r4 + rr][j]);
          }
        }
        if (c + 1 < nchunk) store((c + 1) & 1);
        __syncthreads();
      }
      const int kb = pass * KP;
#pragma unroll
      for (int j = 0; j < C2; ++j) {
        const int k = kb + tid * C2 + j;
        const bool kin = k < K;
#pragma unroll
        for (int r = 0; r < R2; ++r) {
          const float dist = (xn[r] - 2.f * dot[r][j]) + en[j];
          const bool take = kin && better(dist, k, bd[r], bk[r]);
          bd[r] = take ? dist : bd[r];
          bk[r] = take ? k : bk[r];
        }
      }
    }
#pragma unroll
    for (int r = 0; r < R2; ++r) {
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
    if (tid < R2) {
      float d0 = red_d[0][tid];
      int k0 = red_k[0][tid];
      for (int w = 1; w < T2 / 64; ++w)
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
    float sq = 0.f;
    for (int i = tid; i < R2 * D; i += T2) {
      const int r = i / D, d = i % D;
      if (r0 + r >= N) continue;
      const float q = E[int64_t(d) * K + sel_k[r]];
      const float rv = resT[d * R2 + r];
      const float diff = q - rv;
      sq = fmaf(diff, diff, sq);
      const float qst = rv + diff;
      resT[d * R2 + r] = rv - qst;
      acc_o[r * D + d] += qst;
    }
    const double bs = block_sum<double>(double(sq), red);
    if (tid == 0) partials[int64_t(s) * gridDim.x + blockIdx.x] = bs;
    __syncthreads();
  }
  for (int i = tid; i < R2 * D; i += T2) {
    const int r = i / D, d = i % D;
    const int64_t row = r0 + r;
    if (row < N) out[row * D + d] = acc_o[r * D + d];
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
  const int64_t nb = (N + ROWS - 1) / ROWS;  // >= the staged kernel's block count (20 rows)
  return size_t(nb) * size_t(S) * sizeof(double) + 16;
}

int sel_rvq_fwd(const float* x, int64_t N, int D, const float* embeds, int S, int K, float* out, int64_t* idx,
                int32_t* counts, double* sqerr, void* ws, size_t ws_bytes, sel_stream_t stream) {
  SEL_REQUIRE(N >= 0 && D > 0 && D <= MAXD && S > 0 && K > 0, SEL_ERR_ARG,
              "bad rvq shape N=%lld D=%d S=%d K=%d", (long long)N, D, S, K);
  SEL_REQUIRE(ws_bytes >= sel_rvq_workspace(N, S, K), SEL_ERR_WORKSPACE, "workspace too small");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  SEL_HIP(hipMemsetAsync(counts, 0, size_t(S) * K * sizeof(int32_t), s));
  const bool staged = D % DC == 0 && K % 4 == 0 && tune(2) == 0;
  const int nb = int((N + (staged ? R2 : ROWS) - 1) / (staged ? R2 : ROWS));
  double* part = static_cast<double*>(ws);
  if (nb > 0 && staged) {
    const size_t lds = (size_t(2) * MAXD * R2 + size_t(2) * DC * KP) * sizeof(float);
    SEL_HIP(hipFuncSetAttribute((const void*)k_rvq_fwd2, hipFuncAttributeMaxDynamicSharedMemorySize, int(lds)));
    hipLaunchKernelGGL(k_rvq_fwd2, dim3(nb), dim3(T2), lds, s, x, N, D, embeds, S, K, out, idx, counts, part);
    SEL_LAUNCH_CHECK();
  } else if (nb > 0) {
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
