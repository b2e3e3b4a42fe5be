// Residual VQ (layers/vq_module.py:61-88 eval mode, ResidualVQ :119-134) on gfx950.
//
// Rows are independent through all stages, so one workgroup carries a block of
// rows through every stage with the residual kept in LDS: per stage the block
// scores every code against its rows, an argmin with lowest-index tie-break
// picks the code, and the row update (straight-through value r + (q - r), next
// residual, running sum) is done in LDS.  Cross-row quantities (commitment SSE,
// code histogram for the perplexity) go to deterministic per-block partials and
// integer atomics.  Three kernel families with one arithmetic (bit-identical
// results, tune key 2): k_rvq_mfma (default, f32-input matrix cores), k_rvq_fwd2
// (codebook staged through LDS, fp32 VALU) and k_rvq_fwd (direct, any D).
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

// Matrix-core variant (default; D % 4 == 0, D <= 64): the 16-row residual
// block is the A operand of v_mfma_f32_16x16x4_f32 (lane l holds
// r[row l&15][d = 4j + (l>>4)] for k-step j: 16 VGPRs at D = 64, loaded from
// LDS once per stage) and the codebook is the B operand.  k_rvq_prep lays each
// stage's codebook out in B-fragment order (per 16-code tile: [j/4][lane][j%4],
// so a lane's operands for four k-steps are one coalesced 16-byte load) and
// computes |e|^2.  Each of the 8 waves scores every 8th code tile with the
// next tile's operands in flight, starting at a block-dependent tile so the
// 320 blocks do not all hit the same L2 lines at once.  The code histogram is a
// separate pass over the indices (k_rvq_hist), off the per-stage critical path.
// The f32-input MFMA is bit-for-bit a k-ordered fmaf chain, so with d ascending
// from a zero accumulator every dot product, |e|^2 and |r|^2 (the same
// wave_sum) is the one k_rvq_fwd computes: all variants pick the same codes and
// produce the same outputs.
constexpr int RM = 16;
constexpr int TM = 512;
constexpr int NWM = TM / 64;
constexpr int DM = 64;
using f32x4 = __attribute__((ext_vector_type(4))) float;

struct MfmaGeo {
  int ntile, nj4;  // 16-code tiles; groups of four k-steps (4 dims each), always DM / 16:
                   // fragments past D are zeros, so the tile loads have no runtime bound
  __host__ __device__ MfmaGeo(int D, int K) : ntile((K + 15) / 16), nj4(DM / 16) { (void)D; }
  __host__ __device__ int64_t tile_floats() const { return int64_t(nj4) * 256; }
  __host__ __device__ int64_t stage_floats() const { return int64_t(ntile) * tile_floats(); }
};

// one thread per (stage, tile, j4, lane): four B operands, zero-padded past D and K
__global__ __launch_bounds__(256) void k_rvq_prep(const float* __restrict__ embeds, int S, int D, int K,
                                                  float* __restrict__ ep, float* __restrict__ en,
                                                  int32_t* __restrict__ counts) {
  const MfmaGeo g(D, K);
  const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < int64_t(S) * K) counts[i] = 0;  // the code histogram (k_rvq_hist adds into it; no memset launch)
  const int64_t total = int64_t(S) * g.stage_floats() / 4;
  if (i < total) {
    const int lane = int(i & 63);
    const int64_t q = i >> 6;
    const int j4 = int(q % g.nj4);
    const int64_t st = q / g.nj4;  // s * ntile + tile
    const int tile = int(st % g.ntile);
    const int64_t s = st / g.ntile;
    const int k = tile * 16 + (lane & 15);
    const float* E = embeds + s * D * K;
    float v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int d = 4 * (4 * j4 + e) + (lane >> 4);
      v[e] = (d < D && k < K) ? E[int64_t(d) * K + k] : 0.f;
    }
    reinterpret_cast<float4*>(ep)[i] = make_float4(v[0], v[1], v[2], v[3]);
  }
  if (i < int64_t(S) * K) {  // |e|^2: fmaf over d ascending from 0 (k_rvq_fwd's en)
    const int64_t s = i / K, k = i - s * K;
    const float* E = embeds + s * D * K + k;
    float v = 0.f;
#pragma unroll 16
    for (int d = 0; d < D; ++d) v = fmaf(E[int64_t(d) * K], E[int64_t(d) * K], v);
    en[i] = v;
  }
}

constexpr int SM = 16;  // max stages of the matrix-core variant (per-stage state in LDS)

// timing ablations of the matrix-core kernel (diagnostic builds only, wrong
// results): 1 no tile loop, 4 no codebook gather in the row update, 8 no |e|^2
// staging; 0 in every product build
#ifndef SEL_RVQ_ABL
#define SEL_RVQ_ABL 0
#endif

// RG row groups of 16 rows per block share every codebook tile: each wave's
// B operands (4 KB per 16-code tile, read from L2) feed RG independent MFMA
// chains.  RG = 2 halves the codebook reads per row (the hypothesis: the L2 ->
// CU rate binds at C3, 320 blocks x 8 stages x 256 KB) at the same busiest-CU
// MFMA work, but measured slower (160 blocks, one per CU, at 2 waves per SIMD:
// 169 -> 193 us per forward), so RG = 1 is the default (tune key 39 = 2: RG = 2).
// Tile-loop schedule: the next tile's B operands are requested one tile ahead
// with branch-free addresses (past the last tile of a stage: the next stage's
// first tile; past the last stage: this tile again), |e|^2 of the stage is read
// from LDS (staged at the stage start), and operands past D are zeros (resT is
// zero-padded to DM dims, k_rvq_prep zero-pads the B fragments), so the loads
// and the MFMA chain have no runtime bound: a zero product on a zero-based accumulator
// (never -0) adds exactly nothing, so results equal the chain over d < D.  The
// earlier form waited for vmcnt(0) in every tile's epilogue (a global |e|^2
// load issued after the prefetch): each tile exposed the prefetch's L2 latency.
template <int RG>
__global__ __launch_bounds__(TM) __attribute__((amdgpu_waves_per_eu(RG == 1 ? 4 : 2))) void k_rvq_mfma(
    const float* __restrict__ x, int64_t N, int D, const float* __restrict__ embeds, int S, int K,
    const float* __restrict__ ep_all, const float* __restrict__ en_all, float* __restrict__ out,
    int64_t* __restrict__ idx, double* __restrict__ partials) {
  constexpr int RB = RM * RG;      // rows per block
  __shared__ float resT[DM * RB];  // [d][row]: the A-fragment reads hit 64 distinct banks
  __shared__ float acc_o[RB * DM];
  __shared__ float xn[RB];
  __shared__ float red_d[NWM][RB];
  __shared__ int red_k[NWM][RB];
  __shared__ int sel_k[SM][RB];    // chosen codes, written to idx after the last stage
  __shared__ float sq_t[SM][TM];   // per-thread SSE per stage, reduced after the last stage
  __shared__ double red[16];
  extern __shared__ float en_l[];  // |e|^2 of the current stage (K floats, dynamic)

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int col = lane & 15, h = lane >> 4;
  const int64_t r0 = int64_t(blockIdx.x) * RB;
  for (int i = tid; i < RB * DM; i += TM) {
    const int r = i / DM, d = i % DM;
    const int64_t row = r0 + r;
    resT[d * RB + r] = row < N && d < D ? x[row * D + d] : 0.f;
    if (d < D) acc_o[r * D + d] = 0.f;
  }
  const MfmaGeo g(D, K);
  const int ntile = g.ntile, nj4 = g.nj4;
  const int rot = int((blockIdx.x * 4u) % unsigned(ntile));  // L2 de-synchronisation across blocks
  // wave w scores tiles w, w + 8, ... in a block-rotated order with the next
  // tile's operands in flight (one tile keeps the kernel at 4 waves/SIMD); the
  // last tile of a stage prefetches the next stage's first one
  auto tile_of = [&](int p) {
    const int t = p + rot;
    return t >= ntile ? t - ntile : t;
  };
  // wave w scores tiles w, w + 8, ... in a block-rotated order with the next
  // tile's operands in flight (one tile keeps the kernel at 4 waves/SIMD); the
  // last tile of a stage prefetches the next stage's first one
  float4 cur[DM / 16], nxt[DM / 16];
  auto load = [&](int st, int p, float4 (&b)[DM / 16]) {
    const float4* src = reinterpret_cast<const float4*>(ep_all + int64_t(st) * g.stage_floats()) +
                        int64_t(tile_of(p)) * (nj4 * 64) + lane;
#pragma unroll
    for (int j4 = 0; j4 < DM / 16; ++j4) b[j4] = src[j4 * 64];
  };
  if (wave < ntile) load(0, wave, cur);
  __syncthreads();

  for (int s = 0; s < S; ++s) {
    const float* __restrict__ E = embeds + int64_t(s) * D * K;
    const float* __restrict__ enS = en_all + int64_t(s) * K;
    if constexpr (!(SEL_RVQ_ABL & 8))
      for (int k = tid; k < K; k += TM) en_l[k] = enS[k];
    for (int r = wave; r < RB; r += NWM) {
      float v = 0.f;
      for (int d = lane; d < D; d += 64) v = fmaf(resT[d * RB + r], resT[d * RB + r], v);
      v = wave_sum(v);
      if (lane == 0) xn[r] = v;
    }
    __syncthreads();
    float a[RG][DM / 4];
#pragma unroll
    for (int q = 0; q < RG; ++q)
#pragma unroll
      for (int j = 0; j < DM / 4; ++j) a[q][j] = resT[(4 * j + h) * RB + RM * q + col];
    float xr[RG][4];
#pragma unroll
    for (int q = 0; q < RG; ++q)
#pragma unroll
      for (int i = 0; i < 4; ++i) xr[q][i] = xn[RM * q + 4 * h + i];
    float bd[RG][4];
    int bk[RG][4];
#pragma unroll
    for (int q = 0; q < RG; ++q)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        bd[q][i] = __builtin_inff();
        bk[q][i] = 0x7fffffff;
      }
    // one tile: request the next one into `fill`, score this one from `use`
    // (the loop alternates the two buffers: a register copy between them
    // would make every tile wait for its own prefetch)
    auto tile = [&](int p, const float4 (&use)[DM / 16], float4 (&fill)[DM / 16]) {
      const bool more = p + NWM < ntile;
      load(more || s + 1 >= S ? s : s + 1, more ? p + NWM : (s + 1 < S ? wave : p), fill);
      __builtin_amdgcn_sched_barrier(0);  // the requests go out before this tile's MFMAs
      f32x4 c[RG];
#pragma unroll
      for (int q = 0; q < RG; ++q) c[q] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < DM / 4; ++j) {
        const float4 bv = use[j >> 2];
        const float bj = (j & 3) == 0 ? bv.x : (j & 3) == 1 ? bv.y : (j & 3) == 2 ? bv.z : bv.w;
#pragma unroll
        for (int q = 0; q < RG; ++q) c[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[q][j], bj, c[q], 0, 0, 0);
      }
      const int k = tile_of(p) * 16 + col;
      const bool kin = k < K;
      const float ek = en_l[kin ? k : 0];
#pragma unroll
      for (int q = 0; q < RG; ++q)
#pragma unroll
        for (int i = 0; i < 4; ++i) {  // C/D map: col = lane & 15 (code), row = 4 (lane >> 4) + i
          const float dist = (xr[q][i] - 2.f * c[q][i]) + ek;
          const bool take = kin && better(dist, k, bd[q][i], bk[q][i]);
          bd[q][i] = take ? dist : bd[q][i];
          bk[q][i] = take ? k : bk[q][i];
        }
    };
    // the buffer holding this stage's first tile alternates with the parity of
    // the tiles scored so far (no register copies)
    const int tpw = wave < ntile ? (ntile - wave + NWM - 1) / NWM : 0;
    auto stage_tiles = [&](float4 (&X)[DM / 16], float4 (&Y)[DM / 16]) {
      int p = (SEL_RVQ_ABL & 1) ? ntile : wave;
      for (; p + NWM < ntile; p += 2 * NWM) {
        tile(p, X, Y);
        tile(p + NWM, Y, X);
      }
      if (p < ntile) tile(p, X, Y);
    };
    if (((s * tpw) & 1) == 0)
      stage_tiles(cur, nxt);
    else
      stage_tiles(nxt, cur);
#pragma unroll
    for (int q = 0; q < RG; ++q)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float d0 = bd[q][i];
        int k0 = bk[q][i];
#pragma unroll
        for (int o = 8; o > 0; o >>= 1) {  // the 16 lanes of one row group
          const float d1 = __shfl_xor(d0, o, 64);
          const int k1 = __shfl_xor(k0, o, 64);
          if (better(d1, k1, d0, k0)) {
            d0 = d1;
            k0 = k1;
          }
        }
        if (col == 0) {
          red_d[wave][RM * q + 4 * h + i] = d0;
          red_k[wave][RM * q + 4 * h + i] = k0;
        }
      }
    __syncthreads();
    if (tid < RB) {
      float d0 = red_d[0][tid];
      int k0 = red_k[0][tid];
      for (int w = 1; w < NWM; ++w)
        if (better(red_d[w][tid], red_k[w][tid], d0, k0)) {
          d0 = red_d[w][tid];
          k0 = red_k[w][tid];
        }
      if constexpr (SEL_RVQ_ABL != 0) k0 = min(max(k0, 0), K - 1);  // ablations leave rows unscored
      sel_k[s][tid] = k0;
    }
    __syncthreads();
    float sq = 0.f;
    for (int i = tid; i < RB * D; i += TM) {
      const int r = i / D, d = i % D;
      if (r0 + r >= N) continue;
      const float rv = resT[d * RB + r];
      const float q = (SEL_RVQ_ABL & 4) ? rv : E[int64_t(d) * K + sel_k[s][r]];
      const float diff = q - rv;
      sq = fmaf(diff, diff, sq);
      const float qst = rv + diff;
      resT[d * RB + r] = rv - qst;
      acc_o[r * D + d] += qst;
    }
    sq_t[s][tid] = sq;
    __syncthreads();
  }
  for (int i = tid; i < RB * D; i += TM) {
    const int r = i / D, d = i % D;
    const int64_t row = r0 + r;
    if (row < N) out[row * D + d] = acc_o[r * D + d];
  }
  for (int i = tid; i < S * RB; i += TM) {
    const int st = i / RB, r = i % RB;
    if (r0 + r < N) idx[int64_t(st) * N + r0 + r] = sel_k[st][r];
  }
  for (int st = 0; st < S; ++st) {
    const double bs = block_sum<double>(double(sq_t[st][tid]), red);
    if (tid == 0) partials[int64_t(st) * gridDim.x + blockIdx.x] = bs;
  }
}

// code histogram of one stage's indices: LDS bins, then one global add per bin
constexpr int kHistRows = 4096;
constexpr int kHistMaxK = 8192;
// (round 6) the first block of each stage also sums the stage's per-block SSE
// partials into sqerr[s] -- k_rvq_sqerr's loop over the first 256 threads and
// the same block_sum (the other waves add exact zeros): one launch less
__global__ __launch_bounds__(512) void k_rvq_hist(const int64_t* __restrict__ idx, int64_t N, int K,
                                                  int32_t* __restrict__ counts, const double* __restrict__ partials,
                                                  int nb, double* __restrict__ sqerr) {
  __shared__ int32_t bins[kHistMaxK];
  __shared__ double red[16];
  const int s = blockIdx.y;
  if (blockIdx.x == 0) {  // block-uniform
    double v = 0.0;
    if (threadIdx.x < 256)
      for (int i = threadIdx.x; i < nb; i += 256) v += partials[int64_t(s) * nb + i];
    v = block_sum<double>(v, red);
    if (threadIdx.x == 0) sqerr[s] = v;
  }
  for (int k = threadIdx.x; k < K; k += blockDim.x) bins[k] = 0;
  __syncthreads();
  const int64_t a = int64_t(blockIdx.x) * kHistRows, b = std::min<int64_t>(N, a + kHistRows);
  for (int64_t i = a + threadIdx.x; i < b; i += blockDim.x) atomicAdd(&bins[idx[int64_t(s) * N + i]], 1);
  __syncthreads();
  for (int k = threadIdx.x; k < K; k += blockDim.x)
    if (bins[k]) atomicAdd(&counts[int64_t(s) * K + k], bins[k]);
}

inline size_t en_offset(int64_t N, int S) {
  const int64_t nb = (N + ROWS - 1) / ROWS;  // >= every variant's block count (16 / 20 rows)
  return (size_t(nb) * size_t(S) * sizeof(double) + 255) & ~size_t(255);
}
inline size_t ep_offset(int64_t N, int S, int K) {
  return (en_offset(N, S) + size_t(S) * size_t(K) * sizeof(float) + 255) & ~size_t(255);
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
  // per-block SSE partials, then |e|^2 per (stage, code) for the matrix-core variant
  // + the B-fragment-ordered codebook copy for the matrix-core variant (any D <= 64)
  if (N < 0 || S < 0 || K < 0) return 0;  // (sel_rvq_fwd rejects the shape itself)
  return ep_offset(N, S, K) + size_t(S) * size_t(MfmaGeo(DM, K).stage_floats()) * sizeof(float);
}

int sel_rvq_fwd(const float* x, int64_t N, int D, const float* embeds, int S, int K, float* out, int64_t* idx,
                int32_t* counts, double* sqerr, void* ws, size_t ws_bytes, sel_stream_t stream) {
  SEL_REQUIRE(N >= 0 && D > 0 && D <= MAXD && S > 0 && K > 0, SEL_ERR_ARG,
              "bad rvq shape N=%lld D=%d S=%d K=%d", (long long)N, D, S, K);
  SEL_REQUIRE(ws_bytes >= sel_rvq_workspace(N, S, K), SEL_ERR_WORKSPACE, "workspace too small");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  // tune key 2: 0 = matrix-core kernel where it applies, 1 = direct, 2 = staged
  const int variant = tune(2);
  const bool mfma = D % 4 == 0 && D <= DM && K <= kHistMaxK && S <= SM && variant == 0;
  // (the matrix-core path zeroes the histogram in k_rvq_prep)
  if (!mfma || N == 0) SEL_HIP(hipMemsetAsync(counts, 0, size_t(S) * K * sizeof(int32_t), s));
  const bool staged = !mfma && D % DC == 0 && K % 4 == 0 && variant != 1;
  // matrix-core rows per block: one 16-row group (tune key 39 = 2: two groups
  // sharing each codebook tile, measured slower at C3: 169 -> 193 us per RVQ
  // forward with its prep / histogram / finish, alternating in one call)
  const int mrows = tune(39) == 2 && (N + 2 * RM - 1) / (2 * RM) >= 128 ? 2 * RM : RM;
  const int rows = mfma ? mrows : staged ? R2 : ROWS;
  const int nb = int((N + rows - 1) / rows);
  double* part = static_cast<double*>(ws);
  if (nb > 0 && mfma) {
    float* en = reinterpret_cast<float*>(static_cast<char*>(ws) + en_offset(N, S));
    float* ep = reinterpret_cast<float*>(static_cast<char*>(ws) + ep_offset(N, S, K));
    const int64_t nprep = std::max<int64_t>(int64_t(S) * MfmaGeo(D, K).stage_floats() / 4, int64_t(S) * K);
    hipLaunchKernelGGL(k_rvq_prep, dim3(unsigned((nprep + 255) / 256)), dim3(256), 0, s, embeds, S, D, K, ep, en,
                       counts);
    SEL_LAUNCH_CHECK();
    const size_t lds = size_t(K) * sizeof(float);  // |e|^2 of one stage
    if (rows == 2 * RM) {
      SEL_HIP(hipFuncSetAttribute((const void*)k_rvq_mfma<2>, hipFuncAttributeMaxDynamicSharedMemorySize, int(lds)));
      hipLaunchKernelGGL(k_rvq_mfma<2>, dim3(nb), dim3(TM), lds, s, x, N, D, embeds, S, K, ep, en, out, idx, part);
    } else {
      SEL_HIP(hipFuncSetAttribute((const void*)k_rvq_mfma<1>, hipFuncAttributeMaxDynamicSharedMemorySize, int(lds)));
      hipLaunchKernelGGL(k_rvq_mfma<1>, dim3(nb), dim3(TM), lds, s, x, N, D, embeds, S, K, ep, en, out, idx, part);
    }
    SEL_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_rvq_hist, dim3(unsigned((N + kHistRows - 1) / kHistRows), unsigned(S)), dim3(512), 0, s,
                       idx, N, K, counts, part, nb, sqerr);
    SEL_LAUNCH_CHECK();
    return SEL_OK;  // (sqerr summed by k_rvq_hist)
  } else if (nb > 0 && staged) {
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
