// HiFi-GAN multi-scale + multi-period discriminator on gfx950
// (models/vocoder/HiFiGAN.py:308-395, models/vocoder/modules/discriminator.py:26-447)
// and the GAN losses (losses/adversarial_loss.py, losses/feat_match_loss.py).
//
// Every discriminator layer — the grouped, strided k41 Conv1d of the MSD, the
// (k,1) Conv2d of the MPD (a 1-D conv along T/p with the p columns as extra
// sequences), the dense k5/k3/k2 output convs — and every adjoint is ONE
// primitive (include/sel.h sel_dconv_desc):
//
//   out[b, j, col(g, o)] = sum_{i<K, r<S, c<Cg} Wp[g][o][i][r][c] * x[b, j+q0+i, r*Cs + g*Cg + c]
//
// over channels-last rows.  A stride-s conv is run on the PHASE VIEW of its
// input (rows of s consecutive samples: x[b, s*t + r, c] = view[b, t, r*C + c],
// a free reinterpretation when the row count is padded to a multiple of s), so
// it becomes a stride-1 conv with ceil(K/s)+1 taps over s*C channels and no
// wasted output rows; its adjoint is the same primitive on gout with So = s
// output phases.  Groups index disjoint channel slices, so no MFMA lane ever
// multiplies a structural zero of a grouped weight (a group narrower than the
// 32-wide MFMA tile is padded to 32 output channels; only the MSD's 8-input /
// 16-output-channel layer pays that, 2x on 4% of the flops).
//
//   MFMA kernel (Cg % 8 == 0): v_mfma_f32_32x32x16_bf16 (bf16 path) or
//     v_mfma_f32_32x32x2_f32 (exact-fp32 parity path).  Reduction vectors are
//     8 consecutive channels of one (tap, phase): each 32-lane half of a wave
//     feeds one vector per MFMA.  The input span of a BM-row tile is staged once
//     per 32-channel chunk and re-read by every tap; weights are staged per tap
//     group.  Epilogue: + bias, LeakyReLU, or (+ res) * LeakyReLU'(aux) for the
//     adjoint, rows past Tvalid written as exact zeros (the next layer's padding).
//   VALU kernel: the 1-channel input / 1-channel output layers (first and last
//     conv of every sub-discriminator and their adjoints), where a 32-wide MFMA
//     tile would be 1/32 useful.
//   Weight gradient: gW = sum_rows gout^T x as split-row partials (MFMA with
//     transposing LDS reads for bf16, VALU for fp32 / thin layers), then one
//     deterministic reduction fused with the unpack to the torch layout and the
//     weight-norm backward (torch.nn.utils.weight_norm, used by the MPD).
#include <algorithm>

#include "sel_common.h"

namespace sel {
namespace conv {
// conv.hip: discriminator layers on the generator's warp-specialised kernel
int dconv_ws_fwd(const sel_dconv_desc* d, const void* x, const void* wp, const float* bias, const void* aux,
                 const void* res, void* out, hipStream_t s);
// -1: shape not supported there, 0: per-sequence tiles, 1: flat tiles across sequences
int dconv_ws_mode(const sel_dconv_desc* d);
// true: dconv_ws_fwd runs the shape on the eight-wave 256 x 256 kernel (k_conv_ws8)
bool dconv_ws8_ok(const sel_dconv_desc* d);
}  // namespace conv
namespace dconv {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef short v8i16 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ float to_f(float v) { return v; }
__device__ __forceinline__ float to_f(__bf16 v) { return float(v); }
template <typename T> __device__ __forceinline__ T from_f(float v);
template <> __device__ __forceinline__ float from_f<float>(float v) { return v; }
template <> __device__ __forceinline__ __bf16 from_f<__bf16>(float v) { return __bf16(v); }

// XCD-aware tile order of the row-tile x (group, column tile) grids: the
// launcher rounds grid.x (row tiles) up to a multiple of 8; linear block ids
// are dealt round-robin to the 8 XCDs, so decoding id -> (xcd = id % 8, slot =
// id / 8) -> (row tile 8 (slot / ny) + xcd, y = slot % ny) puts every (group,
// column) block of one row tile on ONE XCD, one after the other: the input rows
// they all read (a grouped layer's blocks each read a 64-B slice of every row)
// are fetched into that XCD's L2 once.  false: a padding block (row tile >= nx).
// (C5, alternating in one call: 45.14 / 45.05 ms per step against 45.21 / 45.24
// with the plain 2-D order)
__device__ __forceinline__ bool xcd_rowtile(int nx, int& rt, int& y) {
  const int ny = gridDim.y;
  const int64_t id = int64_t(blockIdx.y) * gridDim.x + blockIdx.x;
  const int64_t slot = id >> 3;
  rt = int((slot / ny) * 8 + (id & 7));
  y = int(slot % ny);
  return rt < nx;
}

__device__ __forceinline__ float leaky(float v, float s) { return v > 0.f ? v : v * s; }
__device__ __forceinline__ float leaky_grad(float y, float s) { return y > 0.f ? 1.f : s; }

using D = sel_dconv_desc;

__device__ __forceinline__ int64_t in_col(const D& d, int g, int r, int c) {
  return int64_t(r) * d.Cs + int64_t(g) * d.Cg + c;
}
__device__ __forceinline__ int64_t out_col(const D& d, int g, int o) {
  const int ro = o / d.Ng, no = o - ro * d.Ng;
  return int64_t(ro) * d.Ns + int64_t(g) * d.Ng + no;
}

template <typename T> struct Elt;
template <> struct Elt<__bf16> { static constexpr int VEC = 8; static constexpr int P = 40; };  // 80-B LDS rows
template <> struct Elt<float> { static constexpr int VEC = 4; static constexpr int P = 36; };   // 144-B LDS rows

constexpr int CH = 32;  // reduction channels per staged chunk
constexpr int KC = 8;   // taps per staged weight group

// ---------------------------------------------------------------------------
// MFMA primitive.  Block = BM output rows of one sequence x BN local output
// channels of one group; 4 waves as 2 x 2 (wave tile BM/2 x BN/2, 32x32 MFMA
// sub-tiles).  LDS: x span [BM + K - 1][P] of the current 32-channel chunk,
// weights [BN][KC][P] of the current tap group.
// ---------------------------------------------------------------------------
// Epilogue of one 32x32 accumulator (operands swapped: lane -> output row
// lane & 31, element e -> output channel ob + (e & 3) + 8 (e >> 2) + 4 (lane >> 5)):
// + bias, + res, * LeakyReLU'(aux), LeakyReLU; rows past Tvalid written as exact
// zeros.  bf16 with contiguous output columns (col = col0 + o - o0): each run
// of 4 channels is one 8-byte load / store; otherwise per element.
template <typename T>
__device__ __forceinline__ void dconv_epilogue(const D& d, int g, int ob, int no_per_g, int64_t orow, bool valid,
                                               const floatx16& a, const float* __restrict__ bias,
                                               const T* __restrict__ aux, const T* __restrict__ res,
                                               T* __restrict__ out, bool contig) {
  const int hl = (threadIdx.x & 63) >> 5;
  if constexpr (sizeof(T) == 2) {
    if (contig) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int o = ob + 8 * q + 4 * hl;
        if (o >= no_per_g) continue;  // no_per_g % 4 == 0 (contig)
        const int64_t col = out_col(d, g, o);
        typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
        bf16x4 rv = {}, av = {}, ov;
        if (valid && res) rv = *reinterpret_cast<const bf16x4*>(res + orow + col);
        if (valid && aux) av = *reinterpret_cast<const bf16x4*>(aux + orow + col);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float v = 0.f;
          if (valid) {
            v = a[4 * q + e];
            if (bias) v += bias[col + e];
            if (res) v += float(rv[e]);
            if (aux) v *= leaky_grad(float(av[e]), d.slope);
            if (d.act) v = leaky(v, d.slope);
          }
          ov[e] = __bf16(v);
        }
        *reinterpret_cast<bf16x4*>(out + orow + col) = ov;
      }
      return;
    }
  }
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int o = ob + (e & 3) + 8 * (e >> 2) + 4 * hl;
    if (o >= no_per_g) continue;
    const int64_t col = out_col(d, g, o);
    float v = 0.f;
    if (valid) {
      v = a[e];
      if (bias) v += bias[col];
      if (res) v += to_f(res[orow + col]);
      if (aux) v *= leaky_grad(to_f(aux[orow + col]), d.slope);
      if (d.act) v = leaky(v, d.slope);
    }
    out[orow + col] = from_f<T>(v);
  }
}

// output columns of a group contiguous in runs of 4 (8-byte aligned)
__device__ __forceinline__ bool dconv_contig4(const D& d) {
  return (d.So == 1 || d.Ns == d.Ng) && (d.Ng & 3) == 0 && (d.ldo & 3) == 0 && (d.G == 1 || d.So == 1);
}

template <typename T, int BM, int BN>
__global__ __launch_bounds__(256) void k_dconv_mfma(D d, const T* __restrict__ x, const T* __restrict__ wp,
                                                    const float* __restrict__ bias, const T* __restrict__ aux,
                                                    const T* __restrict__ res, T* __restrict__ out) {
  constexpr int P = Elt<T>::P;
  constexpr int VEC = Elt<T>::VEC;
  constexpr int WAVES_N = BN / 32, WAVES_M = 4 / WAVES_N;
  constexpr int TM = BM / (32 * WAVES_M);
  static_assert(TM >= 1 && WAVES_N * WAVES_M == 4, "tile");
  extern __shared__ __align__(16) unsigned char smem[];
  T* const xs = reinterpret_cast<T*>(smem);
  const int span = BM + d.K - 1;
  T* const ws = xs + span * P;  // [BN][KC][P]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int tps = (d.Tvo + BM - 1) / BM;
  int rt_, by_;
  if (!xcd_rowtile(d.B * tps, rt_, by_)) return;
  const int b = rt_ / tps;
  const int j0 = (rt_ % tps) * BM;
  const int no_per_g = d.So * d.Ng;
  const int ntile_g = (no_per_g + BN - 1) / BN;
  const int g = by_ / ntile_g;
  const int o0 = (by_ % ntile_g) * BN;
  const int64_t xrow0 = int64_t(b) * d.Tvs;
  const int nred = d.S * d.Cg;  // reduction channels per tap

  floatx16 acc[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[i][e] = 0.f;

  // this lane's output rows (B operand column) and channel (A operand row)
  int lrow[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) lrow[i] = wm * (BM / WAVES_M) + i * 32 + (lane & 31);
  const int half = lane >> 5;
  const int nw_ = wn * 32 + (lane & 31);
  const int vpr = CH / VEC;

  for (int cc = 0; cc < nred; cc += CH) {
    const int chn = nred - cc < CH ? nred - cc : CH;  // multiple of 8 (host-checked)
    __syncthreads();
    // stage x span rows [j0 + q0, j0 + q0 + span) x chunk channels (vectors of VEC)
    for (int idx = tid; idx < span * vpr; idx += 256) {
      const int rr = idx / vpr, v = idx % vpr;
      const int t = j0 + d.q0 + rr;
      const int ch = cc + v * VEC;
      uint4 val = make_uint4(0, 0, 0, 0);
      if (t >= 0 && t < d.Tv && v * VEC < chn) {
        const int rph = ch / d.Cg, c = ch - rph * d.Cg;
        val = *reinterpret_cast<const uint4*>(x + (xrow0 + t) * d.ldx + in_col(d, g, rph, c));
      }
      *reinterpret_cast<uint4*>(xs + rr * P + v * VEC) = val;
    }
    for (int k0 = 0; k0 < d.K; k0 += KC) {
      const int kn = d.K - k0 < KC ? d.K - k0 : KC;
      if (k0) __syncthreads();
      for (int idx = tid; idx < BN * KC * vpr; idx += 256) {
        const int v = idx % vpr, kk = (idx / vpr) % KC, n = idx / (vpr * KC);
        uint4 val = make_uint4(0, 0, 0, 0);
        if (kk < kn && o0 + n < no_per_g && v * VEC < chn)
          val = *reinterpret_cast<const uint4*>(
              wp + ((int64_t(g) * no_per_g + o0 + n) * d.K + k0 + kk) * nred + cc + v * VEC);
        *reinterpret_cast<uint4*>(ws + (n * KC + kk) * P + v * VEC) = val;
      }
      __syncthreads();
      for (int kk = 0; kk < kn; ++kk) {
        const int k = k0 + kk;
        if constexpr (sizeof(T) == 2) {
#pragma unroll
          for (int h = 0; h < CH / 16; ++h) {
            if (h * 16 >= chn) break;
            const int co = 16 * h + 8 * half;
            const bf16x8 bw = *reinterpret_cast<const bf16x8*>(ws + (nw_ * KC + kk) * P + co);
#pragma unroll
            for (int i = 0; i < TM; ++i) {
              const bf16x8 af = *reinterpret_cast<const bf16x8*>(xs + (lrow[i] + k) * P + co);
              acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bw, af, acc[i], 0, 0, 0);
            }
          }
        } else {
          for (int c2 = 0; c2 < chn; c2 += 2) {
            const int co = c2 + half;
            const float bw = ws[(nw_ * KC + kk) * P + co];
#pragma unroll
            for (int i = 0; i < TM; ++i) {
              const float af = xs[(lrow[i] + k) * P + co];
              acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(bw, af, acc[i], 0, 0, 0);
            }
          }
        }
      }
    }
  }

  // epilogue (operands swapped: lane -> output row lane & 31 of its sub-tile,
  // element e -> channel (e & 3) + 8 (e >> 2) + 4 (lane >> 5) of the wave's 32)
  const bool contig = dconv_contig4(d);
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int j = j0 + lrow[i];
    if (j >= d.Tvo) continue;
    const int64_t orow = (int64_t(b) * d.Tvo + j) * d.ldo;
    dconv_epilogue<T>(d, g, o0 + wn * 32, no_per_g, orow, j < d.Tvalid, acc[i], bias, aux, res, out, contig);
  }
}

// ---------------------------------------------------------------------------
// k_dconv_mfma with a register-prefetched pipeline (bf16): the (32-channel
// chunk, 8-tap group) stages run in the same order with the same MFMAs (same
// bits), but the next stage's weight slice (and, at a chunk boundary, the next
// input span) is fetched into registers while the current stage's MFMAs run;
// k_dconv_mfma staged both synchronously, exposing a load latency per stage
// (the MSD's 41-tap grouped convs: 2 chunks x 6 tap groups per tile).
// ---------------------------------------------------------------------------
template <int BM, int BN>
__global__ __launch_bounds__(256) void k_dconv_gpf(D d, const __bf16* __restrict__ x, const __bf16* __restrict__ wp,
                                                   const float* __restrict__ bias, const __bf16* __restrict__ aux,
                                                   const __bf16* __restrict__ res, __bf16* __restrict__ out) {
  constexpr int P = Elt<__bf16>::P;
  constexpr int WAVES_N = BN / 32, WAVES_M = 4 / WAVES_N;
  constexpr int TM = BM / (32 * WAVES_M);
  constexpr int XV = ((BM + KC * 8) * 4 + 255) / 256;  // span rows (<= BM + K - 1 <= BM + 63) x 4 vectors
  constexpr int WV = (BN * KC * 4 + 255) / 256;
  static_assert(TM >= 1 && WAVES_N * WAVES_M == 4, "tile");
  extern __shared__ __align__(16) unsigned char smem[];
  __bf16* const xs = reinterpret_cast<__bf16*>(smem);
  const int span = BM + d.K - 1;
  __bf16* const ws = xs + span * P;  // [BN][KC][P]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int tps = (d.Tvo + BM - 1) / BM;
  int rt_, by_;
  if (!xcd_rowtile(d.B * tps, rt_, by_)) return;
  const int b = rt_ / tps;
  const int j0 = (rt_ % tps) * BM;
  const int no_per_g = d.So * d.Ng;
  const int ntile_g = (no_per_g + BN - 1) / BN;
  const int g = by_ / ntile_g;
  const int o0 = (by_ % ntile_g) * BN;
  const int64_t xrow0 = int64_t(b) * d.Tvs;
  const int nred = d.S * d.Cg;
  const int nchunk = (nred + CH - 1) / CH;
  const int ntg = (d.K + KC - 1) / KC;
  const int nstage = nchunk * ntg;

  floatx16 acc[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[i][e] = 0.f;
  int lrow[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) lrow[i] = wm * (BM / WAVES_M) + i * 32 + (lane & 31);
  const int half = lane >> 5;
  const int nw_ = wn * 32 + (lane & 31);

  uint4 xr[XV], wr[WV];
  bool xok[XV], wok[WV];
  auto load_x = [&](int cc) {
#pragma unroll
    for (int u = 0; u < XV; ++u) {
      const int idx = tid + u * 256;
      const int rr = idx >> 2, v = idx & 3;
      const int t = j0 + d.q0 + rr;
      const int ch = cc + v * 8;
      xok[u] = rr < span && t >= 0 && t < d.Tv && ch < nred;
      const int rph = (xok[u] ? ch : 0) / d.Cg, c = (xok[u] ? ch : 0) - rph * d.Cg;
      if ((u * 256) / 4 < span)
        xr[u] = *reinterpret_cast<const uint4*>(x + (xrow0 + (xok[u] ? t : 0)) * d.ldx + in_col(d, g, rph, c));
    }
  };
  auto store_x = [&]() {
#pragma unroll
    for (int u = 0; u < XV; ++u) {
      const int idx = tid + u * 256;
      const int rr = idx >> 2, v = idx & 3;
      if (rr >= span) continue;
      *reinterpret_cast<uint4*>(xs + rr * P + v * 8) = xok[u] ? xr[u] : make_uint4(0, 0, 0, 0);
    }
  };
  auto load_w = [&](int cc, int k0) {
    const int kn = d.K - k0 < KC ? d.K - k0 : KC;
#pragma unroll
    for (int u = 0; u < WV; ++u) {
      const int idx = tid + u * 256;
      const int v = idx & 3, kk = (idx >> 2) % KC, n = idx / (4 * KC);
      wok[u] = n < BN && kk < kn && o0 + n < no_per_g && cc + v * 8 < nred;
      wr[u] = *reinterpret_cast<const uint4*>(
          wp + ((int64_t(g) * no_per_g + (wok[u] ? o0 + n : 0)) * d.K + (wok[u] ? k0 + kk : 0)) * nred +
          (wok[u] ? cc + v * 8 : 0));
    }
  };
  auto store_w = [&]() {
#pragma unroll
    for (int u = 0; u < WV; ++u) {
      const int idx = tid + u * 256;
      const int v = idx & 3, kk = (idx >> 2) % KC, n = idx / (4 * KC);
      if (n >= BN) continue;
      *reinterpret_cast<uint4*>(ws + (n * KC + kk) * P + v * 8) = wok[u] ? wr[u] : make_uint4(0, 0, 0, 0);
    }
  };

  load_x(0);
  load_w(0, 0);
  for (int st = 0; st < nstage; ++st) {
    const int ci = st / ntg, tg = st - ci * ntg;
    const int cc = ci * CH, k0 = tg * KC;
    __syncthreads();  // every wave is done with the previous stage's LDS
    if (tg == 0) store_x();
    store_w();
    __syncthreads();
    if (st + 1 < nstage) {  // next stage's operands in flight during this stage's MFMAs
      const int ci1 = (st + 1) / ntg, tg1 = (st + 1) - ci1 * ntg;
      if (tg1 == 0) load_x(ci1 * CH);
      load_w(ci1 * CH, tg1 * KC);
    }
    const int kn = d.K - k0 < KC ? d.K - k0 : KC;
    const int chn = nred - cc < CH ? nred - cc : CH;
    for (int kk = 0; kk < kn; ++kk) {
      const int k = k0 + kk;
#pragma unroll
      for (int h = 0; h < CH / 16; ++h) {
        if (h * 16 >= chn) break;
        const int co = 16 * h + 8 * half;
        const bf16x8 bw = *reinterpret_cast<const bf16x8*>(ws + (nw_ * KC + kk) * P + co);
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const bf16x8 af = *reinterpret_cast<const bf16x8*>(xs + (lrow[i] + k) * P + co);
          acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bw, af, acc[i], 0, 0, 0);
        }
      }
    }
  }

  const bool contig = dconv_contig4(d);
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int j = j0 + lrow[i];
    if (j >= d.Tvo) continue;
    const int64_t orow = (int64_t(b) * d.Tvo + j) * d.ldo;
    dconv_epilogue<__bf16>(d, g, o0 + wn * 32, no_per_g, orow, j < d.Tvalid, acc[i], bias, aux, res, out, contig);
  }
}

// ---------------------------------------------------------------------------
// Register-prefetched MFMA primitive for one group with a contiguous reduction
// row (G == 1, S == 1 or Cs == Cg: every MPD layer and the MSD's dense ones)
// and K <= 8 taps: the next 32-channel chunk's input span and ALL K weight
// slices are fetched into registers while the current chunk's MFMAs run (the
// tap-grouped kernel above stages each chunk synchronously: ~5% of the bf16
// peak on the MPD's 512/1024-wide layers, profiles/r2_c5_kernel_stats.md).
// ---------------------------------------------------------------------------
constexpr int PF_KMAX = 8;

template <int BM, int BN>
__global__ __launch_bounds__(256) void k_dconv_pf(D d, const __bf16* __restrict__ x, const __bf16* __restrict__ wp,
                                                  const float* __restrict__ bias, const __bf16* __restrict__ aux,
                                                  const __bf16* __restrict__ res, __bf16* __restrict__ out) {
  constexpr int P = Elt<__bf16>::P;
  constexpr int WAVES_N = BN / 32, WAVES_M = 4 / WAVES_N;
  constexpr int TM = BM / (32 * WAVES_M);
  constexpr int XV = ((BM + PF_KMAX - 1) * 4 + 255) / 256;
  constexpr int WV = (PF_KMAX * BN * 4 + 255) / 256;
  static_assert(TM >= 1 && WAVES_N * WAVES_M == 4, "tile");
  extern __shared__ __align__(16) unsigned char smem[];
  __bf16* const xs = reinterpret_cast<__bf16*>(smem);
  const int span = BM + d.K - 1;
  __bf16* const ws = xs + span * P;  // [K][BN][P]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int hl = lane >> 5;
  const int tps = (d.Tvo + BM - 1) / BM;
  int rt_, by_;
  if (!xcd_rowtile(d.B * tps, rt_, by_)) return;
  const int b = rt_ / tps;
  const int j0 = (rt_ % tps) * BM;
  const int no_per_g = d.So * d.Ng;
  const int o0 = by_ * BN;
  const int nred = d.S * d.Cg;
  const int nchunk = (nred + CH - 1) / CH;

  const __bf16* xsrc[XV];
  bool xok[XV];
  int xsub[XV];
#pragma unroll
  for (int u = 0; u < XV; ++u) {
    const int v = tid + u * 256, rr = v >> 2;
    const int t = j0 + d.q0 + rr;
    xok[u] = rr < span && t >= 0 && t < d.Tv;
    xsub[u] = (v & 3) * 8;
    xsrc[u] = x + (int64_t(b) * d.Tvs + (xok[u] ? t : 0)) * d.ldx + xsub[u];
  }
  const __bf16* wsrc[WV];
  bool wok[WV];
#pragma unroll
  for (int u = 0; u < WV; ++u) {
    const int v = tid + u * 256;
    const int k = v / (BN * 4), n = (v >> 2) % BN;
    wok[u] = k < d.K && o0 + n < no_per_g;
    wsrc[u] = wp + (int64_t(wok[u] ? o0 + n : 0) * d.K + (wok[u] ? k : 0)) * nred + (v & 3) * 8;
  }
  uint4 xr[XV], wr[WV];
  auto load = [&](int cc) {
#pragma unroll
    for (int u = 0; u < XV; ++u)
      if ((u * 256) / 4 < span) xr[u] = *reinterpret_cast<const uint4*>(xsrc[u] + (cc + xsub[u] < nred ? cc : 0));
#pragma unroll
    for (int u = 0; u < WV; ++u)
      if ((u * 256) / (BN * 4) < d.K) wr[u] = *reinterpret_cast<const uint4*>(wsrc[u] + (cc + (((tid + u * 256) & 3) * 8) < nred ? cc : 0));
  };
  auto store = [&](int cc) {
#pragma unroll
    for (int u = 0; u < XV; ++u) {
      const int v = tid + u * 256;
      if ((v >> 2) >= span) continue;
      const uint4 val = (xok[u] && cc + xsub[u] < nred) ? xr[u] : make_uint4(0, 0, 0, 0);
      *reinterpret_cast<uint4*>(xs + (v >> 2) * P + xsub[u]) = val;
    }
#pragma unroll
    for (int u = 0; u < WV; ++u) {
      const int v = tid + u * 256;
      const int k = v / (BN * 4), n = (v >> 2) % BN;
      if (k >= d.K) continue;
      const uint4 val = (wok[u] && cc + (v & 3) * 8 < nred) ? wr[u] : make_uint4(0, 0, 0, 0);
      *reinterpret_cast<uint4*>(ws + (k * BN + n) * P + (v & 3) * 8) = val;
    }
  };

  floatx16 acc[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[i][e] = 0.f;
  int lrow[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) lrow[i] = wm * (BM / WAVES_M) + i * 32 + (lane & 31);
  const int nw_ = wn * 32 + (lane & 31);

  load(0);
  for (int ch = 0; ch < nchunk; ++ch) {
    const int cc = ch * CH;
    if (ch) __syncthreads();
    store(cc);
    __syncthreads();
    if (ch + 1 < nchunk) load(cc + CH);
    const int chn = nred - cc < CH ? nred - cc : CH;
    for (int k = 0; k < d.K; ++k) {
#pragma unroll
      for (int h = 0; h < CH / 16; ++h) {
        if (h * 16 >= chn) break;
        const int co = 16 * h + 8 * hl;
        const bf16x8 bw = *reinterpret_cast<const bf16x8*>(ws + (k * BN + nw_) * P + co);
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const bf16x8 af = *reinterpret_cast<const bf16x8*>(xs + (lrow[i] + k) * P + co);
          acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bw, af, acc[i], 0, 0, 0);
        }
      }
    }
  }

  // epilogue as k_dconv_mfma
  const bool contig = dconv_contig4(d);
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int j = j0 + lrow[i];
    if (j >= d.Tvo) continue;
    const int64_t orow = (int64_t(b) * d.Tvo + j) * d.ldo;
    dconv_epilogue<__bf16>(d, 0, o0 + wn * 32, no_per_g, orow, j < d.Tvalid, acc[i], bias, aux, res, out, contig);
  }
}

// ---------------------------------------------------------------------------
// VALU primitive (any Cg; used when S*Cg*K or the group output width is tiny).
// One thread per (row, output channel); the reduction walks (i, r, c).
// ---------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void k_dconv_valu(D d, const T* __restrict__ x, const T* __restrict__ wp,
                                                    const float* __restrict__ bias, const T* __restrict__ aux,
                                                    const T* __restrict__ res, T* __restrict__ out) {
  const int no_per_g = d.So * d.Ng;
  const int64_t nout = int64_t(d.G) * no_per_g;
  const int64_t total = int64_t(d.B) * d.Tvo * nout;
  const int nred = d.S * d.Cg;
  for (int64_t idx = int64_t(blockIdx.x) * 256 + threadIdx.x; idx < total; idx += int64_t(gridDim.x) * 256) {
    const int64_t row = idx / nout;
    const int oc = int(idx - row * nout);
    const int g = oc / no_per_g, o = oc - g * no_per_g;
    const int b = int(row / d.Tvo), j = int(row - int64_t(b) * d.Tvo);
    const int64_t orow = row * d.ldo;
    const int64_t col = out_col(d, g, o);
    float v = 0.f;
    if (j < d.Tvalid) {
      const T* w = wp + (int64_t(g) * no_per_g + o) * d.K * nred;
      for (int i = 0; i < d.K; ++i) {
        const int t = j + d.q0 + i;
        if (t < 0 || t >= d.Tv) continue;
        const T* xr = x + (int64_t(b) * d.Tvs + t) * d.ldx;
        for (int r = 0; r < d.S; ++r)
          for (int c = 0; c < d.Cg; ++c) v += to_f(w[i * nred + r * d.Cg + c]) * to_f(xr[in_col(d, g, r, c)]);
      }
      if (bias) v += bias[col];
      if (res) v += to_f(res[orow + col]);
      if (aux) v *= leaky_grad(to_f(aux[orow + col]), d.slope);
      if (d.act) v = leaky(v, d.slope);
    }
    out[orow + col] = from_f<T>(v);
  }
}

// Short-reduction primitive (K * S * Cg <= 64, one group, single output phase,
// Ng % 8 == 0): the 1-channel-input convs (MSD k15, MPD k5/s3 -> 2 taps x 3
// phases) and the adjoints of the 1-channel-output convs.  One thread = one
// output row x 8 consecutive channels: the row's input window in registers, the
// weights in LDS (fp32), one 16-B (bf16) / 32-B (fp32) store.

template <typename T, int KR>
__global__ __launch_bounds__(256) void k_dconv_short(D d, const T* __restrict__ x, const T* __restrict__ wp,
                                                     const float* __restrict__ bias, const T* __restrict__ aux,
                                                     const T* __restrict__ res, T* __restrict__ out) {
  constexpr int RW = 4;   // rows per thread: each weight read from LDS serves RW rows
  extern __shared__ float wsh[];  // [K * nred][Ng] (transposed: a thread's 8 channels are 2 float4)
  const int nred = d.S * d.Cg;
  for (int e = threadIdx.x; e < d.Ng * KR; e += 256) {
    const int n = e / KR, k = e - n * KR;
    wsh[k * d.Ng + n] = to_f(wp[e]);
  }
  __syncthreads();
  // tap offset and input column of reduction element e (kernel-uniform: hoisted
  // out of the row loop, where the runtime divisions cost ~60 VALU per element)
  int tap[KR], col[KR];
#pragma unroll
  for (int e = 0; e < KR; ++e) {
    const int i = e / nred, rc = e - i * nred;
    const int r = rc / d.Cg, c = rc - r * d.Cg;
    tap[e] = d.q0 + i;
    col[e] = int(in_col(d, 0, r, c));
  }
  const int n8 = d.Ng / 8;
  const int rows = d.B * d.Tvo;  // < 2^31 (host check)
  const int total = (rows + RW - 1) / RW * n8;
  for (int idx = int(blockIdx.x) * 256 + threadIdx.x; idx < total; idx += int(gridDim.x) * 256) {
    const int rg = idx / n8;
    const int n0 = (idx - rg * n8) * 8;
    float xw[RW][KR];
    int64_t orow[RW];
    bool valid[RW];
    int row = rg * RW, b = row / d.Tvo, j = row - b * d.Tvo;
#pragma unroll
    for (int q = 0; q < RW; ++q) {
      orow[q] = row < rows ? int64_t(row) * d.ldo : -1;
      valid[q] = row < rows && j < d.Tvalid;
      const T* xb = x + int64_t(b) * d.Tvs * d.ldx;
#pragma unroll
      for (int e = 0; e < KR; ++e) {
        const int t = j + tap[e];
        xw[q][e] = (valid[q] && t >= 0 && t < d.Tv) ? to_f(xb[int64_t(t) * d.ldx + col[e]]) : 0.f;
      }
      ++row;
      if (++j == d.Tvo) j = 0, ++b;
    }
    float acc[RW][8];
#pragma unroll
    for (int q = 0; q < RW; ++q)
#pragma unroll
      for (int c = 0; c < 8; ++c) acc[q][c] = 0.f;
#pragma unroll
    for (int e = 0; e < KR; ++e) {
      const float4 w0 = *reinterpret_cast<const float4*>(wsh + e * d.Ng + n0);
      const float4 w1 = *reinterpret_cast<const float4*>(wsh + e * d.Ng + n0 + 4);
      const float w[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
#pragma unroll
      for (int q = 0; q < RW; ++q)
#pragma unroll
        for (int c = 0; c < 8; ++c) acc[q][c] = fmaf(w[c], xw[q][e], acc[q][c]);
    }
#pragma unroll
    for (int q = 0; q < RW; ++q) {
      if (orow[q] < 0) continue;
      T ov[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        float a = 0.f;
        if (valid[q]) {
          const int64_t col = n0 + c;
          a = acc[q][c];
          if (bias) a += bias[col];
          if (res) a += to_f(res[orow[q] + col]);
          if (aux) a *= leaky_grad(to_f(aux[orow[q] + col]), d.slope);
          if (d.act) a = leaky(a, d.slope);
        }
        ov[c] = from_f<T>(a);
      }
      if constexpr (sizeof(T) == 2) {
        *reinterpret_cast<uint4*>(out + orow[q] + n0) = *reinterpret_cast<uint4*>(ov);
      } else {
        *reinterpret_cast<uint4*>(out + orow[q] + n0) = *reinterpret_cast<uint4*>(ov);
        *reinterpret_cast<uint4*>(out + orow[q] + n0 + 4) = *reinterpret_cast<uint4*>(ov + 4);
      }
    }
  }
}

// Staged form of the short-reduction forward for a contiguous phase view (G = 1,
// Cs = Cg, ldx = S*Cg = NR: the 1-channel-input convs): reduction element
// e = i*NR + rc of output row j reads x[j + q0 + i][rc], i.e. the flat window
// xs[(j - j0)*NR + e] of a tile staged once in LDS.  k_dconv_short issues KR
// per-lane global loads per row (the MSD's k15 1 -> 128 conv: 60 loads per
// thread, bound by the texture unit's address rate at 645 us for 393 MB of
// output); here a thread's RW rows read one (RW + K - 1)*NR-float window from LDS.
template <typename T, int K, int NR>
__global__ __launch_bounds__(256) void k_dconv_shortx(D d, const T* __restrict__ x, const T* __restrict__ wp,
                                                      const float* __restrict__ bias, const T* __restrict__ aux,
                                                      const T* __restrict__ res, T* __restrict__ out) {
  constexpr int KR = K * NR, RW = 8, XW = (RW + K - 1) * NR;
  extern __shared__ float sh[];
  float* const wsh = sh;            // [KR][Ng]
  float* const xs = sh + KR * d.Ng;  // [(RB + K - 1) * NR]
  for (int e = threadIdx.x; e < d.Ng * KR; e += 256) {
    const int n = e / KR, k = e - n * KR;
    wsh[k * d.Ng + n] = to_f(wp[e]);
  }
  const int n8 = d.Ng / 8, RL = 256 / n8, RB = RL * RW;
  const int rl = threadIdx.x / n8, n0 = (threadIdx.x - rl * n8) * 8;
  const int tps = (d.Tvo + RB - 1) / RB, ntiles = d.B * tps;
  // (a one-tile-ahead register fetch of the window was measured neutral on C5
  // in round 2 and dropped)
  const int np = (RB + K - 1) * NR;
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int b = tile / tps, j0 = (tile - b * tps) * RB;
    __syncthreads();  // the previous tile's window reads are done (and the weights are in)
    for (int p = threadIdx.x; p < np; p += 256) {
      const int t = j0 + d.q0 + p / NR;
      xs[p] = (t >= 0 && t < d.Tv) ? to_f(x[(int64_t(b) * d.Tvs + t) * NR + p % NR]) : 0.f;
    }
    __syncthreads();
    const int jr = rl * RW;
    if (j0 + jr >= d.Tvo) continue;
    float xw[XW];
#pragma unroll
    for (int u = 0; u < XW; ++u) xw[u] = xs[jr * NR + u];
    // channel pairs as 2-vectors: one packed fp32 FMA (v_pk_fma_f32) per pair,
    // per element the same fused multiply-add as fmaf, so bit-identical
    typedef float shx_f2 __attribute__((ext_vector_type(2)));
    shx_f2 acc2[RW][4];
#pragma unroll
    for (int q = 0; q < RW; ++q)
#pragma unroll
      for (int c = 0; c < 4; ++c) acc2[q][c] = shx_f2{0.f, 0.f};
#pragma unroll
    for (int e = 0; e < KR; ++e) {
      const float4 w0 = *reinterpret_cast<const float4*>(wsh + e * d.Ng + n0);
      const float4 w1 = *reinterpret_cast<const float4*>(wsh + e * d.Ng + n0 + 4);
      const shx_f2 w[4] = {shx_f2{w0.x, w0.y}, shx_f2{w0.z, w0.w}, shx_f2{w1.x, w1.y}, shx_f2{w1.z, w1.w}};
#pragma unroll
      for (int q = 0; q < RW; ++q) {
        const float xv = xw[q * NR + e];
        const shx_f2 x2 = shx_f2{xv, xv};
#pragma unroll
        for (int c = 0; c < 4; ++c) acc2[q][c] = __builtin_elementwise_fma(w[c], x2, acc2[q][c]);
      }
    }
    float acc[RW][8];
#pragma unroll
    for (int q = 0; q < RW; ++q)
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[q][2 * c] = acc2[q][c].x, acc[q][2 * c + 1] = acc2[q][c].y;
#pragma unroll
    for (int q = 0; q < RW; ++q) {
      const int j = j0 + jr + q;
      if (j >= d.Tvo) break;
      const int64_t orow = (int64_t(b) * d.Tvo + j) * d.ldo;
      const bool valid = j < d.Tvalid;
      T ov[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        float a = 0.f;
        if (valid) {
          const int64_t col = n0 + c;
          a = acc[q][c];
          if (bias) a += bias[col];
          if (res) a += to_f(res[orow + col]);
          if (aux) a *= leaky_grad(to_f(aux[orow + col]), d.slope);
          if (d.act) a = leaky(a, d.slope);
        }
        ov[c] = from_f<T>(a);
      }
      if constexpr (sizeof(T) == 2) {
        *reinterpret_cast<uint4*>(out + orow + n0) = *reinterpret_cast<uint4*>(ov);
      } else {
        *reinterpret_cast<uint4*>(out + orow + n0) = *reinterpret_cast<uint4*>(ov);
        *reinterpret_cast<uint4*>(out + orow + n0 + 4) = *reinterpret_cast<uint4*>(ov + 4);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Weight gradient partials.  gW[g][o][i][r][c] = sum over rows (b, j < Tvalid)
// of gout[b, j, col(g, o)] * x[b, j + q0 + i, r*Cs + g*Cg + c]; bias partials
// gb[col] = sum gout.  part[split][...] (fp32), reduced by k_dwgrad_finish.
// ---------------------------------------------------------------------------
// VALU: thread per weight element, rows of its split.
template <typename T>
__global__ __launch_bounds__(256) void k_dwgrad_valu(D d, const T* __restrict__ gout, const T* __restrict__ x,
                                                     int rows_per_split, float* __restrict__ part,
                                                     float* __restrict__ bpart) {
  const int no_per_g = d.So * d.Ng;
  const int nred = d.S * d.Cg;
  const int64_t nw = int64_t(d.G) * no_per_g * d.K * nred;
  const int64_t nb = bpart ? int64_t(d.G) * no_per_g : 0;
  const int64_t total_rows = int64_t(d.B) * d.Tvalid;
  const int64_t r0 = int64_t(blockIdx.y) * rows_per_split;
  const int64_t r1 = r0 + rows_per_split < total_rows ? r0 + rows_per_split : total_rows;
  for (int64_t idx = int64_t(blockIdx.x) * 256 + threadIdx.x; idx < nw + nb; idx += int64_t(gridDim.x) * 256) {
    float acc = 0.f;
    if (idx < nw) {
      const int rc = int(idx % nred);
      const int i = int((idx / nred) % d.K);
      const int64_t go = idx / (int64_t(nred) * d.K);
      const int g = int(go / no_per_g), o = int(go - int64_t(g) * no_per_g);
      const int rph = rc / d.Cg, c = rc - rph * d.Cg;
      const int64_t oc = out_col(d, g, o), ic = in_col(d, g, rph, c);
      int b = int(r0 / d.Tvalid), j = int(r0 - int64_t(b) * d.Tvalid);  // one division, then a row walk
      for (int64_t rr = r0; rr < r1; ++rr) {
        const int t = j + d.q0 + i;
        if (t >= 0 && t < d.Tv)
          acc += to_f(gout[(int64_t(b) * d.Tvo + j) * d.ldo + oc]) * to_f(x[(int64_t(b) * d.Tvs + t) * d.ldx + ic]);
        if (++j == d.Tvalid) j = 0, ++b;
      }
      part[int64_t(blockIdx.y) * nw + idx] = acc;
    } else {
      const int64_t go = idx - nw;
      const int g = int(go / no_per_g), o = int(go - int64_t(g) * no_per_g);
      const int64_t oc = out_col(d, g, o);
      int b = int(r0 / d.Tvalid), j = int(r0 - int64_t(b) * d.Tvalid);
      for (int64_t rr = r0; rr < r1; ++rr) {
        acc += to_f(gout[(int64_t(b) * d.Tvo + j) * d.ldo + oc]);
        if (++j == d.Tvalid) j = 0, ++b;
      }
      bpart[int64_t(blockIdx.y) * nb + go] = acc;
    }
  }
}

// bf16 MFMA weight gradient (Cg % 8 == 0, group output width a multiple of 16).
// Block = (16*NT local outputs o, 32 reduction channels (r, c), tap group of
// <= WG_TAPS taps, split of 64-row tiles).  Both operands reduce over ROWS of the
// row-major LDS tiles and are read with ds_read_b64_tr_b16 (gfx950 transposing
// LDS read), v_mfma_f32_16x16x32_bf16.
constexpr int WG_BM = 64;
constexpr int WG_TAPS = 8;

__device__ __forceinline__ v4i16 tr_read(const __bf16* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4i16*)(p));
}
__device__ __forceinline__ bf16x8 tr_frag(const __bf16* p, int pitch) {
  const v4i16 lo = tr_read(p);
  const v4i16 hi = tr_read(p + 16 * pitch);
  const v8i16 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, v);
}

template <int NT>
__global__ __launch_bounds__(256) void k_dwgrad_mfma(D d, const __bf16* __restrict__ gout,
                                                     const __bf16* __restrict__ x, int tiles_per_seq,
                                                     int tiles_per_split, int ntg, float* __restrict__ part) {
  constexpr int BN = 16 * NT;
  constexpr int PG = BN + 16;  // (PG/2) dwords = 8 x odd: conflict-free transposing reads
  constexpr int PX = 32 + 16;
  constexpr int WPN = 4 / NT;  // waves per 16-wide output sub-tile
  constexpr int MAXJ = (WG_TAPS * 2 + WPN - 1) / WPN;
  extern __shared__ __align__(16) unsigned char smem[];
  __bf16* const gs = reinterpret_cast<__bf16*>(smem);
  __bf16* const xs = gs + WG_BM * PG;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nt = wave % NT, wsub = wave / NT;
  const int no_per_g = d.So * d.Ng;
  const int ntile_g = (no_per_g + BN - 1) / BN;
  const int g = blockIdx.x / ntile_g;
  const int o0 = (blockIdx.x % ntile_g) * BN;
  const int nred = d.S * d.Cg;
  const int cc = blockIdx.y * 32;
  const int tgi = blockIdx.z % ntg, split = blockIdx.z / ntg;
  const int k0 = tgi * WG_TAPS;
  const int kn = d.K - k0 < WG_TAPS ? d.K - k0 : WG_TAPS;
  const int span = WG_BM + kn - 1;
  const int64_t ntiles = int64_t(d.B) * tiles_per_seq;
  const int64_t tb = int64_t(split) * tiles_per_split;
  const int64_t te = tb + tiles_per_split < ntiles ? tb + tiles_per_split : ntiles;
  const int npairs = kn * 2;
  const int gq_ = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;

  floatx4 acc[MAXJ];
#pragma unroll
  for (int j = 0; j < MAXJ; ++j) acc[j] = floatx4{0.f, 0.f, 0.f, 0.f};

  // forward layers (So == 1): the 8 outputs of a vector are contiguous columns,
  // and the next tile's gout / x vectors are fetched into registers while this
  // tile's MFMAs run (same MFMAs in the same order as the synchronous loop below)
  const bool vec = d.So == 1 && (d.ldo & 7) == 0 && (d.Ng & 7) == 0;
  if (vec) {
    constexpr int GQ = (WG_BM * (BN / 8) + 255) / 256;
    constexpr int XQ = ((WG_BM + WG_TAPS - 1) * 4 + 255) / 256;
    uint4 gq[GQ], xq[XQ];
    bool gok[GQ], xok[XQ];
    auto load = [&](int64_t tile) {
      const int b = int(tile / tiles_per_seq);
      const int j0 = int(tile % tiles_per_seq) * WG_BM;
#pragma unroll
      for (int u = 0; u < GQ; ++u) {
        const int idx = tid + u * 256;
        const int rr = idx / (BN / 8), v = (idx % (BN / 8)) * 8;
        const int j = j0 + rr;
        gok[u] = idx < WG_BM * (BN / 8) && j < d.Tvalid && o0 + v < no_per_g;
        gq[u] = *reinterpret_cast<const uint4*>(gout + (int64_t(b) * d.Tvo + (gok[u] ? j : 0)) * d.ldo +
                                                out_col(d, g, gok[u] ? o0 + v : 0));
      }
#pragma unroll
      for (int u = 0; u < XQ; ++u) {
        const int idx = tid + u * 256;
        const int rr = idx >> 2, v = (idx & 3) * 8;
        const int t = j0 + d.q0 + k0 + rr;
        const int ch = cc + v;
        xok[u] = rr < span && t >= 0 && t < d.Tv && ch < nred;
        const int rph = (xok[u] ? ch : 0) / d.Cg, c = (xok[u] ? ch : 0) - rph * d.Cg;
        if ((u * 256) / 4 < span)
          xq[u] = *reinterpret_cast<const uint4*>(x + (int64_t(b) * d.Tvs + (xok[u] ? t : 0)) * d.ldx +
                                                  in_col(d, g, rph, c));
      }
    };
    if (tb < te) load(tb);
    for (int64_t tile = tb; tile < te; ++tile) {
      __syncthreads();
#pragma unroll
      for (int u = 0; u < GQ; ++u) {
        const int idx = tid + u * 256;
        if (idx >= WG_BM * (BN / 8)) continue;
        const int rr = idx / (BN / 8), v = (idx % (BN / 8)) * 8;
        *reinterpret_cast<uint4*>(gs + rr * PG + v) = gok[u] ? gq[u] : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < XQ; ++u) {
        const int idx = tid + u * 256;
        const int rr = idx >> 2, v = (idx & 3) * 8;
        if (rr >= span) continue;
        *reinterpret_cast<uint4*>(xs + rr * PX + v) = xok[u] ? xq[u] : make_uint4(0, 0, 0, 0);
      }
      __syncthreads();
      if (tile + 1 < te) load(tile + 1);
#pragma unroll
      for (int grp = 0; grp < WG_BM / 32; ++grp) {
        const bf16x8 A = tr_frag(gs + (grp * 32 + 4 * gq_ + q) * PG + nt * 16 + 4 * p, PG);
#pragma unroll
        for (int j = 0; j < MAXJ; ++j) {
          const int pr = wsub + WPN * j;
          if (pr >= npairs) break;
          const int k = pr >> 1, ct = pr & 1;
          const bf16x8 Bf = tr_frag(xs + (grp * 32 + 4 * gq_ + q + k) * PX + ct * 16 + 4 * p, PX);
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A, Bf, acc[j], 0, 0, 0);
        }
      }
    }
  }
  for (int64_t tile = vec ? te : tb; tile < te; ++tile) {
    const int b = int(tile / tiles_per_seq);
    const int j0 = int(tile % tiles_per_seq) * WG_BM;
    __syncthreads();
    for (int idx = tid; idx < WG_BM * (BN / 8); idx += 256) {
      const int rr = idx / (BN / 8), v = (idx % (BN / 8)) * 8;
      const int j = j0 + rr;
      __bf16 vals[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int o = o0 + v + e;
        vals[e] = (j < d.Tvalid && o < no_per_g) ? gout[(int64_t(b) * d.Tvo + j) * d.ldo + out_col(d, g, o)]
                                                 : __bf16(0.f);
      }
      *reinterpret_cast<uint4*>(gs + rr * PG + v) = *reinterpret_cast<uint4*>(vals);
    }
    for (int idx = tid; idx < span * 4; idx += 256) {
      const int rr = idx >> 2, v = (idx & 3) * 8;
      const int t = j0 + d.q0 + k0 + rr;
      const int ch = cc + v;
      uint4 val = make_uint4(0, 0, 0, 0);
      if (t >= 0 && t < d.Tv && ch < nred) {
        const int rph = ch / d.Cg, c = ch - rph * d.Cg;
        val = *reinterpret_cast<const uint4*>(x + (int64_t(b) * d.Tvs + t) * d.ldx + in_col(d, g, rph, c));
      }
      *reinterpret_cast<uint4*>(xs + rr * PX + v) = val;
    }
    __syncthreads();
#pragma unroll
    for (int grp = 0; grp < WG_BM / 32; ++grp) {
      const bf16x8 A = tr_frag(gs + (grp * 32 + 4 * gq_ + q) * PG + nt * 16 + 4 * p, PG);
#pragma unroll
      for (int j = 0; j < MAXJ; ++j) {
        const int pr = wsub + WPN * j;
        if (pr >= npairs) break;
        const int k = pr >> 1, ct = pr & 1;
        const bf16x8 Bf = tr_frag(xs + (grp * 32 + 4 * gq_ + q + k) * PX + ct * 16 + 4 * p, PX);
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A, Bf, acc[j], 0, 0, 0);
      }
    }
  }
  const int64_t nw = int64_t(d.G) * no_per_g * d.K * nred;
  float* pdst = part + int64_t(split) * nw;
#pragma unroll
  for (int j = 0; j < MAXJ; ++j) {
    const int pr = wsub + WPN * j;
    if (pr >= npairs) break;
    const int k = k0 + (pr >> 1), ct = pr & 1;
    const int ch = cc + ct * 16 + (lane & 15);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int o = o0 + nt * 16 + 4 * (lane >> 4) + e;
      if (o < no_per_g && ch < nred) pdst[((int64_t(g) * no_per_g + o) * d.K + k) * nred + ch] = acc[j][e];
    }
  }
}

// Weight gradient for one group with a contiguous reduction row and K <= 8
// taps (every MPD layer, the MSD's dense ones): the generator's k_wgrad3_bf16
// scheme on the dconv descriptor.  A block owns 32*NT output x 32*CT reduction
// channels x ALL taps over a contiguous range of 128-row tiles of one
// sequence: gout and x are read once per block (the 16-wide per-tap-group
// kernel above re-read them (N/32)*(nred/32) times, ~5% of the bf16 peak),
// double-buffered in LDS with a register prefetch of the next tile, operands
// through transposing reads, 32x32x16 MFMA.
constexpr int W3_BM = 128, W3_HALO = 64;

// bpart != nullptr: the bias partials of the same split too (per output column,
// summed from the staged gout tiles by the first reduction-channel block of
// each column block: gap rows are staged as zeros), replacing a separate pass
// over gout (k_dbias_part_v) per layer.
template <int NT, int CT, int MAXT>
__global__ __launch_bounds__(256) void k_dwgrad_w3(D d, const __bf16* __restrict__ gout, const __bf16* __restrict__ x,
                                                   int tiles_per_seq, int64_t n_tiles, int tiles_per_split,
                                                   float* __restrict__ part, int flat_p, float* __restrict__ bpart) {
  constexpr int NB = 32 * NT, CB = 32 * CT;
  constexpr int XROWS = W3_BM + W3_HALO;
  constexpr int GV = W3_BM * NB / 8 / 256;
  constexpr int XV = XROWS * CB / 8 / 256;
  constexpr int GS = NT * W3_BM * 32, XS = CT * XROWS * 32;
  constexpr int WPN = 4 / NT;
  extern __shared__ __align__(16) unsigned char smem[];
  __bf16* const base = reinterpret_cast<__bf16*>(smem);  // [buf]{G[NT][128][32], X[CT][192][32]}

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t split = blockIdx.x;
  const int n0 = blockIdx.y * NB, c0 = blockIdx.z * CB;
  const int nred = d.S * d.Cg;
  const int64_t tb = split * tiles_per_split;
  const int64_t te = tb + tiles_per_split < n_tiles ? tb + tiles_per_split : n_tiles;
  const int span = W3_BM + d.K - 1;
  const int P = CT * d.K;
  const int RG = P >= WPN ? 1 : WPN / P;
  const int WPP = WPN / RG;
  const int nt = wave / WPN, wsub = wave % WPN;
  const int rg = wsub / WPP, pw = wsub % WPP;
  const int RROWS = W3_BM / RG;

  uint4 gr[GV], xr[XV];
  bool gok[GV], xok[XV];
  // branch-free buffer loads (sel_common.h ru_bload): invalid rows and a dead
  // request (live = false) read nothing, so the request is counted exactly and
  // the MFMA phase does not wait on it
  auto load = [&](int64_t tile, bool live) {
    // flat_p > 0: one row space over all sequences (pitch flat_p, zero gaps; see
    // conv.hip dconv_ws_fwd), rows valid by their position in their sequence
    const int b = int(tile / tiles_per_seq);
    const int j0 = int(tile % tiles_per_seq) * W3_BM;
    const int nflat = flat_p * d.B;
    const __amdgpu_buffer_rsrc_t rg = ru_rsrc(gout + int64_t(b) * d.Tvo * d.ldo, int64_t(d.B - b) * d.Tvo * d.ldo);
    const __amdgpu_buffer_rsrc_t rx = ru_rsrc(x + int64_t(b) * d.Tvs * d.ldx, int64_t(d.B - b) * d.Tvs * d.ldx);
#pragma unroll
    for (int u = 0; u < GV; ++u) {
      const int v = tid + u * 256;
      const int j = j0 + v / (NB / 8);
      gok[u] = flat_p ? j < nflat && j % flat_p < d.Tvalid : j < d.Tvalid;
      gr[u] = ru_bload(rg, live && gok[u] ? (j * d.ldo + n0 + (v % (NB / 8)) * 8) * 2 : RU_OOB);
    }
#pragma unroll
    for (int u = 0; u < XV; ++u) {
      const int v = tid + u * 256;
      const int r = v / (CB / 8);
      const int t = j0 + d.q0 + r;
      xok[u] = r < span && t >= 0 && (flat_p ? t < nflat && t % flat_p < d.Tv : t < d.Tv);
      xr[u] = ru_bload(rx, live && xok[u] ? (t * d.ldx + c0 + (v % (CB / 8)) * 8) * 2 : RU_OOB);
    }
  };
  auto store = [&](int buf) {
    __bf16* g = base + buf * (GS + XS);
    __bf16* xx = g + GS;
#pragma unroll
    for (int u = 0; u < GV; ++u) {
      const int v = tid + u * 256;
      const int r = v / (NB / 8), c8 = v % (NB / 8);
      *reinterpret_cast<uint4*>(g + (c8 >> 2) * (W3_BM * 32) + r * 32 + (c8 & 3) * 8) =
          gok[u] ? gr[u] : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < XV; ++u) {
      if (u * 256 / (CB / 8) >= span) continue;
      const int v = tid + u * 256;
      const int r = v / (CB / 8), c8 = v % (CB / 8);
      *reinterpret_cast<uint4*>(xx + (c8 >> 2) * (XROWS * 32) + r * 32 + (c8 & 3) * 8) =
          xok[u] ? xr[u] : make_uint4(0, 0, 0, 0);
    }
  };

  int xoff[MAXT];
#pragma unroll
  for (int j = 0; j < MAXT; ++j) {
    int p = pw + WPP * j;
    p = p < P ? p : P - 1;
    xoff[j] = (p / d.K) * (XROWS * 32) + (p % d.K) * 32;
  }
  floatx16 acc[MAXT];
#pragma unroll
  for (int j = 0; j < MAXT; ++j)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[j][e] = 0.f;

  const int h = lane >> 5;
  const int col = ((lane >> 4) & 1) * 16 + 4 * (lane & 3);
  const int q = (lane & 15) >> 2;
  const int lrow = (4 * h + q) * 32 + col;

  const bool bias_on = bpart != nullptr && blockIdx.z == 0;  // block-uniform
  const int bn = tid % NB;
  float bsum = 0.f;
  if (tb < te) load(tb, true);
  int buf = 0;
  for (int64_t tile = tb; tile < te; ++tile, buf ^= 1) {
    store(buf);
    __syncthreads();
    load(tile + 1 < te ? tile + 1 : tile, tile + 1 < te);  // unconditional: exact counts
    if (bias_on) {
      const __bf16* gb = base + buf * (GS + XS) + (bn >> 5) * (W3_BM * 32) + (bn & 31);
      for (int r = tid / NB; r < W3_BM; r += 256 / NB) bsum += float(gb[r * 32]);
    }
    const __bf16* g = base + buf * (GS + XS) + nt * (W3_BM * 32);
    const __bf16* xx = base + buf * (GS + XS) + GS;
    for (int kh = 0; kh < RROWS / 16; ++kh) {
      const int R = (rg * RROWS + kh * 16) * 32 + lrow;
      const v4i16 a0 = tr_read(g + R);
      const v4i16 a1 = tr_read(g + R + 8 * 32);
      const bf16x8 A = __builtin_bit_cast(bf16x8, __builtin_shufflevector(a0, a1, 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
      for (int j = 0; j < MAXT; ++j) {
        const v4i16 b0 = tr_read(xx + xoff[j] + R);
        const v4i16 b1 = tr_read(xx + xoff[j] + R + 8 * 32);
        const bf16x8 Bf = __builtin_bit_cast(bf16x8, __builtin_shufflevector(b0, b1, 0, 1, 2, 3, 4, 5, 6, 7));
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A, Bf, acc[j], 0, 0, 0);
      }
    }
  }

  const int64_t nw = int64_t(d.Ng) * d.K * nred;
  float* pdst = part + split * nw;
  if (RG == 1) {
#pragma unroll
    for (int j = 0; j < MAXT; ++j) {
      const int p = pw + WPP * j;
      if (p >= P) break;
      const int ct = p / d.K, k = p % d.K;
      const int c = c0 + ct * 32 + (lane & 31);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int n = n0 + nt * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        pdst[(int64_t(n) * d.K + k) * nred + c] = acc[j][r];
      }
    }
  } else {
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem);  // [wave][32*32]
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      red[wave * 1024 + row * 32 + (lane & 31)] = acc[0][r];
    }
    __syncthreads();
    for (int i = tid; i < NT * P * 1024; i += 256) {
      const int e = i & 1023, pi = (i >> 10) % P, ni = (i >> 10) / P;
      float v = 0.f;
      for (int r = 0; r < RG; ++r) v += red[(ni * WPN + r * WPP + pi) * 1024 + e];
      const int ct = pi / d.K, k = pi % d.K;
      const int n = n0 + ni * 32 + (e >> 5), c = c0 + ct * 32 + (e & 31);
      pdst[(int64_t(n) * d.K + k) * nred + c] = v;
    }
  }
  if (bias_on) {  // the 256 / NB row lanes of each column, added in lane order
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem);
    red[tid] = bsum;
    __syncthreads();
    if (tid < NB) {
      float v = 0.f;
      for (int q = 0; q < 256 / NB; ++q) v += red[q * NB + tid];
      bpart[split * d.Ng + n0 + tid] = v;
    }
  }
}

// bias partials for the MFMA wgrad path: gb[col] over a split of rows.  Block =
// 64 output columns x 4 row lanes (a row's 64 columns are one coalesced read),
// row walk without divisions, the 4 lanes summed in LDS.
template <typename T>
__global__ __launch_bounds__(256) void k_dbias_part(D d, const T* __restrict__ gout, int rows_per_split,
                                                    float* __restrict__ bpart) {
  __shared__ float red[4][64];
  const int no_per_g = d.So * d.Ng;
  const int64_t nb = int64_t(d.G) * no_per_g;
  const int64_t total_rows = int64_t(d.B) * d.Tvalid;
  const int64_t r0 = int64_t(blockIdx.y) * rows_per_split;
  const int64_t r1 = r0 + rows_per_split < total_rows ? r0 + rows_per_split : total_rows;
  const int cl = threadIdx.x & 63, ly = threadIdx.x >> 6;
  const int64_t go = int64_t(blockIdx.x) * 64 + cl;
  float acc = 0.f;
  if (go < nb) {
    const int g = int(go / no_per_g), o = int(go - int64_t(g) * no_per_g);
    const int64_t oc = out_col(d, g, o);
    int64_t rr = r0 + ly;
    int b = int(rr / d.Tvalid), j = int(rr - int64_t(b) * d.Tvalid);
    for (; rr < r1; rr += 4) {
      acc += to_f(gout[(int64_t(b) * d.Tvo + j) * d.ldo + oc]);
      j += 4;
      while (j >= d.Tvalid) j -= d.Tvalid, ++b;
    }
  }
  red[ly][cl] = acc;
  __syncthreads();
  if (ly == 0 && go < nb) bpart[int64_t(blockIdx.y) * nb + go] = (red[0][cl] + red[1][cl]) + (red[2][cl] + red[3][cl]);
}

// Vector form (bf16, So == 1, 8-aligned contiguous columns): a thread sums 8
// consecutive columns with 16-B loads over every 32nd row of the split, the 32
// row lanes are added in order through LDS (the scalar kernel above issued one
// 2-byte load per lane and row: ~1 TB/s).
__global__ __launch_bounds__(256) void k_dbias_part_v(D d, const __bf16* __restrict__ gout, int rows_per_split,
                                                      float* __restrict__ bpart) {
  __shared__ float red[32][65];
  const int64_t nb = int64_t(d.G) * d.Ng;
  const int64_t total_rows = int64_t(d.B) * d.Tvalid;
  const int64_t r0 = int64_t(blockIdx.y) * rows_per_split;
  const int64_t r1 = r0 + rows_per_split < total_rows ? r0 + rows_per_split : total_rows;
  const int cg = threadIdx.x & 7, ly = threadIdx.x >> 3;
  const int64_t c0 = int64_t(blockIdx.x) * 64 + cg * 8;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c0 < nb) {
    int64_t rr = r0 + ly;
    int b = int(rr / d.Tvalid), j = int(rr - int64_t(b) * d.Tvalid);
    for (; rr < r1; rr += 32) {
      const uint4 raw = *reinterpret_cast<const uint4*>(gout + (int64_t(b) * d.Tvo + j) * d.ldo + c0);
      const __bf16* v = reinterpret_cast<const __bf16*>(&raw);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += float(v[e]);
      j += 32;
      while (j >= d.Tvalid) j -= d.Tvalid, ++b;
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) red[ly][cg * 8 + e] = acc[e];
  __syncthreads();
  const int64_t go = int64_t(blockIdx.x) * 64 + threadIdx.x;
  if (threadIdx.x < 64 && go < nb) {
    float t = 0.f;
    for (int l = 0; l < 32; ++l) t += red[l][threadIdx.x];
    bpart[int64_t(blockIdx.y) * nb + go] = t;
  }
}

// bias partials of a forward layer's gout: the vector kernel where it applies
// (tune key 25 = 1: the scalar one)
void launch_dbias_part(const sel_dconv_desc* d, const __bf16* gout, int rows_per_split, int bsplit, float* bpart,
                       hipStream_t s) {
  const int64_t nb = int64_t(d->G) * d->So * d->Ng;
  dim3 bg(unsigned((nb + 63) / 64), unsigned(bsplit));
  if (d->So == 1 && nb % 8 == 0 && d->ldo % 8 == 0 && tune(25) != 1)
    hipLaunchKernelGGL(k_dbias_part_v, bg, dim3(256), 0, s, *d, gout, rows_per_split, bpart);
  else
    hipLaunchKernelGGL(k_dbias_part<__bf16>, bg, dim3(256), 0, s, *d, gout, rows_per_split, bpart);
}

// Partial sums over groups of PRESUM splits (coalesced over the weights), so the
// final per-output reduction reads at most PRESUM partials.
constexpr int PRESUM = 16;
__global__ __launch_bounds__(256) void k_presum(const float* __restrict__ part, int nsplit, int64_t n,
                                                float* __restrict__ out) {
  const int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x;
  if (i >= n) return;
  const int s0 = blockIdx.y * PRESUM, s1 = s0 + PRESUM < nsplit ? s0 + PRESUM : nsplit;
  float acc = 0.f;
  int sp = s0;
  for (; sp + 4 <= s1; sp += 4) {
    const float a0 = part[int64_t(sp) * n + i], a1 = part[int64_t(sp + 1) * n + i], a2 = part[int64_t(sp + 2) * n + i],
                a3 = part[int64_t(sp + 3) * n + i];
    acc += (a0 + a1) + (a2 + a3);
  }
  for (; sp < s1; ++sp) acc += part[int64_t(sp) * n + i];
  out[int64_t(blockIdx.y) * n + i] = acc;
}

// Weight gradient of the short-reduction layers (K * S * Cg = KR in {2, 3, 6, 15},
// one group, one output phase): block = a row range; thread = one output channel
// n x one row lane, KR + 1 accumulators (weights and bias) over its rows; the row
// lanes summed in LDS; one partial per block.
template <typename T, int KR>
__global__ __launch_bounds__(256) void k_dwgrad_short(D d, const T* __restrict__ gout, const T* __restrict__ x,
                                                      int rows_per_split, float* __restrict__ part,
                                                      float* __restrict__ bpart) {
  __shared__ float red[256 * (KR + 1) <= 4096 ? 256 * (KR + 1) : 4096];
  const int N = d.Ng;
  const int nl = N < 256 ? N : 256;  // lanes over n (N <= 256 here)
  const int RL = 256 / nl;
  const int n = threadIdx.x % nl, rl = threadIdx.x / nl;
  const int nred = d.S * d.Cg;
  const int64_t total_rows = int64_t(d.B) * d.Tvalid;
  const int64_t r0 = int64_t(blockIdx.x) * rows_per_split;
  const int64_t r1 = r0 + rows_per_split < total_rows ? r0 + rows_per_split : total_rows;
  float acc[KR + 1];
#pragma unroll
  for (int e = 0; e <= KR; ++e) acc[e] = 0.f;
  int tap[KR], col[KR];  // hoisted as in k_dconv_short
#pragma unroll
  for (int e = 0; e < KR; ++e) {
    const int i = e / nred, rc = e - i * nred;
    const int r = rc / d.Cg, c = rc - r * d.Cg;
    tap[e] = d.q0 + i;
    col[e] = int(in_col(d, 0, r, c));
  }
  int64_t rr = r0 + rl;
  if (rr < r1 && threadIdx.x < nl * RL) {
    int b = int(rr / d.Tvalid), j = int(rr - int64_t(b) * d.Tvalid);
    for (; rr < r1; rr += RL) {
      const float gv = to_f(gout[(int64_t(b) * d.Tvo + j) * d.ldo + n]);
      const T* xb = x + int64_t(b) * d.Tvs * d.ldx;
#pragma unroll
      for (int e = 0; e < KR; ++e) {
        const int t = j + tap[e];
        if (t >= 0 && t < d.Tv) acc[e] = fmaf(gv, to_f(xb[int64_t(t) * d.ldx + col[e]]), acc[e]);
      }
      acc[KR] += gv;
      j += RL;
      while (j >= d.Tvalid) j -= d.Tvalid, ++b;
    }
  }
  // reduce the RL row lanes: red[rl][n][e]
#pragma unroll
  for (int e = 0; e <= KR; ++e) {
    if (threadIdx.x < nl * RL) red[(rl * nl + n) * (KR + 1) + e] = acc[e];
  }
  __syncthreads();
  for (int o = threadIdx.x; o < nl * (KR + 1); o += 256) {
    float sum = 0.f;
    for (int l = 0; l < RL; ++l) sum += red[l * nl * (KR + 1) + o];
    const int nn = o / (KR + 1), e = o - nn * (KR + 1);
    if (e < KR) part[int64_t(blockIdx.x) * N * KR + int64_t(nn) * KR + e] = sum;
    else if (bpart) bpart[int64_t(blockIdx.x) * N + nn] = sum;
  }
}

// Staged weight gradient of the same layers (contiguous phase view, see
// k_dconv_shortx): a thread owns 2 output channels (one 4-B gout load per row)
// and 16 consecutive rows of each tile, whose x windows come from the tile staged
// in LDS, 4 rows per register window; blocks accumulate over their tiles and
// reduce their row lanes into one partial.  k_dwgrad_short's per-row global x
// loads ran the MSD's k15 1 -> 128 layer at 2.6 ms for 393 MB of gout.
template <typename T, int K, int NR>
__global__ __launch_bounds__(256) void k_dwgrad_shortx(D d, const T* __restrict__ gout, const T* __restrict__ x,
                                                       float* __restrict__ part, float* __restrict__ bpart) {
  constexpr int KR = K * NR, RR = 16, XW = (4 + K - 1) * NR;
  extern __shared__ float sh[];  // x window [(RB + K - 1) * NR], then the row-lane reduction [RL][Ng][KR + 1]
  const int N = d.Ng, NL = N / 2, RL = 256 / NL, RB = RL * RR;
  const int rl = threadIdx.x / NL, n = (threadIdx.x - rl * NL) * 2;
  float a0[KR + 1], a1[KR + 1];
#pragma unroll
  for (int e = 0; e <= KR; ++e) a0[e] = a1[e] = 0.f;
  const int tps = (d.Tvalid + RB - 1) / RB, ntiles = d.B * tps;
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int b = tile / tps, j0 = (tile - b * tps) * RB;
    __syncthreads();
    for (int p = threadIdx.x; p < (RB + K - 1) * NR; p += 256) {
      const int t = j0 + d.q0 + p / NR;
      sh[p] = (t >= 0 && t < d.Tv) ? to_f(x[(int64_t(b) * d.Tvs + t) * NR + p % NR]) : 0.f;
    }
    __syncthreads();
    const T* grow = gout + int64_t(b) * d.Tvo * d.ldo + n;
#pragma unroll 1
    for (int q4 = 0; q4 < RR; q4 += 4) {
      const int jl = rl * RR + q4;
      if (j0 + jl >= d.Tvalid) break;
      float gx[4], gy[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int j = j0 + jl + r;
        gx[r] = gy[r] = 0.f;
        if (j < d.Tvalid) {
          const T* gp = grow + int64_t(j) * d.ldo;
          gx[r] = to_f(gp[0]);
          gy[r] = to_f(gp[1]);
        }
      }
      float xw[XW];
#pragma unroll
      for (int u = 0; u < XW; ++u) xw[u] = sh[jl * NR + u];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
#pragma unroll
        for (int e = 0; e < KR; ++e) {
          a0[e] = fmaf(gx[r], xw[r * NR + e], a0[e]);
          a1[e] = fmaf(gy[r], xw[r * NR + e], a1[e]);
        }
        a0[KR] += gx[r];
        a1[KR] += gy[r];
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int e = 0; e <= KR; ++e) {
    sh[(rl * N + n) * (KR + 1) + e] = a0[e];
    sh[(rl * N + n + 1) * (KR + 1) + e] = a1[e];
  }
  __syncthreads();
  for (int o = threadIdx.x; o < N * (KR + 1); o += 256) {
    float sum = 0.f;
    for (int l = 0; l < RL; ++l) sum += sh[l * N * (KR + 1) + o];
    const int nn = o / (KR + 1), e = o - nn * (KR + 1);
    if (e < KR) part[int64_t(blockIdx.x) * N * KR + int64_t(nn) * KR + e] = sum;
    else if (bpart) bpart[int64_t(blockIdx.x) * N + nn] = sum;
  }
}

// ---------------------------------------------------------------------------
// Weight packing (torch Conv1d / (k,1) Conv2d weight [N][Cg][Kt], optional
// weight norm w = g * v / ||v||) into the phase-view forms:
//   fwd  Wp[g][n][i][r][c] = w[g*Ng + n][c][s*(q0 + i) + r + pad]   (0 if out of [0, Kt))
//   dgrad Wd[g][(r,c)][i'][n] = Wp[g][n][K-1-i'][r][c]
// ---------------------------------------------------------------------------
struct PackGeo {
  int N, Cg, Kt, s, pad, G, K, q0;
};

__host__ __device__ inline PackGeo pack_geo(int N, int Cg, int Kt, int s, int pad, int G) {
  PackGeo p{N, Cg, Kt, s, pad, G, 0, 0};
  // q0 = floor(-pad / s), K = floor((Kt - 1 - pad) / s) - q0 + 1
  const int a = -pad;
  p.q0 = a >= 0 ? a / s : -((-a + s - 1) / s);
  const int e = Kt - 1 - pad;
  const int qe = e >= 0 ? e / s : -((-e + s - 1) / s);
  p.K = qe - p.q0 + 1;
  return p;
}

// one block per output channel n: ||v_n|| then the packed weights
template <typename T>
__device__ __forceinline__ void dpack_channel(const PackGeo& pg, int mode, const float* __restrict__ w,
                                              const float* __restrict__ wg, T* __restrict__ out, int n);

template <typename T>
__global__ __launch_bounds__(256) void k_dpack(PackGeo pg, int mode, const float* __restrict__ w,
                                               const float* __restrict__ wg, T* __restrict__ out) {
  dpack_channel<T>(pg, mode, w, wg, out, blockIdx.x);
}

// batched form: block ranges per job in the kernel argument
constexpr int DPM_MAXJ = 24;
struct DPackJobs {
  PackGeo pg[DPM_MAXJ];
  const float* w[DPM_MAXJ];
  const float* wg[DPM_MAXJ];
  void* out[DPM_MAXJ];
  int mode[DPM_MAXJ];
  int bstart[DPM_MAXJ + 1];
  int njobs;
};

template <typename T>
__global__ __launch_bounds__(256) void k_dpack_many(DPackJobs dj) {
  int j = 0;
  while (j + 1 < dj.njobs && int(blockIdx.x) >= dj.bstart[j + 1]) ++j;  // block-uniform
  dpack_channel<T>(dj.pg[j], dj.mode[j], dj.w[j], dj.wg[j], static_cast<T*>(dj.out[j]),
                   int(blockIdx.x) - dj.bstart[j]);
}

// mode-2 jobs: the adjoint form as a tiled transpose of the forward form just
// packed (Wp[g][nl][i][rc] -> Wd[g][rc][K-1-i][nl]): pure data movement, so the
// adjoint holds exactly the forward form's values, with coalesced reads and
// writes (the per-channel adjoint pack writes every element Ng apart).
// Block = (job, group, 64 output channels, 64 (tap, reduction) columns).
struct DPackTrJobs {
  PackGeo pg[DPM_MAXJ];
  const void* src[DPM_MAXJ];
  void* out[DPM_MAXJ];
  int ntn[DPM_MAXJ], ntc[DPM_MAXJ];  // channel / column tiles per group
  int bstart[DPM_MAXJ + 1];
  int njobs;
};

template <typename T>
__global__ __launch_bounds__(256) void k_dpack_tr_many(DPackTrJobs dj) {
  __shared__ T tile[64][65];
  int j = 0;
  while (j + 1 < dj.njobs && int(blockIdx.x) >= dj.bstart[j + 1]) ++j;  // block-uniform
  const PackGeo& pg = dj.pg[j];
  const T* __restrict__ src = static_cast<const T*>(dj.src[j]);
  T* __restrict__ out = static_cast<T*>(dj.out[j]);
  const int lb = int(blockIdx.x) - dj.bstart[j];
  const int ct = lb % dj.ntc[j], nt = (lb / dj.ntc[j]) % dj.ntn[j], g = lb / (dj.ntc[j] * dj.ntn[j]);
  const int Ng = pg.N / pg.G, nred = pg.s * pg.Cg, cols = pg.K * nred;
  const int nl0 = nt * 64, c0 = ct * 64;
  const int t = threadIdx.x, lo = t & 63, hi = t >> 6;
#pragma unroll 4
  for (int r = hi; r < 64; r += 4) {  // rows = output channels, columns = (i, rc) contiguous
    const int nl = nl0 + r, c = c0 + lo;
    if (nl < Ng && c < cols) tile[r][lo] = src[(int64_t(g) * Ng + nl) * cols + c];
  }
  __syncthreads();
#pragma unroll 4
  for (int q = hi; q < 64; q += 4) {  // column q of the tile -> one Wd row, channels contiguous
    const int c = c0 + q, nl = nl0 + lo;
    if (nl < Ng && c < cols) {
      const int i = c / nred, rc = c - i * nred;
      out[((int64_t(g) * nred + rc) * pg.K + (pg.K - 1 - i)) * Ng + nl] = tile[lo][q];
    }
  }
}

template <typename T>
__device__ __forceinline__ void dpack_channel(const PackGeo& pg, int mode, const float* __restrict__ w,
                                              const float* __restrict__ wg, T* __restrict__ out, int n) {
  __shared__ float red[16];
  const int per = pg.Cg * pg.Kt;
  float scale = 1.f;
  if (wg) {
    float ss = 0.f;
    for (int e = threadIdx.x; e < per; e += 256) {
      const float v = w[int64_t(n) * per + e];
      ss += v * v;
    }
    ss = block_sum(ss, red);
    if (threadIdx.x == 0) red[0] = ss;
    __syncthreads();
    scale = wg[n] / sqrtf(red[0]);
  }
  const int Ng = pg.N / pg.G, g = n / Ng, nl = n - g * Ng;
  const int nred = pg.s * pg.Cg;
  for (int e = threadIdx.x; e < pg.K * nred; e += 256) {
    const int i = e / nred, rc = e - i * nred;
    const int r = rc / pg.Cg, c = rc - r * pg.Cg;
    const int k = pg.s * (pg.q0 + i) + r + pg.pad;
    const float v = (k >= 0 && k < pg.Kt) ? w[(int64_t(n) * pg.Cg + c) * pg.Kt + k] * scale : 0.f;
    if (mode == 0) {
      out[((int64_t(g) * Ng + nl) * pg.K + i) * nred + rc] = from_f<T>(v);
    } else {  // dgrad: [g][(r,c)][K-1-i][n]
      out[((int64_t(g) * nred + rc) * pg.K + (pg.K - 1 - i)) * Ng + nl] = from_f<T>(v);
    }
  }
}

// Final wgrad reduction: sum the split partials, unpack to the torch layout,
// and (weight norm) gv = (g/||v||) (gw - w_hat (w_hat . gw)), gg = w_hat . gw.
// One block per output channel n; the partials are walked in their packed
// (tap, phase, channel) order, so each split's slice is one coalesced read, and
// scattered once into the torch (channel, tap) positions.
__device__ __forceinline__ void dwgrad_finish_channel(const PackGeo& pg, const float* __restrict__ part, int nsplit,
                                                      const float* __restrict__ bpart, int bsplit,
                                                      const float* __restrict__ v, const float* __restrict__ wg,
                                                      float* __restrict__ gw, float* __restrict__ gg,
                                                      float* __restrict__ gb, int n);

__global__ __launch_bounds__(256) void k_dwgrad_finish(PackGeo pg, const float* __restrict__ part, int nsplit,
                                                       const float* __restrict__ bpart, int bsplit,
                                                       const float* __restrict__ v, const float* __restrict__ wg,
                                                       float* __restrict__ gw, float* __restrict__ gg,
                                                       float* __restrict__ gb) {
  dwgrad_finish_channel(pg, part, nsplit, bpart, bsplit, v, wg, gw, gg, gb, blockIdx.x);
}

// batched form (sel_dconv_wgrad_finish_many): the final reductions of several
// layers in one launch, block ranges per job in the kernel argument (a
// sub-discriminator's layers finish together after its chain backward instead
// of one launch per layer)
constexpr int DWF_MAXJ = 24;
struct DwgradJobs {
  PackGeo pg[DWF_MAXJ];
  const float* part[DWF_MAXJ];
  const float* bpart[DWF_MAXJ];
  const float* v[DWF_MAXJ];
  const float* wg[DWF_MAXJ];
  float* gw[DWF_MAXJ];
  float* gg[DWF_MAXJ];
  float* gb[DWF_MAXJ];
  int nsplit[DWF_MAXJ], bsplit[DWF_MAXJ];
  int bstart[DWF_MAXJ + 1];
  int njobs;
};

__global__ __launch_bounds__(256) void k_dwgrad_finish_many(DwgradJobs dj) {
  int j = 0;
  while (j + 1 < dj.njobs && int(blockIdx.x) >= dj.bstart[j + 1]) ++j;  // block-uniform
  dwgrad_finish_channel(dj.pg[j], dj.part[j], dj.nsplit[j], dj.bpart[j], dj.bsplit[j], dj.v[j], dj.wg[j], dj.gw[j],
                        dj.gg[j], dj.gb[j], int(blockIdx.x) - dj.bstart[j]);
}

__device__ __forceinline__ void dwgrad_finish_channel(const PackGeo& pg, const float* __restrict__ part, int nsplit,
                                                      const float* __restrict__ bpart, int bsplit,
                                                      const float* __restrict__ v, const float* __restrict__ wg,
                                                      float* __restrict__ gw, float* __restrict__ gg,
                                                      float* __restrict__ gb, int n) {
  __shared__ float red[16];
  __shared__ float bc[2];
  const int per = pg.Cg * pg.Kt;
  const int Ng = pg.N / pg.G, g = n / Ng, nl = n - g * Ng;
  const int nred = pg.s * pg.Cg;
  const int64_t nw = int64_t(pg.N) * pg.K * nred;
  const int64_t base = (int64_t(g) * Ng + nl) * pg.K * nred;
  float dot = 0.f, vv = 0.f;
  for (int e = threadIdx.x; e < pg.K * nred; e += 256) {
    const int i = e / nred, rc = e - i * nred;
    const int r = rc / pg.Cg, c = rc - r * pg.Cg;
    const int k = pg.s * (pg.q0 + i) + r + pg.pad;
    if (k < 0 || k >= pg.Kt) continue;  // structural zero of the phase view
    float acc = 0.f;
    int sp = 0;
    for (; sp + 4 <= nsplit; sp += 4) {  // 4 loads in flight, fixed order
      const float a0 = part[int64_t(sp) * nw + base + e], a1 = part[int64_t(sp + 1) * nw + base + e],
                  a2 = part[int64_t(sp + 2) * nw + base + e], a3 = part[int64_t(sp + 3) * nw + base + e];
      acc += (a0 + a1) + (a2 + a3);
    }
    for (; sp < nsplit; ++sp) acc += part[int64_t(sp) * nw + base + e];
    const int64_t o = int64_t(n) * per + c * pg.Kt + k;
    gw[o] = acc;
    if (v) {
      const float vv_ = v[o];
      dot += vv_ * acc;
      vv += vv_ * vv_;
    }
  }
  if (gb) {  // the bias partials of this n, spread over the block (fixed order per thread)
    float acc = 0.f;
    for (int sp = threadIdx.x; sp < bsplit; sp += 256) acc += bpart[int64_t(sp) * pg.N + n];
    acc = block_sum(acc, red);
    if (threadIdx.x == 0) gb[n] = acc;
  }
  if (!v) return;
  dot = block_sum(dot, red);
  if (threadIdx.x == 0) bc[0] = dot;
  vv = block_sum(vv, red);
  if (threadIdx.x == 0) bc[1] = vv;
  __syncthreads();
  const float nv = sqrtf(bc[1]);
  const float gn = wg[n];
  // w = gn * v / nv ; dL/dgn = (v . gw) / nv ; dL/dv = gn/nv * (gw - v (v . gw) / nv^2)
  if (threadIdx.x == 0) gg[n] = bc[0] / nv;
  const float a = gn / nv, bcoef = gn * bc[0] / (nv * nv * nv);
  __syncthreads();  // every gw[o] of this n written before the in-place update
  for (int e = threadIdx.x; e < per; e += 256) {
    const int64_t o = int64_t(n) * per + e;
    gw[o] = a * gw[o] - bcoef * v[o];
  }
}

// ---------------------------------------------------------------------------
// Data movement of the discriminator front-ends
// ---------------------------------------------------------------------------
// AvgPool1d(kernel 4, stride 2, padding 2, count_include_pad) between MSD scales
// (discriminator.py:428-447): (B, T) fp32 -> (B, Tout_alloc) with zeros past To.
__global__ void k_avgpool_fwd(const float* __restrict__ x, int B, int T, int ldx, int kw, int st, int pad,
                              int To, int ldo, float* __restrict__ y) {
  const int64_t total = int64_t(B) * ldo;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < total; i += int64_t(gridDim.x) * blockDim.x) {
    const int b = int(i / ldo), t = int(i - int64_t(b) * ldo);
    float v = 0.f;
    if (t < To) {
      for (int k = 0; k < kw; ++k) {
        const int u = t * st + k - pad;
        if (u >= 0 && u < T) v += x[int64_t(b) * ldx + u];
      }
      v /= float(kw);
    }
    y[i] = v;
  }
}

__global__ void k_avgpool_bwd(const float* __restrict__ gy, int B, int T, int ldx, int kw, int st, int pad, int To,
                              int ldo, float* __restrict__ gx) {
  const int64_t total = int64_t(B) * ldx;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < total; i += int64_t(gridDim.x) * blockDim.x) {
    const int b = int(i / ldx), u = int(i - int64_t(b) * ldx);
    float v = 0.f;
    if (u < T) {
      // outputs t with t*st + k - pad == u, 0 <= k < kw
      const int lo = (u + pad - kw + 1 + st - 1) / st > 0 ? (u + pad - kw + 1 + st - 1) / st : 0;
      for (int t = lo; t * st - pad <= u && t < To; ++t) v += gy[int64_t(b) * ldo + t];
      v /= float(kw);
    }
    gx[i] = v;
  }
}

// MPD front-end (discriminator.py:120-126): reflect-pad T to a multiple of the
// period p, view (B, 1, T/p, p) -> our (B*p, L_alloc) sequences (column-major
// over the p columns), rows past L zero.  Backward folds the reflect pad.
__global__ void k_mpd_fold(const float* __restrict__ x, int B, int T, int ldx, int p, int L, int Lalloc,
                           float* __restrict__ y) {
  const int64_t total = int64_t(B) * p * Lalloc;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < total; i += int64_t(gridDim.x) * blockDim.x) {
    const int64_t seq = i / Lalloc;
    const int l = int(i - seq * Lalloc);
    const int b = int(seq / p), col = int(seq - int64_t(b) * p);
    float v = 0.f;
    if (l < L) {
      int u = l * p + col;
      if (u >= T) u = 2 * (T - 1) - u;  // reflect (F.pad mode "reflect")
      v = x[int64_t(b) * ldx + u];
    }
    y[i] = v;
  }
}

__global__ void k_mpd_unfold(const float* __restrict__ gy, int B, int T, int ldx, int p, int L, int Lalloc,
                             float* __restrict__ gx) {
  const int64_t total = int64_t(B) * ldx;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < total; i += int64_t(gridDim.x) * blockDim.x) {
    const int b = int(i / ldx), u = int(i - int64_t(b) * ldx);
    float v = 0.f;
    if (u < T) {
      v = gy[(int64_t(b) * p + u % p) * Lalloc + u / p];
      const int up = 2 * (T - 1) - u;  // padded position mirrored onto u
      if (up >= T && up < L * p) v += gy[(int64_t(b) * p + up % p) * Lalloc + up / p];
    }
    gx[i] = v;
  }
}

// ---------------------------------------------------------------------------
// GAN losses over strided (up to 4-D) views: sum |a - b| (feature matching) or
// sum (a - target)^2 (LSGAN) / sum min(+-a - 1, 0) (hinge), fp64 block partials,
// and their elementwise gradients written into a buffer of the same view.
// ---------------------------------------------------------------------------
struct View4 {
  int64_t size[4];
  int64_t stride[4];
};

// 4-D index of flat element i (last dim fastest) with 32-bit divisions (the host
// permutes the views to memory order, so the last dim is the contiguous one)
struct Idx4 {
  uint32_t i0, i1, i2, i3;
};
__device__ __forceinline__ Idx4 unflat(const View4& v, uint32_t i) {
  Idx4 r;
  const uint32_t s3 = uint32_t(v.size[3]), s2 = uint32_t(v.size[2]), s1 = uint32_t(v.size[1]);
  uint32_t q = i / s3;
  r.i3 = i - q * s3;
  uint32_t q2 = q / s2;
  r.i2 = q - q2 * s2;
  r.i0 = q2 / s1;
  r.i1 = q2 - r.i0 * s1;
  return r;
}
__device__ __forceinline__ int64_t off4(const View4& v, const Idx4& x) {
  return int64_t(x.i0) * v.stride[0] + int64_t(x.i1) * v.stride[1] + int64_t(x.i2) * v.stride[2] +
         int64_t(x.i3) * v.stride[3];
}

// per-element loss term and its derivative (times coef c)
__device__ __forceinline__ float gan_val(int kind, float x, float y, float target) {
  if (kind == 0) return fabsf(x - y);                  // L1
  if (kind == 1) return (x - target) * (x - target);   // MSE to target
  if (kind == 2) return fminf(x - 1.f, 0.f);           // hinge real: min(x - 1, 0)
  if (kind == 3) return fminf(-x - 1.f, 0.f);          // hinge fake: min(-x - 1, 0)
  return x;                                            // plain sum (generator hinge: -mean)
}
__device__ __forceinline__ float gan_dval(int kind, float x, float y, float target, float c) {
  if (kind == 0) {
    const float dlt = x - y;
    return dlt > 0.f ? c : (dlt < 0.f ? -c : 0.f);
  }
  if (kind == 1) return 2.f * (x - target) * c;
  if (kind == 2) return x - 1.f < 0.f ? c : 0.f;
  if (kind == 3) return -x - 1.f < 0.f ? -c : 0.f;
  return c;
}

template <typename T>
__global__ __launch_bounds__(256) void k_gan_reduce(int kind, const T* __restrict__ a, View4 va,
                                                    const T* __restrict__ b, View4 vb, float target, int64_t n,
                                                    double* __restrict__ partials) {
  __shared__ double red[16];
  float s = 0.f;  // per-thread partial (<= a few hundred terms), fp64 across threads and blocks
  for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += int64_t(gridDim.x) * 256) {
    const Idx4 ix = unflat(va, uint32_t(i));
    const float x = to_f(a[off4(va, ix)]);
    s += gan_val(kind, x, kind == 0 ? to_f(b[off4(vb, ix)]) : 0.f, target);
  }
  const double t = block_sum(double(s), red);
  if (threadIdx.x == 0) partials[blockIdx.x] = t;
}

// 16-B vector forms: every view's last dim contiguous with a multiple of V = 16 /
// sizeof(T) elements, the other strides multiples of V and the bases 16-B
// aligned (the channels-last feature maps): one index decomposition and one
// 16-B load per V elements instead of per element
template <typename T>
struct Vec16 {
  static constexpr int V = 16 / sizeof(T);
  T v[V];
};

template <typename T>
__global__ __launch_bounds__(256) void k_gan_reduce_v(int kind, const T* __restrict__ a, View4 va,
                                                      const T* __restrict__ b, View4 vb, float target, uint32_t nv,
                                                      double* __restrict__ partials) {
  constexpr int V = Vec16<T>::V;
  __shared__ double red[16];
  float s = 0.f;
  for (uint32_t iv = blockIdx.x * 256u + threadIdx.x; iv < nv; iv += gridDim.x * 256u) {
    const Idx4 ix = unflat(va, iv * V);
    const Vec16<T> xa = *reinterpret_cast<const Vec16<T>*>(a + off4(va, ix));
    Vec16<T> xb;
    if (kind == 0) xb = *reinterpret_cast<const Vec16<T>*>(b + off4(vb, ix));
#pragma unroll
    for (int e = 0; e < V; ++e) s += gan_val(kind, to_f(xa.v[e]), kind == 0 ? to_f(xb.v[e]) : 0.f, target);
  }
  const double t = block_sum(double(s), red);
  if (threadIdx.x == 0) partials[blockIdx.x] = t;
}

__global__ void k_gan_finish(const double* __restrict__ partials, int nblocks, double scale, float* __restrict__ out,
                             int accumulate) {
  __shared__ double red[16];
  double s = 0.0;
  for (int i = threadIdx.x; i < nblocks; i += blockDim.x) s += partials[i];
  s = block_sum(s, red);
  if (threadIdx.x == 0) out[0] = float(s * scale) + (accumulate ? out[0] : 0.f);
}

// grad[i] (+)= coef * dv/da (coef is a device scalar: the upstream grad / n)
template <typename T>
__global__ __launch_bounds__(256) void k_gan_grad(int kind, const T* __restrict__ a, View4 va,
                                                  const T* __restrict__ b, View4 vb, float target, int64_t n,
                                                  const float* __restrict__ gscale, float mult,
                                                  T* __restrict__ grad, View4 vg, int accumulate) {
  const float c = gscale[0] * mult;
  for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += int64_t(gridDim.x) * 256) {
    const Idx4 ix = unflat(va, uint32_t(i));
    const float x = to_f(a[off4(va, ix)]);
    const float gv = gan_dval(kind, x, kind == 0 ? to_f(b[off4(vb, ix)]) : 0.f, target, c);
    const int64_t o = off4(vg, ix);
    grad[o] = from_f<T>(accumulate ? to_f(grad[o]) + gv : gv);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void k_gan_grad_v(int kind, const T* __restrict__ a, View4 va,
                                                    const T* __restrict__ b, View4 vb, float target, uint32_t nv,
                                                    const float* __restrict__ gscale, float mult,
                                                    T* __restrict__ grad, View4 vg, int accumulate) {
  constexpr int V = Vec16<T>::V;
  const float c = gscale[0] * mult;
  for (uint32_t iv = blockIdx.x * 256u + threadIdx.x; iv < nv; iv += gridDim.x * 256u) {
    const Idx4 ix = unflat(va, iv * V);
    const Vec16<T> xa = *reinterpret_cast<const Vec16<T>*>(a + off4(va, ix));
    Vec16<T> xb, go;
    if (kind == 0) xb = *reinterpret_cast<const Vec16<T>*>(b + off4(vb, ix));
    Vec16<T>* gp = reinterpret_cast<Vec16<T>*>(grad + off4(vg, ix));
    if (accumulate) go = *gp;
#pragma unroll
    for (int e = 0; e < V; ++e) {
      const float gv = gan_dval(kind, to_f(xa.v[e]), kind == 0 ? to_f(xb.v[e]) : 0.f, target, c);
      go.v[e] = from_f<T>(accumulate ? to_f(go.v[e]) + gv : gv);
    }
    *gp = go;
  }
}

// the 16-B vector kernels apply to this view (see Vec16)
template <typename T>
bool vec_view(const void* base, const View4& v) {
  constexpr int V = 16 / sizeof(T);
  return (reinterpret_cast<uintptr_t>(base) & 15) == 0 && v.stride[3] == 1 && v.size[3] % V == 0 &&
         v.stride[0] % V == 0 && v.stride[1] % V == 0 && v.stride[2] % V == 0;
}

}  // namespace dconv
}  // namespace sel

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
using namespace sel;
using namespace sel::dconv;

namespace {

int check(const sel_dconv_desc* d) {
  SEL_REQUIRE(d != nullptr, SEL_ERR_ARG, "null dconv descriptor");
  SEL_REQUIRE(d->B > 0 && d->Tv >= 0 && d->Tvs >= d->Tv && d->Tvs > 0 && d->Tvo > 0 && d->Tvalid >= 0 && d->Tvalid <= d->Tvo && d->K > 0 &&
                  d->S > 0 && d->Cg > 0 && d->G > 0 && d->So > 0 && d->Ng > 0,
              SEL_ERR_ARG, "bad dconv shape B=%d Tv=%d Tvo=%d Tvalid=%d K=%d S=%d Cg=%d G=%d So=%d Ng=%d", d->B,
              d->Tv, d->Tvo, d->Tvalid, d->K, d->S, d->Cg, d->G, d->So, d->Ng);
  SEL_REQUIRE(int64_t(d->S - 1) * d->Cs + int64_t(d->G) * d->Cg <= d->ldx, SEL_ERR_ARG,
              "input columns exceed the row pitch ldx=%d", d->ldx);
  SEL_REQUIRE(int64_t(d->So - 1) * d->Ns + int64_t(d->G) * d->Ng <= d->ldo, SEL_ERR_ARG,
              "output columns exceed the row pitch ldo=%d", d->ldo);
  return SEL_OK;
}

bool mfma_ok(const sel_dconv_desc* d, int dtype) {
  const int vec = dtype == SEL_BF16 ? 8 : 4;
  // 8-channel (bf16) / 4-channel (fp32) vectors may not straddle a phase or a
  // group.  A group narrower than the 32-wide MFMA tile still runs on the
  // matrix cores when its reduction is long (the 1-channel-output convs and the
  // adjoints of the 1-channel-input convs: K * S * Cg >= 256 products per output,
  // where the VALU kernel's per-thread strided row walk is far slower than a
  // 1/32-filled MFMA tile fed from LDS)
  const int width = d->So * d->Ng;
  return d->Cg % vec == 0 && d->Cs % vec == 0 && d->ldx % vec == 0 && (d->S * d->Cg) % 8 == 0 && d->K <= 64 &&
         (width >= 16 || d->K * d->S * d->Cg >= 256);
}

// Very narrow outputs with a short reduction (the MPD first layer's adjoint:
// 3 output phases x 1 channel from 2 taps x 32 channels of gout): one thread
// per output row computes all `width` outputs from 16-B input vectors, weights
// in LDS as fp32 (the generic VALU kernel walked the reduction with one 2-byte
// load per product and thread).  bf16, one group, contiguous reduction row.
template <int MAXW>
__global__ __launch_bounds__(256) void k_dconv_tiny(D d, const __bf16* __restrict__ x, const __bf16* __restrict__ wp,
                                                    const float* __restrict__ bias, const __bf16* __restrict__ aux,
                                                    const __bf16* __restrict__ res, __bf16* __restrict__ out) {
  extern __shared__ float wsm[];  // [width][K][nred]
  const int width = d.So * d.Ng, nred = d.S * d.Cg;
  for (int e = threadIdx.x; e < width * d.K * nred; e += 256) wsm[e] = float(wp[e]);
  __syncthreads();
  const int64_t rows = int64_t(d.B) * d.Tvo;
  for (int64_t row = int64_t(blockIdx.x) * 256 + threadIdx.x; row < rows; row += int64_t(gridDim.x) * 256) {
    const int b = int(row / d.Tvo), j = int(row - int64_t(b) * d.Tvo);
    const bool valid = j < d.Tvalid;
    float acc[MAXW];
#pragma unroll
    for (int o = 0; o < MAXW; ++o) acc[o] = 0.f;
    if (valid) {
      for (int i = 0; i < d.K; ++i) {
        const int t = j + d.q0 + i;
        if (t < 0 || t >= d.Tv) continue;
        const __bf16* xr = x + (int64_t(b) * d.Tvs + t) * d.ldx;
        for (int v = 0; v < nred; v += 8) {
          const uint4 raw = *reinterpret_cast<const uint4*>(xr + v);
          const __bf16* xv = reinterpret_cast<const __bf16*>(&raw);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float xf = float(xv[e]);
#pragma unroll
            for (int o = 0; o < MAXW; ++o)
              if (o < width) acc[o] = fmaf(wsm[(o * d.K + i) * nred + v + e], xf, acc[o]);
          }
        }
      }
    }
    const int64_t orow = (int64_t(b) * d.Tvo + j) * d.ldo;
#pragma unroll
    for (int o = 0; o < MAXW; ++o) {
      if (o >= width) break;
      const int64_t col = out_col(d, 0, o);
      float v = 0.f;
      if (valid) {
        v = acc[o];
        if (bias) v += bias[col];
        if (res) v += float(res[orow + col]);
        if (aux) v *= leaky_grad(float(aux[orow + col]), d.slope);
        if (d.act) v = leaky(v, d.slope);
      }
      out[orow + col] = __bf16(v);
    }
  }
}

bool tiny_ok(const sel_dconv_desc* d, int dtype) {
  const int width = d->So * d->Ng, nred = d->S * d->Cg;
  return dtype == SEL_BF16 && d->G == 1 && (d->S == 1 || d->Cs == d->Cg) && width <= 4 && nred % 8 == 0 &&
         d->ldx % 8 == 0 && size_t(width) * d->K * nred * sizeof(float) <= 48 * 1024 && tune(31) != 1;
}

int launch_tiny(const sel_dconv_desc* d, const void* x, const void* wp, const float* bias, const void* aux,
                const void* res, void* out, hipStream_t s) {
  const int width = d->So * d->Ng, nred = d->S * d->Cg;
  const size_t lds = size_t(width) * d->K * nred * sizeof(float);
  const int64_t rows = int64_t(d->B) * d->Tvo;
  const unsigned blocks = unsigned(std::min<int64_t>((rows + 255) / 256, 4096));
  hipLaunchKernelGGL(k_dconv_tiny<4>, dim3(blocks), dim3(256), lds, s, *d, static_cast<const __bf16*>(x),
                     static_cast<const __bf16*>(wp), bias, static_cast<const __bf16*>(aux),
                     static_cast<const __bf16*>(res), static_cast<__bf16*>(out));
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

template <typename T, int BM, int BN>
int launch_mfma(const sel_dconv_desc* d, const void* x, const void* wp, const float* bias, const void* aux,
                const void* res, void* out, hipStream_t s) {
  constexpr int P = Elt<T>::P;
  const size_t lds = (size_t(BM + d->K - 1) * P + size_t(BN) * KC * P) * sizeof(T);
  SEL_REQUIRE(lds <= 160 * 1024, SEL_ERR_UNSUPPORTED, "dconv tile needs %zu B of LDS", lds);
  const int tps = (d->Tvo + BM - 1) / BM;
  const int ntg = (d->So * d->Ng + BN - 1) / BN;
  dim3 grid(unsigned((int64_t(d->B) * tps + 7) / 8 * 8), unsigned(ntg * d->G));  // xcd_rowtile
  if constexpr (sizeof(T) == 2) {
    // register-prefetched pipeline (same stages, same bits; tune key 30 = 1: off);
    // its prefetch registers cover a span of BM + 63 rows
    if (tune(30) != 1 && d->K - 1 <= KC * 8) {
      auto kg = k_dconv_gpf<BM, BN>;
      if (lds > 64 * 1024)
        SEL_HIP(hipFuncSetAttribute((const void*)kg, hipFuncAttributeMaxDynamicSharedMemorySize, int(lds)));
      hipLaunchKernelGGL(kg, grid, dim3(256), lds, s, *d, static_cast<const __bf16*>(x),
                         static_cast<const __bf16*>(wp), bias, static_cast<const __bf16*>(aux),
                         static_cast<const __bf16*>(res), static_cast<__bf16*>(out));
      SEL_LAUNCH_CHECK();
      return SEL_OK;
    }
  }
  auto kern = k_dconv_mfma<T, BM, BN>;
  if (lds > 64 * 1024)
    SEL_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, int(lds)));
  hipLaunchKernelGGL(kern, grid, dim3(256), lds, s, *d, static_cast<const T*>(x), static_cast<const T*>(wp), bias,
                     static_cast<const T*>(aux), static_cast<const T*>(res), static_cast<T*>(out));
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

template <typename T>
int launch_valu(const sel_dconv_desc* d, const void* x, const void* wp, const float* bias, const void* aux,
                const void* res, void* out, hipStream_t s) {
  const int64_t total = int64_t(d->B) * d->Tvo * d->G * d->So * d->Ng;
  const unsigned blocks = unsigned(std::min<int64_t>((total + 255) / 256, 65536));
  hipLaunchKernelGGL(k_dconv_valu<T>, dim3(blocks), dim3(256), 0, s, *d, static_cast<const T*>(x),
                     static_cast<const T*>(wp), bias, static_cast<const T*>(aux), static_cast<const T*>(res),
                     static_cast<T*>(out));
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

// instantiated reductions: MSD first conv (15 taps), MPD first conv (2 taps x 3
// phases), the adjoints of the 1-channel output convs (3 / 2 taps)
bool short_kr_ok(int kr) { return kr == 2 || kr == 3 || kr == 6 || kr == 15; }

bool short_ok(const sel_dconv_desc* d) {
  return d->G == 1 && d->So == 1 && d->Ng % 8 == 0 && d->ldo % 8 == 0 && short_kr_ok(d->K * d->S * d->Cg) &&
         int64_t(d->B) * d->Tvo + 4 < (int64_t(1) << 31) &&
         size_t(d->Ng) * d->K * d->S * d->Cg * sizeof(float) <= 64 * 1024;
}

// the staged kernel's (K, NR) instances; nullptr: use k_dconv_short
template <typename T>
decltype(&k_dconv_shortx<T, 15, 1>) shortx_kernel(const sel_dconv_desc* d) {
  const int nr = d->S * d->Cg, n8 = d->Ng / 8;
  if (tune(18) == 1 || d->G != 1 || d->So != 1 || d->Cs != d->Cg || d->ldx != nr || d->Ng % 8 != 0 || n8 > 256 ||
      256 % n8 != 0)
    return nullptr;
  const int K = d->K;
  if (K == 15 && nr == 1) return k_dconv_shortx<T, 15, 1>;
  if (K == 2 && nr == 3) return k_dconv_shortx<T, 2, 3>;
  if (K == 3 && nr == 1) return k_dconv_shortx<T, 3, 1>;
  if (K == 2 && nr == 1) return k_dconv_shortx<T, 2, 1>;
  if (K == 6 && nr == 1) return k_dconv_shortx<T, 6, 1>;
  if (K == 1 && nr == 2) return k_dconv_shortx<T, 1, 2>;
  if (K == 1 && nr == 3) return k_dconv_shortx<T, 1, 3>;
  return nullptr;
}

template <typename T>
int launch_short(const sel_dconv_desc* d, const void* x, const void* wp, const float* bias, const void* aux,
                 const void* res, void* out, hipStream_t s) {
  if (auto kx = shortx_kernel<T>(d)) {
    // tune key 18: 1 = the unstaged kernel
    const int kr = d->K * d->S * d->Cg, rb = 256 / (d->Ng / 8) * 8;
    const size_t lds = (size_t(d->Ng) * kr + size_t(rb + d->K - 1) * d->S * d->Cg) * sizeof(float);
    const int64_t ntiles = int64_t(d->B) * ((d->Tvo + rb - 1) / rb);
    const unsigned blocks = unsigned(std::min<int64_t>(ntiles, 2048));
    if (lds > 64 * 1024)
      SEL_HIP(hipFuncSetAttribute((const void*)kx, hipFuncAttributeMaxDynamicSharedMemorySize, int(lds)));
    hipLaunchKernelGGL(kx, dim3(blocks), dim3(256), lds, s, *d, static_cast<const T*>(x), static_cast<const T*>(wp),
                       bias, static_cast<const T*>(aux), static_cast<const T*>(res), static_cast<T*>(out));
    SEL_LAUNCH_CHECK();
    return SEL_OK;
  }
  const int64_t total = (int64_t(d->B) * d->Tvo + 3) / 4 * (d->Ng / 8);
  const unsigned blocks = unsigned(std::min<int64_t>((total + 255) / 256, 16384));
  const int kr = d->K * d->S * d->Cg;
  const size_t lds = size_t(d->Ng) * kr * sizeof(float);
  auto kern = kr == 2 ? k_dconv_short<T, 2> : kr == 3 ? k_dconv_short<T, 3> : kr == 6 ? k_dconv_short<T, 6>
                                                                                    : k_dconv_short<T, 15>;
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), lds, s, *d, static_cast<const T*>(x), static_cast<const T*>(wp),
                     bias, static_cast<const T*>(aux), static_cast<const T*>(res), static_cast<T*>(out));
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

template <int BM, int BN>
int launch_pf(const sel_dconv_desc* d, const void* x, const void* wp, const float* bias, const void* aux,
              const void* res, void* out, hipStream_t s) {
  constexpr int P = Elt<__bf16>::P;
  const size_t lds = (size_t(BM + d->K - 1) + size_t(d->K) * BN) * P * sizeof(__bf16);
  const int tps = (d->Tvo + BM - 1) / BM;
  const int ntg = (d->So * d->Ng + BN - 1) / BN;
  dim3 grid(unsigned((int64_t(d->B) * tps + 7) / 8 * 8), unsigned(ntg));  // xcd_rowtile
  auto kern = k_dconv_pf<BM, BN>;
  if (lds > 64 * 1024)
    SEL_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, int(lds)));
  hipLaunchKernelGGL(kern, grid, dim3(256), lds, s, *d, static_cast<const __bf16*>(x), static_cast<const __bf16*>(wp),
                     bias, static_cast<const __bf16*>(aux), static_cast<const __bf16*>(res), static_cast<__bf16*>(out));
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

// the prefetching kernel's shapes: bf16, one group, contiguous reduction rows, K <= 8
bool pf_ok(const sel_dconv_desc* d, int dtype) {
  return dtype == SEL_BF16 && d->G == 1 && (d->S == 1 || d->Cs == d->Cg) && d->K <= PF_KMAX && tune(16) != 1;
}

// Kernel family a forward / adjoint launch of this shape takes (include/sel.h
// SEL_DPATH_*): the single decision both the launcher and sel_dconv_kernel use.
struct FwdPlan {
  int path, bm, bn;
};

FwdPlan plan_fwd(const sel_dconv_desc* d, int dtype) {
  if (tune(9) == 1) return {SEL_DPATH_VALU, 0, 0};
  if (!mfma_ok(d, dtype)) {
    if (short_ok(d)) return {shortx_kernel<float>(d) ? SEL_DPATH_SHORTX : SEL_DPATH_SHORT, 0, 0};
    // tune key 31 = 1: the generic VALU kernel instead of the narrow-output one
    if (tiny_ok(d, dtype)) return {SEL_DPATH_TINY, 0, 0};
    return {SEL_DPATH_VALU, 0, 0};
  }
  const int width = d->So * d->Ng;
  const int64_t rows = int64_t(d->B) * d->Tvo;
  const bool bf = dtype == SEL_BF16;
  if (bf) {
    // the MPD's >= 128-wide one-group layers and adjoints: warp-specialised
    // 256 x 128 tiles (conv.hip k_conv_ws_bf16; tune key 21: 1 = off)
    if (tune(21) != 1 && width % 128 == 0 && d->S * d->Cg >= 64 && rows * (width / 128) >= 65536) {
      const int m = sel::conv::dconv_ws_mode(d);
      if (m >= 0) return {m == 1 ? SEL_DPATH_WS_FLAT : SEL_DPATH_WS, 256, sel::conv::dconv_ws8_ok(d) ? 256 : 128};
    }
    if (width > 32 && pf_ok(d, dtype)) {
      // tune key 19: tile A/B (1: 256x64, 2: 128x128, 3: 256x128)
      if (tune(19) == 1) return {SEL_DPATH_PF, 256, 64};
      if (tune(19) == 3 && width % 128 == 0) return {SEL_DPATH_PF, 256, 128};
      // 128-column tiles halve the input re-staging per output (MPD 512 -> 1024 k5 s3: 8.4 -> 5.5 ms,
      // 1024 -> 1024 k5: 1.22 -> 0.80 ms at the probe's sizes, tools/dconv_probe.py, bit-identical)
      if (width % 128 == 0 && (tune(19) == 2 || (tune(19) == 0 && rows * (width / 128) >= 65536)))
        return {SEL_DPATH_PF, 128, 128};
      if (rows * (width / 64) < 65536) return {SEL_DPATH_PF, 64, 64};
      return {SEL_DPATH_PF, 128, 64};
    }
  }
  int bm, bn;
  // narrow groups: 32-wide tiles; short sequences / few rows: 64-row tiles
  if (width <= 32) {
    bn = 32;
    bm = rows * d->G < 131072 ? 128 : 256;
  } else if (rows * d->G * (width / 64) < 65536) {
    bm = 64, bn = 64;
  } else {
    // 256-row tiles: each staged tap group of weights serves twice the rows (the
    // MSD's 41-tap grouped layers: C5 50.5 -> 49.7 ms/step; tune key 28 bit 0 = 128 rows)
    bm = bf && !(tune(28) & 1) ? 256 : 128, bn = 64;
  }
  // register-prefetched pipeline (same stages, same bits; tune key 30 = 1: off)
  const bool gpf = bf && tune(30) != 1 && d->K - 1 <= KC * 8;
  return {gpf ? SEL_DPATH_GPF : SEL_DPATH_MFMA, bm, bn};
}

template <typename T>
int dispatch_fwd(const sel_dconv_desc* d, const void* x, const void* wp, const float* bias, const void* aux,
                 const void* res, void* out, hipStream_t s, int dtype) {
  const FwdPlan p = plan_fwd(d, dtype);
  switch (p.path) {
    case SEL_DPATH_VALU: return launch_valu<T>(d, x, wp, bias, aux, res, out, s);
    case SEL_DPATH_SHORT:
    case SEL_DPATH_SHORTX: return launch_short<T>(d, x, wp, bias, aux, res, out, s);
    case SEL_DPATH_TINY: return launch_tiny(d, x, wp, bias, aux, res, out, s);
    default: break;
  }
  if constexpr (sizeof(T) == 2) {
    if (p.path == SEL_DPATH_WS || p.path == SEL_DPATH_WS_FLAT)
      return sel::conv::dconv_ws_fwd(d, x, wp, bias, aux, res, out, s);
    if (p.path == SEL_DPATH_PF) {
      if (p.bm == 256 && p.bn == 64) return launch_pf<256, 64>(d, x, wp, bias, aux, res, out, s);
      if (p.bm == 256) return launch_pf<256, 128>(d, x, wp, bias, aux, res, out, s);
      if (p.bn == 128) return launch_pf<128, 128>(d, x, wp, bias, aux, res, out, s);
      if (p.bm == 64) return launch_pf<64, 64>(d, x, wp, bias, aux, res, out, s);
      return launch_pf<128, 64>(d, x, wp, bias, aux, res, out, s);
    }
  }
  // k_dconv_mfma / k_dconv_gpf (launch_mfma makes the same gpf choice)
  if (p.bn == 32) {
    if (p.bm == 128) return launch_mfma<T, 128, 32>(d, x, wp, bias, aux, res, out, s);
    return launch_mfma<T, 256, 32>(d, x, wp, bias, aux, res, out, s);
  }
  if (p.bm == 64) return launch_mfma<T, 64, 64>(d, x, wp, bias, aux, res, out, s);
  if (p.bm == 256) return launch_mfma<T, 256, 64>(d, x, wp, bias, aux, res, out, s);
  return launch_mfma<T, 128, 64>(d, x, wp, bias, aux, res, out, s);
}

struct WgPlanD {
  int flat_p;  // k_dwgrad_w3 flat tiling pitch (0: per-sequence tiles)
  bool mfma, shortk, w3;
  int w3_nt, w3_ct, w3_maxt;
  int nsplit, bsplit;
  int rows_per_split, brows_per_split;
  int tiles_per_seq, tiles_per_split, ntg, nt;
};

// split-partial budget per layer (bytes; tune key 45 > 0: MB, A/B sweeps)
inline int64_t wg_cap() { return int64_t(tune(45) > 0 ? tune(45) : 64) << 20; }

WgPlanD wg_plan(const sel_dconv_desc* d, int dtype) {
  WgPlanD p{};
  const int width = d->So * d->Ng;
  const int nred = d->S * d->Cg;
  p.mfma = dtype == SEL_BF16 && d->Cg % 8 == 0 && d->Cs % 8 == 0 && d->ldx % 8 == 0 && nred % 8 == 0 &&
           width % 16 == 0 && tune(9) != 1;
  const int64_t rows = int64_t(d->B) * d->Tvalid;
  const int64_t nw = int64_t(d->G) * width * d->K * nred;
  p.shortk = !p.mfma && tune(9) != 1 && d->G == 1 && d->So == 1 && d->Ng <= 256 && (256 % d->Ng) == 0 &&
             short_kr_ok(d->K * nred);
  if (p.shortk) {
    const int64_t want = std::max<int64_t>(1, std::min<int64_t>(2048, rows / 64));
    p.rows_per_split = int((rows + want - 1) / want);
    p.nsplit = int((rows + p.rows_per_split - 1) / p.rows_per_split);
    p.bsplit = p.nsplit;
    return p;
  }
  p.w3 = p.mfma && d->G == 1 && d->So == 1 && (d->S == 1 || d->Cs == d->Cg) && d->K <= 8 && width % 32 == 0 &&
         nred % 32 == 0 && d->ldo % 8 == 0 && tune(16) != 1 &&
         // gout and x as buffer resources (ru_rsrc): ru_region_ok
         ru_region_ok(int64_t(d->B) * d->Tvo * d->ldo * 2) && ru_region_ok(int64_t(d->B) * d->Tvs * d->ldx * 2);
  if (p.w3) {
    p.w3_nt = width % 64 == 0 ? 2 : 1;
    p.w3_ct = nred % 64 == 0 ? 2 : 1;
    const int P = p.w3_ct * d->K, WPN = 4 / p.w3_nt;
    const int RG = P >= WPN ? 1 : WPN / P, WPP = WPN / RG;
    const int need = (P + WPP - 1) / WPP;
    // exact per-wave tile count where an instance exists (the MPD's K = 5 layers at
    // 64 input channels per block: 5 pairs per wave, which the 8-slot form ran
    // with 3 of 8 MFMA slots computing never-stored accumulators)
    p.w3_maxt = need <= 5 ? need : 8;
    // flat tiling across zero-gapped sequences (the conditions of conv.hip
    // dconv_ws_fwd; tune key 26 = 1: off): short MPD columns fill whole tiles
    const int P_ = d->Tvo;
    p.flat_p = tune(26) != 1 && d->Tvs == P_ && P_ - d->Tv >= -d->q0 && P_ - d->Tvalid >= d->q0 + d->K - 1 &&
                       int64_t(d->B) * P_ < (int64_t(1) << 31)
                   ? P_ : 0;
    p.tiles_per_seq = p.flat_p ? int((int64_t(d->B) * P_ + W3_BM - 1) / W3_BM) : (d->Tvalid + W3_BM - 1) / W3_BM;
    const int64_t ntiles = p.flat_p ? p.tiles_per_seq : int64_t(d->B) * p.tiles_per_seq;
    const int64_t blocks = int64_t(width / (32 * p.w3_nt)) * (nred / (32 * p.w3_ct));
    int64_t want = std::max<int64_t>(1, (512 + blocks - 1) / blocks);
    want = std::min<int64_t>(want, std::max<int64_t>(1, wg_cap() / (nw * 4)));
    want = std::min<int64_t>(want, std::max<int64_t>(1, ntiles));
    p.tiles_per_split = int((ntiles + want - 1) / want);
    p.nsplit = int((ntiles + p.tiles_per_split - 1) / p.tiles_per_split);
  } else if (p.mfma) {
    p.nt = width % 32 == 0 ? 2 : 1;
    p.ntg = (d->K + WG_TAPS - 1) / WG_TAPS;
    p.tiles_per_seq = (d->Tvalid + WG_BM - 1) / WG_BM;
    const int64_t ntiles = int64_t(d->B) * p.tiles_per_seq;
    const int64_t blocks = int64_t(d->G) * ((width + 16 * p.nt - 1) / (16 * p.nt)) * ((nred + 31) / 32) * p.ntg;
    int64_t want = std::max<int64_t>(1, (1024 + blocks - 1) / blocks);
    want = std::min<int64_t>(want, std::max<int64_t>(1, wg_cap() / (nw * 4)));
    want = std::min<int64_t>(want, std::max<int64_t>(1, ntiles));
    p.tiles_per_split = int((ntiles + want - 1) / want);
    p.nsplit = int((ntiles + p.tiles_per_split - 1) / p.tiles_per_split);
  } else {
    const int64_t want_threads = int64_t(1) << 20;
    int64_t want = std::max<int64_t>(1, want_threads / std::max<int64_t>(1, nw + int64_t(d->G) * width));
    want = std::min<int64_t>(want, std::max<int64_t>(1, wg_cap() / ((nw + width * d->G) * 4)));
    want = std::min<int64_t>(want, std::max<int64_t>(1, rows));
    p.rows_per_split = int((rows + want - 1) / want);
    p.nsplit = int((rows + p.rows_per_split - 1) / p.rows_per_split);
  }
  int64_t bwant = std::max<int64_t>(1, std::min<int64_t>(256, rows / 256));
  p.brows_per_split = int((rows + bwant - 1) / bwant);
  p.bsplit = int((rows + p.brows_per_split - 1) / std::max(1, p.brows_per_split));
  if (p.bsplit < 1) p.bsplit = 1;
  if (p.w3) p.bsplit = p.nsplit;  // k_dwgrad_w3 writes the bias partials of its own splits
  return p;
}

size_t wg_bytes(const sel_dconv_desc* d, const WgPlanD& p) {
  const int64_t width = int64_t(d->So) * d->Ng;
  const int64_t nw = int64_t(d->G) * width * d->K * d->S * d->Cg;
  const int64_t nb = int64_t(d->G) * width;
  const int64_t ng = (p.nsplit + PRESUM - 1) / PRESUM;
  return size_t(int64_t(p.nsplit) * nw + int64_t(std::max(p.bsplit, p.nsplit)) * nb + (ng + 1) * nw) * sizeof(float) +
         256;
}

hipError_t wgrad_fill(const sel_dconv_desc* d, int dtype, const WgPlanD& p, const void* gout, const void* x,
                      float* part, float* bpart, hipStream_t s) {
  const int width = d->So * d->Ng;
  const int nred = d->S * d->Cg;
  if (p.shortk) {
    const int kr = d->K * nred;
    // staged kernel (tune key 18: 1 = off) where the phase view is contiguous
    if (tune(18) != 1 && d->Cs == d->Cg && d->ldx == nred && d->Ng % 2 == 0 && d->ldo % 2 == 0 &&
        int64_t(d->B) * d->Tvo < (int64_t(1) << 31)) {
      const int rl = 256 / (d->Ng / 2), rb = rl * 16;
      const size_t lds = std::max<size_t>(size_t(rb + d->K - 1) * nred, size_t(rl) * d->Ng * (kr + 1)) * sizeof(float);
      void (*kx)(D, const __bf16*, const __bf16*, float*, float*) = nullptr;
      void (*kf)(D, const float*, const float*, float*, float*) = nullptr;
#define SEL_DWSX(K_, NR_)                                                       \
  if (d->K == K_ && nred == NR_) {                                              \
    kx = k_dwgrad_shortx<__bf16, K_, NR_>;                                      \
    kf = k_dwgrad_shortx<float, K_, NR_>;                                       \
  }
      SEL_DWSX(15, 1) SEL_DWSX(2, 3) SEL_DWSX(3, 1) SEL_DWSX(2, 1) SEL_DWSX(6, 1) SEL_DWSX(1, 2) SEL_DWSX(1, 3)
#undef SEL_DWSX
      if (kx) {
        const void* kern = dtype == SEL_BF16 ? (const void*)kx : (const void*)kf;
        if (lds > 64 * 1024) {
          const hipError_t e = hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
          if (e != hipSuccess) return e;
        }
        if (dtype == SEL_BF16)
          hipLaunchKernelGGL(kx, dim3(p.nsplit), dim3(256), lds, s, *d, static_cast<const __bf16*>(gout),
                             static_cast<const __bf16*>(x), part, bpart);
        else
          hipLaunchKernelGGL(kf, dim3(p.nsplit), dim3(256), lds, s, *d, static_cast<const float*>(gout),
                             static_cast<const float*>(x), part, bpart);
        return hipGetLastError();
      }
    }
#define SEL_DWS(TT, KR)                                                                                     \
  hipLaunchKernelGGL((k_dwgrad_short<TT, KR>), dim3(p.nsplit), dim3(256), 0, s, *d, static_cast<const TT*>(gout), \
                     static_cast<const TT*>(x), p.rows_per_split, part, bpart)
#define SEL_DWS_T(TT) \
  if (kr == 2) SEL_DWS(TT, 2); else if (kr == 3) SEL_DWS(TT, 3); else if (kr == 6) SEL_DWS(TT, 6); else SEL_DWS(TT, 15);
    if (dtype == SEL_BF16) { SEL_DWS_T(__bf16) } else { SEL_DWS_T(float) }
#undef SEL_DWS_T
#undef SEL_DWS
    return hipGetLastError();
  }
  if (p.w3) {
    const int NB = 32 * p.w3_nt, CB = 32 * p.w3_ct;
    const size_t lds = 2 * (size_t(p.w3_nt) * W3_BM * 32 + size_t(p.w3_ct) * (W3_BM + W3_HALO) * 32) * sizeof(__bf16);
    const int64_t ntiles = p.flat_p ? p.tiles_per_seq : int64_t(d->B) * p.tiles_per_seq;
    dim3 grid(unsigned(p.nsplit), unsigned(width / NB), unsigned(nred / CB));
#define SEL_W3(NT_, CT_, MT_)                                                                                    if (p.w3_nt == NT_ && p.w3_ct == CT_ && p.w3_maxt == MT_) {                                                      auto kern = k_dwgrad_w3<NT_, CT_, MT_>;                                                                        if (lds > 64 * 1024) {                                                                                           const hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,                                                int(lds));                                                            if (e != hipSuccess) return e;                                                                               }                                                                                                              hipLaunchKernelGGL(kern, grid, dim3(256), lds, s, *d, static_cast<const __bf16*>(gout),                                            static_cast<const __bf16*>(x), p.tiles_per_seq, ntiles, p.tiles_per_split, part, p.flat_p, bpart);  } else
    SEL_W3(1, 1, 1) SEL_W3(1, 1, 2) SEL_W3(1, 1, 3) SEL_W3(1, 1, 4) SEL_W3(1, 1, 5)
    SEL_W3(1, 2, 1) SEL_W3(1, 2, 2) SEL_W3(1, 2, 3) SEL_W3(1, 2, 4) SEL_W3(1, 2, 5)
    SEL_W3(2, 1, 1) SEL_W3(2, 1, 2) SEL_W3(2, 1, 3) SEL_W3(2, 1, 4) SEL_W3(2, 1, 5) SEL_W3(2, 1, 8)
    SEL_W3(2, 2, 1) SEL_W3(2, 2, 2) SEL_W3(2, 2, 3) SEL_W3(2, 2, 4) SEL_W3(2, 2, 5) SEL_W3(2, 2, 8)
    { return hipErrorInvalidValue; }
#undef SEL_W3
    return hipGetLastError();  // (bias partials: in the kernel, p.bsplit == p.nsplit)
  }
  if (p.mfma) {
    const int bn = 16 * p.nt;
    dim3 grid(unsigned(d->G * ((width + bn - 1) / bn)), unsigned((nred + 31) / 32), unsigned(p.nsplit * p.ntg));
    const size_t lds = (size_t(WG_BM) * (bn + 16) + size_t(WG_BM + WG_TAPS - 1) * 48) * sizeof(__bf16);
    if (p.nt == 2)
      hipLaunchKernelGGL(k_dwgrad_mfma<2>, grid, dim3(256), lds, s, *d, static_cast<const __bf16*>(gout),
                         static_cast<const __bf16*>(x), p.tiles_per_seq, p.tiles_per_split, p.ntg, part);
    else
      hipLaunchKernelGGL(k_dwgrad_mfma<1>, grid, dim3(256), lds, s, *d, static_cast<const __bf16*>(gout),
                         static_cast<const __bf16*>(x), p.tiles_per_seq, p.tiles_per_split, p.ntg, part);
    if (bpart) launch_dbias_part(d, static_cast<const __bf16*>(gout), p.brows_per_split, p.bsplit, bpart, s);
    return hipGetLastError();
  }
  const int64_t nw = int64_t(d->G) * width * d->K * nred;
  const int64_t nb = bpart ? int64_t(d->G) * width : 0;
  dim3 grid(unsigned(std::min<int64_t>((nw + nb + 255) / 256, 65535)), unsigned(p.nsplit));
  if (dtype == SEL_BF16)
    hipLaunchKernelGGL(k_dwgrad_valu<__bf16>, grid, dim3(256), 0, s, *d, static_cast<const __bf16*>(gout),
                       static_cast<const __bf16*>(x), p.rows_per_split, part, bpart);
  else
    hipLaunchKernelGGL(k_dwgrad_valu<float>, grid, dim3(256), 0, s, *d, static_cast<const float*>(gout),
                       static_cast<const float*>(x), p.rows_per_split, part, bpart);
  return hipGetLastError();
}

int launch_blocks(int64_t n) { return int(std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 8192))); }

bool view_ok(const int64_t* size, const int64_t* stride) { return size && stride; }

View4 to_view(const int64_t* size, const int64_t* stride, int ndim) {
  View4 v;
  for (int i = 0; i < 4; ++i) {
    const int src = i - (4 - ndim);
    v.size[i] = src >= 0 ? size[src] : 1;
    v.stride[i] = src >= 0 ? stride[src] : 0;
  }
  return v;
}

}  // namespace

extern "C" {

int sel_dconv_fwd(const sel_dconv_desc* d, int dtype, const void* x, const void* wpack, const float* bias,
                  const void* aux, const void* res, void* out, sel_stream_t stream) {
  if (int rc = check(d)) return rc;
  SEL_REQUIRE(x && wpack && out, SEL_ERR_ARG, "null pointer");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (dtype == SEL_BF16) return dispatch_fwd<__bf16>(d, x, wpack, bias, aux, res, out, s, dtype);
  if (dtype == SEL_F32) return dispatch_fwd<float>(d, x, wpack, bias, aux, res, out, s, dtype);
  set_error("sel_dconv_fwd: unsupported dtype %d", dtype);
  return SEL_ERR_UNSUPPORTED;
}

int sel_dconv_kernel(const sel_dconv_desc* d, int dtype, char* name, size_t cap) {
  if (!d || check(d) != SEL_OK || (dtype != SEL_BF16 && dtype != SEL_F32)) return -1;
  const FwdPlan p = plan_fwd(d, dtype);
  if (name && cap) {
    const char* t = dtype == SEL_BF16 ? "bf16" : "float";
    switch (p.path) {
      case SEL_DPATH_WS:
      case SEL_DPATH_WS_FLAT:
        if (p.bn == 256) snprintf(name, cap, "k_conv_ws8<%d, bf16, 256, 256>", d->K);
        else snprintf(name, cap, "k_conv_ws_bf16<%d>", d->K);
        break;
      case SEL_DPATH_PF: snprintf(name, cap, "k_dconv_pf<%d, %d>", p.bm, p.bn); break;
      case SEL_DPATH_GPF: snprintf(name, cap, "k_dconv_gpf<%d, %d>", p.bm, p.bn); break;
      case SEL_DPATH_MFMA: snprintf(name, cap, "k_dconv_mfma<%s, %d, %d>", t, p.bm, p.bn); break;
      case SEL_DPATH_SHORTX: snprintf(name, cap, "k_dconv_shortx<%s, %d, %d>", t, d->K, d->S * d->Cg); break;
      case SEL_DPATH_SHORT: snprintf(name, cap, "k_dconv_short<%s, %d>", t, d->K * d->S * d->Cg); break;
      case SEL_DPATH_TINY: snprintf(name, cap, "k_dconv_tiny<4>"); break;
      default: snprintf(name, cap, "k_dconv_valu<%s>", t); break;
    }
  }
  return p.path;
}

size_t sel_dconv_wgrad_workspace(const sel_dconv_desc* d, int dtype) {
  if (!d || check(d) != SEL_OK) return 16;
  return wg_bytes(d, wg_plan(d, dtype));
}

int sel_dconv_wgrad(const sel_dconv_desc* d, int dtype, const void* gout, const void* x, int N, int Cg, int Kt,
                    int stride, int pad, const float* v, const float* wg, float* gw, float* gg, float* gb, void* ws,
                    size_t ws_bytes, sel_stream_t stream) {
  sel_dwgrad_job job;
  if (int rc = sel_dconv_wgrad_partials(d, dtype, gout, x, N, Cg, Kt, stride, pad, v, wg, gw, gg, gb, ws, ws_bytes,
                                        &job, stream))
    return rc;
  const PackGeo pg = pack_geo(job.N, job.Cg, job.Kt, job.stride, job.pad, job.G);
  hipLaunchKernelGGL(k_dwgrad_finish, dim3(job.N), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), pg,
                     job.part, job.nsplit, job.bpart, job.bsplit, job.v, job.wg, job.gw, job.gg, job.gb);
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

int sel_dconv_wgrad_finish_many(const sel_dwgrad_job* jobs, int njobs, sel_stream_t stream) {
  SEL_REQUIRE(njobs >= 0 && (njobs == 0 || jobs), SEL_ERR_ARG, "bad wgrad finish job list");
  for (int j = 0; j < njobs; ++j) {
    const sel_dwgrad_job& J = jobs[j];
    SEL_REQUIRE(J.part && J.gw && J.N > 0 && J.Cg > 0 && J.Kt > 0 && J.stride > 0 && J.pad >= 0 && J.G > 0 &&
                    J.N % J.G == 0 && J.nsplit > 0 && J.nsplit <= PRESUM && (!J.gb || (J.bpart && J.bsplit > 0)) &&
                    (!J.v || (J.wg && J.gg)),
                SEL_ERR_ARG, "bad wgrad finish job %d", j);
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  int j = 0;
  while (j < njobs) {
    DwgradJobs dj{};
    int n = 0, blocks = 0;
    for (; j < njobs && n < DWF_MAXJ; ++j, ++n) {
      const sel_dwgrad_job& J = jobs[j];
      dj.pg[n] = pack_geo(J.N, J.Cg, J.Kt, J.stride, J.pad, J.G);
      dj.part[n] = J.part;
      dj.bpart[n] = J.bpart;
      dj.nsplit[n] = J.nsplit;
      dj.bsplit[n] = J.bsplit;
      dj.v[n] = J.v;
      dj.wg[n] = J.wg;
      dj.gw[n] = J.gw;
      dj.gg[n] = J.gg;
      dj.gb[n] = J.gb;
      dj.bstart[n] = blocks;
      blocks += J.N;
    }
    dj.bstart[n] = blocks;
    dj.njobs = n;
    hipLaunchKernelGGL(k_dwgrad_finish_many, dim3(unsigned(blocks)), dim3(256), 0, s, dj);
    SEL_LAUNCH_CHECK();
  }
  return SEL_OK;
}

int sel_dconv_wgrad_partials(const sel_dconv_desc* d, int dtype, const void* gout, const void* x, int N, int Cg,
                             int Kt, int stride, int pad, const float* v, const float* wg, float* gw, float* gg,
                             float* gb, void* ws, size_t ws_bytes, sel_dwgrad_job* job, sel_stream_t stream) {
  SEL_REQUIRE(job != nullptr, SEL_ERR_ARG, "sel_dconv_wgrad_partials: job is NULL");
  if (int rc = check(d)) return rc;
  SEL_REQUIRE(dtype == SEL_BF16 || dtype == SEL_F32, SEL_ERR_UNSUPPORTED, "dtype %d", dtype);
  SEL_REQUIRE(d->So == 1 && d->S == stride && d->G * d->Ng == N && d->Cg == Cg, SEL_ERR_ARG,
              "sel_dconv_wgrad: descriptor must be the forward layer's");
  const PackGeo pg = pack_geo(N, Cg, Kt, stride, pad, d->G);
  SEL_REQUIRE(pg.K == d->K && pg.q0 == d->q0, SEL_ERR_ARG, "tap geometry mismatch (K %d vs %d, q0 %d vs %d)",
              pg.K, d->K, pg.q0, d->q0);
  SEL_REQUIRE(!v || (wg && gg), SEL_ERR_ARG, "weight norm needs v, g and gg");
  const WgPlanD p = wg_plan(d, dtype);
  SEL_REQUIRE(ws_bytes >= wg_bytes(d, p), SEL_ERR_WORKSPACE, "wgrad workspace too small");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  float* part = static_cast<float*>(ws);
  const int64_t nw = int64_t(N) * d->K * d->S * d->Cg;
  float* bpart = gb ? part + int64_t(p.nsplit) * nw : nullptr;
  SEL_HIP(wgrad_fill(d, dtype, p, gout, x, part, bpart, s));
  const int bsplit = (p.mfma || p.shortk) ? p.bsplit : p.nsplit;
  int nsplit = p.nsplit;
  if (nsplit > PRESUM) {  // fold the partials to <= PRESUM per weight before the per-output pass
    float* tmp = part + int64_t(p.nsplit) * nw + int64_t(std::max(p.bsplit, p.nsplit)) * N;
    float* src = part;
    while (nsplit > PRESUM) {
      const int ng = (nsplit + PRESUM - 1) / PRESUM;
      float* dst = src == part ? tmp : part;
      hipLaunchKernelGGL(k_presum, dim3(unsigned((nw + 255) / 256), unsigned(ng)), dim3(256), 0, s, src, nsplit, nw,
                         dst);
      src = dst;
      nsplit = ng;
    }
    part = src;
  }
  *job = sel_dwgrad_job{part, bpart, v, wg, gw, gg, gb, N, Cg, Kt, stride, pad, d->G, nsplit, bsplit};
  return SEL_OK;
}

int sel_dconv_geometry(int Kt, int stride, int pad, int* K, int* q0) {
  SEL_REQUIRE(Kt > 0 && stride > 0 && pad >= 0 && K && q0, SEL_ERR_ARG, "bad conv geometry");
  const PackGeo pg = pack_geo(1, 1, Kt, stride, pad, 1);
  *K = pg.K;
  *q0 = pg.q0;
  return SEL_OK;
}

int sel_dconv_pack(int mode, const float* w, const float* wg, int N, int Cg, int Kt, int stride, int pad, int G,
                   int dtype, void* out, sel_stream_t stream) {
  SEL_REQUIRE(w && out && N > 0 && Cg > 0 && Kt > 0 && stride > 0 && pad >= 0 && G > 0 && N % G == 0 &&
                  (mode == 0 || mode == 1),
              SEL_ERR_ARG, "bad dconv pack arguments");
  const PackGeo pg = pack_geo(N, Cg, Kt, stride, pad, G);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (dtype == SEL_BF16)
    hipLaunchKernelGGL(k_dpack<__bf16>, dim3(N), dim3(256), 0, s, pg, mode, w, wg, static_cast<__bf16*>(out));
  else if (dtype == SEL_F32)
    hipLaunchKernelGGL(k_dpack<float>, dim3(N), dim3(256), 0, s, pg, mode, w, wg, static_cast<float*>(out));
  else {
    set_error("sel_dconv_pack: dtype %d", dtype);
    return SEL_ERR_UNSUPPORTED;
  }
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

int sel_dconv_pack_many(const sel_dpack_job* jobs, int njobs, int dtype, sel_stream_t stream) {
  SEL_REQUIRE(njobs >= 0 && (njobs == 0 || jobs) && (dtype == SEL_BF16 || dtype == SEL_F32), SEL_ERR_ARG,
              "bad dconv pack job list");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  for (int j = 0; j < njobs; ++j) {
    const sel_dpack_job& J = jobs[j];
    SEL_REQUIRE(J.w && J.out && J.N > 0 && J.Cg > 0 && J.Kt > 0 && J.stride > 0 && J.pad >= 0 && J.G > 0 &&
                    J.N % J.G == 0 && (J.mode == 0 || J.mode == 1 || J.mode == 2),
                SEL_ERR_ARG, "bad dconv pack job %d", j);
  }
  // modes 0 / 1 from the torch weights, then the mode-2 transposes of forward
  // forms (possibly packed by the first launch: stream order)
  for (int pass = 0; pass < 2; ++pass) {
    int j = 0;
    while (j < njobs) {
      DPackJobs dj{};
      DPackTrJobs tj{};
      int n = 0, blocks = 0;
      for (; j < njobs && n < DPM_MAXJ; ++j) {
        const sel_dpack_job& J = jobs[j];
        if ((J.mode == 2) != (pass == 1)) continue;
        const PackGeo pg = pack_geo(J.N, J.Cg, J.Kt, J.stride, J.pad, J.G);
        if (pass == 0) {
          dj.pg[n] = pg;
          dj.w[n] = J.w;
          dj.wg[n] = J.wg;
          dj.out[n] = J.out;
          dj.mode[n] = J.mode;
          dj.bstart[n] = blocks;
          blocks += J.N;
        } else {
          tj.pg[n] = pg;
          tj.src[n] = J.w;
          tj.out[n] = J.out;
          tj.ntn[n] = (J.N / J.G + 63) / 64;
          tj.ntc[n] = (pg.K * J.stride * J.Cg + 63) / 64;
          tj.bstart[n] = blocks;
          blocks += J.G * tj.ntn[n] * tj.ntc[n];
        }
        ++n;
      }
      if (n == 0 || blocks == 0) continue;
      if (pass == 0) {
        dj.njobs = n;
        dj.bstart[n] = blocks;
        if (dtype == SEL_BF16)
          hipLaunchKernelGGL(k_dpack_many<__bf16>, dim3(unsigned(blocks)), dim3(256), 0, s, dj);
        else
          hipLaunchKernelGGL(k_dpack_many<float>, dim3(unsigned(blocks)), dim3(256), 0, s, dj);
      } else {
        tj.njobs = n;
        tj.bstart[n] = blocks;
        if (dtype == SEL_BF16)
          hipLaunchKernelGGL(k_dpack_tr_many<__bf16>, dim3(unsigned(blocks)), dim3(256), 0, s, tj);
        else
          hipLaunchKernelGGL(k_dpack_tr_many<float>, dim3(unsigned(blocks)), dim3(256), 0, s, tj);
      }
      SEL_LAUNCH_CHECK();
    }
  }
  return SEL_OK;
}

int sel_avgpool1d_fwd(const float* x, int B, int T, int ldx, int kernel, int stride, int pad, int To, int ldo,
                      float* y, sel_stream_t stream) {
  SEL_REQUIRE(x && y && B > 0 && T > 0 && ldx >= T && kernel > 0 && stride > 0 && ldo >= To && To > 0, SEL_ERR_ARG,
              "bad avgpool arguments");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(k_avgpool_fwd, dim3(launch_blocks(int64_t(B) * ldo)), dim3(256), 0, s, x, B, T, ldx, kernel,
                     stride, pad, To, ldo, y);
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

int sel_avgpool1d_bwd(const float* gy, int B, int T, int ldx, int kernel, int stride, int pad, int To, int ldo,
                      float* gx, sel_stream_t stream) {
  SEL_REQUIRE(gy && gx && B > 0 && T > 0 && ldx >= T && kernel > 0 && stride > 0 && ldo >= To, SEL_ERR_ARG,
              "bad avgpool arguments");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(k_avgpool_bwd, dim3(launch_blocks(int64_t(B) * ldx)), dim3(256), 0, s, gy, B, T, ldx, kernel,
                     stride, pad, To, ldo, gx);
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

int sel_mpd_fold(const float* x, int B, int T, int ldx, int period, int Lalloc, float* y, sel_stream_t stream) {
  SEL_REQUIRE(x && y && B > 0 && period > 0 && T > period && ldx >= T, SEL_ERR_ARG, "bad mpd fold arguments");
  const int L = (T + period - 1) / period;
  SEL_REQUIRE(Lalloc >= L, SEL_ERR_ARG, "Lalloc %d < L %d", Lalloc, L);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(k_mpd_fold, dim3(launch_blocks(int64_t(B) * period * Lalloc)), dim3(256), 0, s, x, B, T, ldx,
                     period, L, Lalloc, y);
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

int sel_mpd_unfold(const float* gy, int B, int T, int ldx, int period, int Lalloc, float* gx, sel_stream_t stream) {
  SEL_REQUIRE(gy && gx && B > 0 && period > 0 && T > period && ldx >= T, SEL_ERR_ARG, "bad mpd unfold arguments");
  const int L = (T + period - 1) / period;
  SEL_REQUIRE(Lalloc >= L, SEL_ERR_ARG, "Lalloc %d < L %d", Lalloc, L);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(k_mpd_unfold, dim3(launch_blocks(int64_t(B) * ldx)), dim3(256), 0, s, gy, B, T, ldx, period, L,
                     Lalloc, gx);
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

size_t sel_gan_workspace(void) { return 1024 * sizeof(double); }

int sel_gan_reduce(int kind, int dtype, const void* a, const int64_t* a_size, const int64_t* a_stride,
                   const void* b, const int64_t* b_size, const int64_t* b_stride, int ndim, float target,
                   double scale, int accumulate, float* out, void* ws, size_t ws_bytes, sel_stream_t stream) {
  SEL_REQUIRE(kind >= 0 && kind <= 4 && a && out && ndim >= 1 && ndim <= 4 && view_ok(a_size, a_stride),
              SEL_ERR_ARG, "bad gan reduce arguments");
  SEL_REQUIRE(kind != 0 || (b && view_ok(b_size, b_stride)), SEL_ERR_ARG, "L1 needs b");
  SEL_REQUIRE(ws_bytes >= sel_gan_workspace(), SEL_ERR_WORKSPACE, "workspace too small");
  int64_t n = 1;
  for (int i = 0; i < ndim; ++i) {
    n *= a_size[i];
    if (kind == 0) SEL_REQUIRE(b_size[i] == a_size[i], SEL_ERR_ARG, "shape mismatch");
  }
  SEL_REQUIRE(n < (int64_t(1) << 32), SEL_ERR_ARG, "view too large (%lld elements)", (long long)n);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const View4 va = to_view(a_size, a_stride, ndim);
  const View4 vb = kind == 0 ? to_view(b_size, b_stride, ndim) : va;
  double* part = static_cast<double*>(ws);
  const void* bb = b ? b : a;
  const bool vec = dtype == SEL_BF16 ? vec_view<__bf16>(a, va) && (kind != 0 || vec_view<__bf16>(bb, vb))
                                     : vec_view<float>(a, va) && (kind != 0 || vec_view<float>(bb, vb));
  const int vw = dtype == SEL_BF16 ? 8 : 4;
  const int64_t nt = vec ? n / vw : n;  // threads' work items
  const int nb = int(std::min<int64_t>(1024, std::max<int64_t>(1, (nt + 255) / 256)));
  if (dtype == SEL_BF16 && vec)
    hipLaunchKernelGGL(k_gan_reduce_v<__bf16>, dim3(nb), dim3(256), 0, s, kind, static_cast<const __bf16*>(a), va,
                       static_cast<const __bf16*>(bb), vb, target, uint32_t(nt), part);
  else if (dtype == SEL_BF16)
    hipLaunchKernelGGL(k_gan_reduce<__bf16>, dim3(nb), dim3(256), 0, s, kind, static_cast<const __bf16*>(a), va,
                       static_cast<const __bf16*>(bb), vb, target, n, part);
  else if (vec)
    hipLaunchKernelGGL(k_gan_reduce_v<float>, dim3(nb), dim3(256), 0, s, kind, static_cast<const float*>(a), va,
                       static_cast<const float*>(bb), vb, target, uint32_t(nt), part);
  else
    hipLaunchKernelGGL(k_gan_reduce<float>, dim3(nb), dim3(256), 0, s, kind, static_cast<const float*>(a), va,
                       static_cast<const float*>(bb), vb, target, n, part);
  hipLaunchKernelGGL(k_gan_finish, dim3(1), dim3(256), 0, s, part, nb, scale, out, accumulate);
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

int sel_gan_grad(int kind, int dtype, const void* a, const int64_t* a_size, const int64_t* a_stride, const void* b,
                 const int64_t* b_size, const int64_t* b_stride, int ndim, float target, const float* gscale,
                 float mult, void* grad, const int64_t* g_stride, int accumulate, sel_stream_t stream) {
  SEL_REQUIRE(kind >= 0 && kind <= 4 && a && grad && gscale && ndim >= 1 && ndim <= 4 && view_ok(a_size, a_stride) &&
                  g_stride,
              SEL_ERR_ARG, "bad gan grad arguments");
  SEL_REQUIRE(kind != 0 || (b && view_ok(b_size, b_stride)), SEL_ERR_ARG, "L1 needs b");
  int64_t n = 1;
  for (int i = 0; i < ndim; ++i) n *= a_size[i];
  SEL_REQUIRE(n < (int64_t(1) << 32), SEL_ERR_ARG, "view too large (%lld elements)", (long long)n);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const View4 va = to_view(a_size, a_stride, ndim);
  const View4 vb = kind == 0 ? to_view(b_size, b_stride, ndim) : va;
  const View4 vg = to_view(a_size, g_stride, ndim);
  const void* bb = b ? b : a;
  const bool vec = dtype == SEL_BF16 ? vec_view<__bf16>(a, va) && vec_view<__bf16>(grad, vg) &&
                                           (kind != 0 || vec_view<__bf16>(bb, vb))
                                     : vec_view<float>(a, va) && vec_view<float>(grad, vg) &&
                                           (kind != 0 || vec_view<float>(bb, vb));
  const int64_t nt = vec ? n / (dtype == SEL_BF16 ? 8 : 4) : n;
  const unsigned nb = unsigned(launch_blocks(nt));
  if (dtype == SEL_BF16 && vec)
    hipLaunchKernelGGL(k_gan_grad_v<__bf16>, dim3(nb), dim3(256), 0, s, kind, static_cast<const __bf16*>(a), va,
                       static_cast<const __bf16*>(bb), vb, target, uint32_t(nt), gscale, mult,
                       static_cast<__bf16*>(grad), vg, accumulate);
  else if (vec)
    hipLaunchKernelGGL(k_gan_grad_v<float>, dim3(nb), dim3(256), 0, s, kind, static_cast<const float*>(a), va,
                       static_cast<const float*>(bb), vb, target, uint32_t(nt), gscale, mult,
                       static_cast<float*>(grad), vg, accumulate);
  else if (dtype == SEL_BF16)
    hipLaunchKernelGGL(k_gan_grad<__bf16>, dim3(nb), dim3(256), 0, s, kind, static_cast<const __bf16*>(a), va,
                       static_cast<const __bf16*>(b ? b : a), vb, target, n, gscale, mult,
                       static_cast<__bf16*>(grad), vg, accumulate);
  else
    hipLaunchKernelGGL(k_gan_grad<float>, dim3(nb), dim3(256), 0, s, kind, static_cast<const float*>(a), va,
                       static_cast<const float*>(b ? b : a), vb, target, n, gscale, mult, static_cast<float*>(grad),
                       vg, accumulate);
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

}  // extern "C"
