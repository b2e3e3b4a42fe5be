// AudioDec conv stack on gfx950 (layers/conv_layer.py, models/autoencoder*/modules/*).
//
// One primitive (see include/sel.h): a stride-1, K-tap, dilated conv over
// channels-last rows, as an implicit GEMM on MFMA.
//   rows  m = (b, t)  -> GEMM M,   output channels n -> GEMM N,
//   reduction r = (tap k, in-channel c).
// A workgroup (4 waves, 2x2) owns a BM x BN output tile.  For each 32-channel
// chunk it stages the input rows [m0 - pad, m0 + BM + (K-1)*dil - pad) ONCE in
// LDS (the causal halo) and re-reads them for every tap (K-fold reuse, the
// point of the implicit GEMM), while the packed weight slice of each tap is
// staged next to it.  ELU of the input is applied while staging (fusing
// residual_unit.py:32 into the conv prologue); bias, ELU-backward multiplier
// and residual add are fused into the epilogue.
//   fp32:  v_mfma_f32_16x16x4_f32 (exact fp32, parity path)
//   bf16:  v_mfma_f32_16x16x32_bf16 with fp32 accumulation (C3 path)
// Weight gradients: split-M reduction with v_mfma_f32_16x16x4_f32 over
// LDS-staged gout/input tiles, deterministic split reduce.
#include <algorithm>

#include "sel_common.h"

namespace sel {
namespace conv {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int CK = 32;  // channels per reduction chunk

template <typename T> struct Pitch;
template <> struct Pitch<float> { static constexpr int v = 36; };   // 144 B rows: conflict-free b128
template <> struct Pitch<__bf16> { static constexpr int v = 40; };  // 80 B rows: conflict-free b128

__device__ __forceinline__ float to_f(float v) { return v; }
__device__ __forceinline__ float to_f(__bf16 v) { return float(v); }
template <typename T> __device__ __forceinline__ T from_f(float v);
template <> __device__ __forceinline__ float from_f<float>(float v) { return v; }
template <> __device__ __forceinline__ __bf16 from_f<__bf16>(float v) { return __bf16(v); }

__device__ __forceinline__ float elu(float v) { return v > 0.f ? v : expm1f(v); }
__device__ __forceinline__ float elu_grad(float v) { return v > 0.f ? 1.f : expf(v); }

struct Args {
  int64_t rows;
  int T, C, N, K, dil, pad, pad_mode, in_elu, bias_period;
};

// Flat input row for (output row m, tap k) or -1 (zero).
__device__ __forceinline__ int64_t in_row(const Args& a, int64_t m, int k) {
  const int64_t b = m / a.T;
  const int t = int(m - b * a.T);
  int ti = t + k * a.dil - a.pad;
  if (ti < 0 || ti >= a.T) {
    if (a.pad_mode == SEL_PAD_ZERO) return -1;
    ti = ti < 0 ? 0 : a.T - 1;
  }
  return b * a.T + ti;
}

// Stage `nrows` input rows starting at flat row g0 (channels [c0, c0+CK)) into LDS.
template <typename T>
__device__ __forceinline__ void stage_rows(const T* __restrict__ in, const Args& a, int64_t g0, int nrows,
                                           int c0, T* __restrict__ xs, bool elu_on) {
  constexpr int P = Pitch<T>::v;
  constexpr int VEC = 16 / sizeof(T);  // elements per 16-B load
  constexpr int PER_ROW = CK / VEC;
  const bool vec_ok = (a.C % VEC == 0) && (c0 + CK <= a.C);
  for (int idx = threadIdx.x; idx < nrows * PER_ROW; idx += blockDim.x) {
    const int r = idx / PER_ROW, v = idx % PER_ROW;
    const int64_t g = g0 + r;
    const int c = c0 + v * VEC;
    T vals[VEC];
    if (g >= 0 && g < a.rows && vec_ok) {
      const uint4 raw = *reinterpret_cast<const uint4*>(in + g * a.C + c);
      *reinterpret_cast<uint4*>(vals) = raw;
    } else {
#pragma unroll
      for (int e = 0; e < VEC; ++e)
        vals[e] = (g >= 0 && g < a.rows && c + e < a.C) ? in[g * a.C + c + e] : from_f<T>(0.f);
    }
    if (elu_on) {
#pragma unroll
      for (int e = 0; e < VEC; ++e) vals[e] = from_f<T>(elu(to_f(vals[e])));
    }
    *reinterpret_cast<uint4*>(xs + r * P + v * VEC) = *reinterpret_cast<uint4*>(vals);
  }
}

// Stage packed weights Wp[n][k][c] for n in [n0, n0+BN), one tap, channels chunk.
template <typename T, int BN>
__device__ __forceinline__ void stage_w(const T* __restrict__ wp, const Args& a, int n0, int k, int c0,
                                        T* __restrict__ ws) {
  constexpr int P = Pitch<T>::v;
  constexpr int VEC = 16 / sizeof(T);
  constexpr int PER_ROW = CK / VEC;
  const bool vec_ok = (a.C % VEC == 0) && (c0 + CK <= a.C);
  for (int idx = threadIdx.x; idx < BN * PER_ROW; idx += blockDim.x) {
    const int r = idx / PER_ROW, v = idx % PER_ROW;
    const int n = n0 + r;
    const int c = c0 + v * VEC;
    T vals[VEC];
    const int64_t base = (int64_t(n) * a.K + k) * a.C + c;
    if (n < a.N && vec_ok) {
      *reinterpret_cast<uint4*>(vals) = *reinterpret_cast<const uint4*>(wp + base);
    } else {
#pragma unroll
      for (int e = 0; e < VEC; ++e) vals[e] = (n < a.N && c + e < a.C) ? wp[base + e] : from_f<T>(0.f);
    }
    *reinterpret_cast<uint4*>(ws + r * P + v * VEC) = *reinterpret_cast<uint4*>(vals);
  }
}

// acc += A(16 rows from xs) * B(16 cols from ws) over one 32-channel chunk.
__device__ __forceinline__ void mma_chunk(floatx4& acc, const float* xs_row, const float* ws_row, int lane,
                                          bool valid) {
  // lane: row/col = lane & 15, channel group 4*(lane >> 4) (+16)
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int c = 16 * h + 4 * (lane >> 4);
    float4 av = *reinterpret_cast<const float4*>(xs_row + c);
    const float4 bv = *reinterpret_cast<const float4*>(ws_row + c);
    if (!valid) av = make_float4(0.f, 0.f, 0.f, 0.f);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av.x, bv.x, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av.y, bv.y, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av.z, bv.z, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av.w, bv.w, acc, 0, 0, 0);
  }
}
__device__ __forceinline__ void mma_chunk(floatx4& acc, const __bf16* xs_row, const __bf16* ws_row,
                                          int lane, bool valid) {
  const int c = 8 * (lane >> 4);
  bf16x8 av = *reinterpret_cast<const bf16x8*>(xs_row + c);
  const bf16x8 bv = *reinterpret_cast<const bf16x8*>(ws_row + c);
  if (!valid) av = bf16x8{};
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc, 0, 0, 0);
}

template <typename TI, typename TO, int BM, int BN>
__global__ __launch_bounds__(256) void k_conv_fwd(Args a, const TI* __restrict__ in,
                                                  const TI* __restrict__ wp,
                                                  const float* __restrict__ bias,
                                                  const TO* __restrict__ aux,
                                                  const TO* __restrict__ res, TO* __restrict__ out) {
  constexpr int P = Pitch<TI>::v;
  constexpr int TM = BM / 32, TN = BN / 32;  // 16x16 tiles per wave (2x2 waves)
  extern __shared__ __align__(16) unsigned char smem[];
  const int halo = (a.K - 1) * a.dil;
  const int span = BM + halo;
  TI* xs = reinterpret_cast<TI*>(smem);
  TI* ws = xs + span * P;

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int64_t m0 = int64_t(blockIdx.x) * BM;
  const int n0 = blockIdx.y * BN;
  const int64_t g0 = m0 - a.pad;

  floatx4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  // per-lane A rows (one per 16-row tile): local row within the block tile
  for (int c0 = 0; c0 < a.C; c0 += CK) {
    __syncthreads();
    stage_rows<TI>(in, a, g0, span, c0, xs, a.in_elu != 0);
    for (int k = 0; k < a.K; ++k) {
      if (k > 0) __syncthreads();
      stage_w<TI, BN>(wp, a, n0, k, c0, ws);
      __syncthreads();
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int lr = wm * (BM / 2) + i * 16 + (lane & 15);
        const int64_t m = m0 + lr;
        // row in xs for (m, k): in_row(m,k) - g0 ; validity from the sample bounds
        int64_t g = m < a.rows ? in_row(a, m, k) : -1;
        const bool valid = g >= 0;
        const int xr = valid ? int(g - g0) : 0;
        const TI* xrow = xs + xr * P;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int nc = wn * (BN / 2) + j * 16 + (lane & 15);
          mma_chunk(acc[i][j], xrow, ws + nc * P, lane, valid);
        }
      }
    }
  }

  // epilogue: col = lane & 15, row = 4*(lane >> 4) + e
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wn * (BN / 2) + j * 16 + (lane & 15);
      if (n >= a.N) continue;
      const float bv = (bias && a.bias_period) ? bias[n % a.bias_period] : 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int64_t m = m0 + wm * (BM / 2) + i * 16 + 4 * (lane >> 4) + e;
        if (m >= a.rows) continue;
        const int64_t o = m * a.N + n;
        float v = acc[i][j][e] + bv;
        if (aux) v *= elu_grad(to_f(aux[o]));
        if (res) v += to_f(res[o]);
        out[o] = from_f<TO>(v);
      }
    }
}

// ---------------------------------------------------------------------------
// weight gradient: gWp[n][k][c] = sum_m gout[m][n] * act(in[row(m,k)][c])
// block = (n-tile BN, c-chunk CK, m-split); all K taps per block.
// ---------------------------------------------------------------------------
constexpr int WG_BM = 64;        // m rows per staged chunk
constexpr int WG_GP = 16;        // pitch padding for fp32 LDS reads
constexpr int WG_MAXT = 16;      // max 16x16 output tiles per wave

template <typename TI, int BN>
__global__ __launch_bounds__(256) void k_conv_wgrad(Args a, const TI* __restrict__ gout,
                                                    const TI* __restrict__ in, int64_t rows_per_split,
                                                    float* __restrict__ part, float* __restrict__ bpart) {
  constexpr int GPITCH = BN + WG_GP;  // fp32
  constexpr int XPITCH = CK + WG_GP;  // fp32
  extern __shared__ __align__(16) unsigned char smem[];
  const int halo = (a.K - 1) * a.dil;
  const int span = WG_BM + halo;
  float* gs = reinterpret_cast<float*>(smem);
  float* xs = gs + WG_BM * GPITCH;

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n0 = blockIdx.x * BN;
  const int c0 = blockIdx.y * CK;
  const int split = blockIdx.z;
  const int64_t mbeg = int64_t(split) * rows_per_split;
  const int64_t mend = std::min<int64_t>(a.rows, mbeg + rows_per_split);

  // output tiles: (k, nt, ct) with nt < BN/16, ct < 2; distributed round-robin over waves
  const int ntile = a.K * (BN / 16) * 2;
  floatx4 acc[WG_MAXT];
#pragma unroll
  for (int j = 0; j < WG_MAXT; ++j) acc[j] = floatx4{0.f, 0.f, 0.f, 0.f};
  float bsum = 0.f;  // bias partial for column (threadIdx.x) when c0 == 0

  for (int64_t mc = mbeg; mc < mend; mc += WG_BM) {
    __syncthreads();
    // stage gout[mc .. mc+64) x [n0, n0+BN) as fp32
    for (int idx = threadIdx.x; idx < WG_BM * BN; idx += blockDim.x) {
      const int r = idx / BN, cc = idx % BN;
      const int64_t m = mc + r;
      const int n = n0 + cc;
      float v = 0.f;
      if (m < mend && n < a.N) v = to_f(gout[m * a.N + n]);
      gs[r * GPITCH + cc] = v;
    }
    // stage input rows [mc - pad, mc + 64 + halo - pad) channels [c0, c0+32) fp32 (+ELU)
    const int64_t g0 = mc - a.pad;
    for (int idx = threadIdx.x; idx < span * CK; idx += blockDim.x) {
      const int r = idx / CK, cc = idx % CK;
      const int64_t g = g0 + r;
      const int c = c0 + cc;
      float v = 0.f;
      if (g >= 0 && g < a.rows && c < a.C) {
        v = to_f(in[g * a.C + c]);
        if (a.in_elu) v = elu(v);
      }
      xs[r * XPITCH + cc] = v;
    }
    __syncthreads();
    if (bpart && c0 == 0 && threadIdx.x < BN) {
      for (int r = 0; r < WG_BM; ++r) bsum += gs[r * GPITCH + threadIdx.x];
    }
    // per-lane row validity / xs row for each (k): rows handled by this lane: mm = 4*q + (lane>>4)
#pragma unroll
    for (int j = 0; j < WG_MAXT; ++j) {
      const int tid = wave + 4 * j;
      if (tid >= ntile) break;
      const int k = tid / ((BN / 16) * 2);
      const int rem = tid % ((BN / 16) * 2);
      const int nt = rem >> 1, ct = rem & 1;
      const float* gcol = gs + nt * 16 + (lane & 15);
      const float* xcol = xs + ct * 16 + (lane & 15);
#pragma unroll 4
      for (int q = 0; q < WG_BM / 4; ++q) {
        const int r = 4 * q + (lane >> 4);
        const int64_t m = mc + r;
        float av = gcol[r * GPITCH];
        float bv = 0.f;
        if (m < mend) {
          const int64_t g = in_row(a, m, k);
          if (g >= 0) bv = xcol[int(g - g0) * XPITCH];
        }
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[j], 0, 0, 0);
      }
    }
  }
  // write partial tiles: part[split][n][k][c]  (C/D: col=c (lane&15), row=n (4*(lane>>4)+e))
  float* pdst = part + int64_t(split) * a.N * a.K * a.C;
#pragma unroll
  for (int j = 0; j < WG_MAXT; ++j) {
    const int tid = wave + 4 * j;
    if (tid >= ntile) break;
    const int k = tid / ((BN / 16) * 2);
    const int rem = tid % ((BN / 16) * 2);
    const int nt = rem >> 1, ct = rem & 1;
    const int c = c0 + ct * 16 + (lane & 15);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int n = n0 + nt * 16 + 4 * (lane >> 4) + e;
      if (n < a.N && c < a.C) pdst[(int64_t(n) * a.K + k) * a.C + c] = acc[j][e];
    }
  }
  if (bpart && c0 == 0 && threadIdx.x < BN && n0 + int(threadIdx.x) < a.N)
    bpart[int64_t(split) * a.N + n0 + threadIdx.x] = bsum;
}

__global__ __launch_bounds__(256) void k_split_reduce(const float* __restrict__ part, int nsplit,
                                                      int64_t n, float* __restrict__ out) {
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += int64_t(gridDim.x) * blockDim.x) {
    float s = 0.f;
    for (int p = 0; p < nsplit; ++p) s += part[int64_t(p) * n + i];
    out[i] = s;
  }
}

// bias grad: sum splits and phases: gb[j] = sum_{p, n % period == j} bpart[p][n]
__global__ void k_bias_reduce(const float* __restrict__ bpart, int nsplit, int N, int period,
                              float* __restrict__ gb) {
  for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < period; j += gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int p = 0; p < nsplit; ++p)
      for (int n = j; n < N; n += period) s += bpart[int64_t(p) * N + n];
    gb[j] = s;
  }
}

// ---------------------------------------------------------------------------
// weight packing
// ---------------------------------------------------------------------------
// strided fwd pack: Wp[co][tap][ph*Cin+ci] = W[co][ci][k(tap,ph)]
__device__ __forceinline__ int strided_k(int tap, int ph, int s) {
  if (tap == 0) return ph >= 1 ? ph - 1 : -1;
  if (tap == 1) return ph + s - 1;
  return ph == 0 ? 2 * s - 1 : -1;
}

template <typename TO>
__global__ void k_pack(int kind, const float* __restrict__ w, int cout, int cin, int K, int s,
                       TO* __restrict__ wp) {
  int64_t total;
  if (kind == SEL_PACK_FWD) total = int64_t(cout) * K * cin;
  else if (kind == SEL_PACK_FWD_STRIDED) total = int64_t(cout) * 3 * s * cin;
  else total = int64_t(s) * cout * 2 * cin;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
       i += int64_t(gridDim.x) * blockDim.x) {
    float v = 0.f;
    if (kind == SEL_PACK_FWD) {
      const int c = int(i % cin);
      const int k = int((i / cin) % K);
      const int n = int(i / (int64_t(cin) * K));
      v = w[(int64_t(n) * cin + c) * K + k];
    } else if (kind == SEL_PACK_FWD_STRIDED) {
      const int Cp = s * cin;
      const int cp = int(i % Cp);
      const int tap = int((i / Cp) % 3);
      const int n = int(i / (int64_t(Cp) * 3));
      const int ph = cp / cin, ci = cp % cin;
      const int k = strided_k(tap, ph, s);
      v = k >= 0 ? w[(int64_t(n) * cin + ci) * (2 * s) + k] : 0.f;
    } else {  // CONVT: Wp[(ph*cout+co)][tap][ci] = Wt[ci][co][tap==0 ? ph+s : ph]
      const int ci = int(i % cin);
      const int tap = int((i / cin) % 2);
      const int nn = int(i / (int64_t(cin) * 2));
      const int ph = nn / cout, co = nn % cout;
      const int k = tap == 0 ? ph + s : ph;
      v = w[(int64_t(ci) * cout + co) * (2 * s) + k];
    }
    wp[i] = from_f<TO>(v);
  }
}

template <typename T>
__global__ void k_pack_dgrad(const T* __restrict__ wp, int N, int K, int C, T* __restrict__ wd) {
  const int64_t total = int64_t(N) * K * C;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
       i += int64_t(gridDim.x) * blockDim.x) {
    // wd[c][j][n] = wp[n][K-1-j][c]
    const int n = int(i % N);
    const int j = int((i / N) % K);
    const int c = int(i / (int64_t(N) * K));
    wd[i] = wp[(int64_t(n) * K + (K - 1 - j)) * C + c];
  }
}

__global__ void k_unpack(int kind, const float* __restrict__ gp, int cout, int cin, int K, int s,
                         float* __restrict__ gw) {
  // iterate over torch-layout elements
  int64_t total = (kind == SEL_PACK_CONVT) ? int64_t(cin) * cout * 2 * s
                                           : int64_t(cout) * cin * (kind == SEL_PACK_FWD ? K : 2 * s);
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
       i += int64_t(gridDim.x) * blockDim.x) {
    float v;
    if (kind == SEL_PACK_FWD) {
      const int k = int(i % K);
      const int ci = int((i / K) % cin);
      const int co = int(i / (int64_t(K) * cin));
      v = gp[(int64_t(co) * K + k) * cin + ci];
    } else if (kind == SEL_PACK_FWD_STRIDED) {
      const int KK = 2 * s;
      const int k = int(i % KK);
      const int ci = int((i / KK) % cin);
      const int co = int(i / (int64_t(KK) * cin));
      int tap, ph;
      if (k <= s - 2) { tap = 0; ph = k + 1; }
      else if (k <= 2 * s - 2) { tap = 1; ph = k - s + 1; }
      else { tap = 2; ph = 0; }
      v = gp[(int64_t(co) * 3 + tap) * (int64_t(s) * cin) + ph * cin + ci];
    } else {
      const int KK = 2 * s;
      const int k = int(i % KK);
      const int co = int((i / KK) % cout);
      const int ci = int(i / (int64_t(KK) * cout));
      const int ph = k < s ? k : k - s;
      const int tap = k < s ? 1 : 0;
      v = gp[(int64_t(ph * cout + co) * 2 + tap) * cin + ci];
    }
    gw[i] = v;
  }
}

template <typename T>
__global__ void k_replicate_fix(Args a, const T* __restrict__ gout, const T* __restrict__ wp,
                                T* __restrict__ gin) {
  // one block per sample b, threads over c
  const int64_t b = blockIdx.x;
  const int64_t row = b * a.T;
  for (int c = threadIdx.x; c < a.C; c += blockDim.x) {
    float s = 0.f;
    for (int n = 0; n < a.N; ++n) s += to_f(gout[row * a.N + n]) * to_f(wp[(int64_t(n) * a.K + 0) * a.C + c]);
    gin[row * a.C + c] = from_f<T>(to_f(gin[row * a.C + c]) + s);
  }
}

template <typename TS, typename TD>
__global__ void k_cast(const TS* __restrict__ s, TD* __restrict__ d, int64_t n) {
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += int64_t(gridDim.x) * blockDim.x)
    d[i] = from_f<TD>(to_f(s[i]));
}

}  // namespace conv
}  // namespace sel

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
using namespace sel;
using namespace sel::conv;

namespace {

int check_desc(const sel_conv_desc* d) {
  SEL_REQUIRE(d != nullptr, SEL_ERR_ARG, "null conv descriptor");
  SEL_REQUIRE(d->rows >= 0 && d->T > 0 && d->rows % d->T == 0, SEL_ERR_ARG,
              "rows (%lld) must be a multiple of T (%d)", (long long)d->rows, d->T);
  SEL_REQUIRE(d->C > 0 && d->N > 0 && d->K > 0 && d->dil > 0 && d->pad >= 0, SEL_ERR_ARG,
              "bad conv shape C=%d N=%d K=%d dil=%d pad=%d", d->C, d->N, d->K, d->dil, d->pad);
  SEL_REQUIRE(d->pad_mode == SEL_PAD_ZERO || (d->pad_mode == SEL_PAD_REPLICATE && d->pad <= (d->K - 1) * d->dil),
              SEL_ERR_ARG, "bad pad mode");
  SEL_REQUIRE(d->bias_period >= 0 && (d->bias_period == 0 || d->N % d->bias_period == 0), SEL_ERR_ARG,
              "bias_period must divide N");
  SEL_REQUIRE((d->K - 1) * d->dil <= 512, SEL_ERR_UNSUPPORTED, "receptive halo > 512 rows");
  return SEL_OK;
}

Args to_args(const sel_conv_desc* d) {
  Args a;
  a.rows = d->rows;
  a.T = d->T;
  a.C = d->C;
  a.N = d->N;
  a.K = d->K;
  a.dil = d->dil;
  a.pad = d->pad;
  a.pad_mode = d->pad_mode;
  a.in_elu = d->in_elu;
  a.bias_period = d->bias_period;
  return a;
}

template <typename TI, typename TO, int BM, int BN>
int launch_fwd(const Args& a, const void* in, const void* wp, const float* bias, const void* aux,
               const void* res, void* out, hipStream_t s) {
  const int span = BM + (a.K - 1) * a.dil;
  const size_t lds = size_t(span + BN) * Pitch<TI>::v * sizeof(TI);
  SEL_REQUIRE(lds <= 160 * 1024, SEL_ERR_UNSUPPORTED, "conv tile needs %zu B of LDS", lds);
  dim3 grid(unsigned((a.rows + BM - 1) / BM), unsigned((a.N + BN - 1) / BN));
  if (grid.x == 0) return SEL_OK;
  auto kern = k_conv_fwd<TI, TO, BM, BN>;
  if (lds > 64 * 1024) SEL_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, int(lds)));
  hipLaunchKernelGGL(kern, grid, dim3(256), lds, s, a, static_cast<const TI*>(in),
                     static_cast<const TI*>(wp), bias, static_cast<const TO*>(aux),
                     static_cast<const TO*>(res), static_cast<TO*>(out));
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

template <typename TI, typename TO>
int dispatch_fwd(const Args& a, const void* in, const void* wp, const float* bias, const void* aux,
                 const void* res, void* out, hipStream_t s) {
  // tile choice: narrow outputs use BN=32; long thin GEMMs BM=128
  if (a.N <= 32) return launch_fwd<TI, TO, 128, 32>(a, in, wp, bias, aux, res, out, s);
  if (a.N <= 64) return launch_fwd<TI, TO, 128, 64>(a, in, wp, bias, aux, res, out, s);
  if (a.rows >= 4096) return launch_fwd<TI, TO, 128, 128>(a, in, wp, bias, aux, res, out, s);
  return launch_fwd<TI, TO, 64, 64>(a, in, wp, bias, aux, res, out, s);
}

constexpr int kWgBN = 64;

void wgrad_plan(const sel_conv_desc* d, int& nsplit, int64_t& rows_per_split) {
  const int ntiles = ((d->N + kWgBN - 1) / kWgBN) * ((d->C + CK - 1) / CK);
  int64_t chunks = (d->rows + WG_BM - 1) / WG_BM;
  int want = std::max(1, 1024 / ntiles);
  nsplit = int(std::min<int64_t>(chunks, want));
  nsplit = std::max(nsplit, 1);
  int64_t cps = (chunks + nsplit - 1) / nsplit;
  rows_per_split = cps * WG_BM;
  nsplit = int((d->rows + rows_per_split - 1) / rows_per_split);
  nsplit = std::max(nsplit, 1);
}

}  // namespace

extern "C" {

int sel_conv_fwd(const sel_conv_desc* d, int in_dtype, int out_dtype, const void* in, const void* wpack,
                 const float* bias, const void* aux, const void* res, void* out, sel_stream_t stream) {
  if (int rc = check_desc(d)) return rc;
  const Args a = to_args(d);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (in_dtype == SEL_F32 && out_dtype == SEL_F32)
    return dispatch_fwd<float, float>(a, in, wpack, bias, aux, res, out, s);
  if (in_dtype == SEL_BF16 && out_dtype == SEL_BF16)
    return dispatch_fwd<__bf16, __bf16>(a, in, wpack, bias, aux, res, out, s);
  if (in_dtype == SEL_BF16 && out_dtype == SEL_F32)
    return dispatch_fwd<__bf16, float>(a, in, wpack, bias, aux, res, out, s);
  set_error("unsupported dtype combination in=%d out=%d", in_dtype, out_dtype);
  return SEL_ERR_UNSUPPORTED;
}

size_t sel_conv_wgrad_workspace(const sel_conv_desc* d) {
  if (!d || d->rows <= 0) return 16;
  int nsplit;
  int64_t rps;
  wgrad_plan(d, nsplit, rps);
  return size_t(nsplit) * (size_t(d->N) * d->K * d->C + d->N) * sizeof(float);
}

int sel_conv_wgrad(const sel_conv_desc* d, int dtype, const void* gout, const void* in, float* gwpack,
                   float* gbias, void* ws, size_t ws_bytes, sel_stream_t stream) {
  if (int rc = check_desc(d)) return rc;
  SEL_REQUIRE(d->K * (kWgBN / 16) * 2 <= 4 * WG_MAXT, SEL_ERR_UNSUPPORTED, "wgrad: K=%d too large", d->K);
  SEL_REQUIRE(ws_bytes >= sel_conv_wgrad_workspace(d), SEL_ERR_WORKSPACE, "workspace too small");
  const Args a = to_args(d);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  int nsplit;
  int64_t rps;
  wgrad_plan(d, nsplit, rps);
  float* part = static_cast<float*>(ws);
  float* bpart = gbias ? part + size_t(nsplit) * d->N * d->K * d->C : nullptr;
  const int span = WG_BM + (d->K - 1) * d->dil;
  const size_t lds = (size_t(WG_BM) * (kWgBN + WG_GP) + size_t(span) * (CK + WG_GP)) * sizeof(float);
  SEL_REQUIRE(lds <= 160 * 1024, SEL_ERR_UNSUPPORTED, "wgrad tile needs %zu B of LDS", lds);
  dim3 grid(unsigned((d->N + kWgBN - 1) / kWgBN), unsigned((d->C + CK - 1) / CK), unsigned(nsplit));
  if (d->rows > 0) {
    if (dtype == SEL_F32) {
      auto kern = k_conv_wgrad<float, kWgBN>;
      if (lds > 64 * 1024) SEL_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, int(lds)));
      hipLaunchKernelGGL(kern, grid, dim3(256), lds, s, a, static_cast<const float*>(gout),
                         static_cast<const float*>(in), rps, part, bpart);
    } else if (dtype == SEL_BF16) {
      auto kern = k_conv_wgrad<__bf16, kWgBN>;
      if (lds > 64 * 1024) SEL_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, int(lds)));
      hipLaunchKernelGGL(kern, grid, dim3(256), lds, s, a, static_cast<const __bf16*>(gout),
                         static_cast<const __bf16*>(in), rps, part, bpart);
    } else {
      set_error("bad dtype %d", dtype);
      return SEL_ERR_ARG;
    }
    SEL_LAUNCH_CHECK();
  }
  const int64_t nw = int64_t(d->N) * d->K * d->C;
  hipLaunchKernelGGL(k_split_reduce, dim3(unsigned(std::min<int64_t>(1024, (nw + 255) / 256))), dim3(256), 0, s,
                     part, nsplit, nw, gwpack);
  SEL_LAUNCH_CHECK();
  if (gbias) {
    hipLaunchKernelGGL(k_bias_reduce, dim3(unsigned((d->bias_period + 255) / 256)), dim3(256), 0, s, bpart,
                       nsplit, d->N, d->bias_period, gbias);
    SEL_LAUNCH_CHECK();
  }
  return SEL_OK;
}

int sel_pack_weight(int kind, const float* w, int cout, int cin, int k, int stride, int dtype, void* wpack,
                    sel_stream_t stream) {
  SEL_REQUIRE(kind >= SEL_PACK_FWD && kind <= SEL_PACK_CONVT, SEL_ERR_ARG, "bad pack kind");
  SEL_REQUIRE(kind == SEL_PACK_FWD || k == 2 * stride, SEL_ERR_UNSUPPORTED,
              "strided/transposed conv needs kernel_size == 2*stride (got %d, %d)", k, stride);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int64_t total = kind == SEL_PACK_FWD ? int64_t(cout) * k * cin
                        : kind == SEL_PACK_FWD_STRIDED ? int64_t(cout) * 3 * stride * cin
                                                       : int64_t(stride) * cout * 2 * cin;
  dim3 grid(unsigned(std::min<int64_t>(4096, (total + 255) / 256)));
  if (dtype == SEL_F32)
    hipLaunchKernelGGL(k_pack<float>, grid, dim3(256), 0, s, kind, w, cout, cin, k, stride,
                       static_cast<float*>(wpack));
  else
    hipLaunchKernelGGL(k_pack<__bf16>, grid, dim3(256), 0, s, kind, w, cout, cin, k, stride,
                       static_cast<__bf16*>(wpack));
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

int sel_pack_dgrad(const void* wpack, int N, int K, int C, int dtype, void* wd, sel_stream_t stream) {
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int64_t total = int64_t(N) * K * C;
  dim3 grid(unsigned(std::min<int64_t>(4096, (total + 255) / 256)));
  if (dtype == SEL_F32)
    hipLaunchKernelGGL(k_pack_dgrad<float>, grid, dim3(256), 0, s, static_cast<const float*>(wpack), N, K, C,
                       static_cast<float*>(wd));
  else
    hipLaunchKernelGGL(k_pack_dgrad<__bf16>, grid, dim3(256), 0, s, static_cast<const __bf16*>(wpack), N, K,
                       C, static_cast<__bf16*>(wd));
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

int sel_unpack_wgrad(int kind, const float* gwpack, int cout, int cin, int k, int stride, float* gw,
                     sel_stream_t stream) {
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int64_t total = int64_t(cout) * cin * (kind == SEL_PACK_FWD ? k : 2 * stride);
  dim3 grid(unsigned(std::min<int64_t>(4096, (total + 255) / 256)));
  hipLaunchKernelGGL(k_unpack, grid, dim3(256), 0, s, kind, gwpack, cout, cin, k, stride, gw);
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

int sel_conv_replicate_fix(const sel_conv_desc* d, int dtype, const void* gout, const void* wpack, void* gin,
                           sel_stream_t stream) {
  if (int rc = check_desc(d)) return rc;
  const Args a = to_args(d);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const unsigned nb = unsigned(d->rows / d->T);
  if (nb == 0) return SEL_OK;
  if (dtype == SEL_F32)
    hipLaunchKernelGGL(k_replicate_fix<float>, dim3(nb), dim3(256), 0, s, a, static_cast<const float*>(gout),
                       static_cast<const float*>(wpack), static_cast<float*>(gin));
  else
    hipLaunchKernelGGL(k_replicate_fix<__bf16>, dim3(nb), dim3(256), 0, s, a, static_cast<const __bf16*>(gout),
                       static_cast<const __bf16*>(wpack), static_cast<__bf16*>(gin));
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

int sel_cast(const void* src, int src_dtype, void* dst, int dst_dtype, int64_t n, sel_stream_t stream) {
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (n <= 0) return SEL_OK;
  dim3 grid(unsigned(std::min<int64_t>(8192, (n + 255) / 256)));
  if (src_dtype == SEL_F32 && dst_dtype == SEL_BF16)
    hipLaunchKernelGGL((k_cast<float, __bf16>), grid, dim3(256), 0, s, static_cast<const float*>(src),
                       static_cast<__bf16*>(dst), n);
  else if (src_dtype == SEL_BF16 && dst_dtype == SEL_F32)
    hipLaunchKernelGGL((k_cast<__bf16, float>), grid, dim3(256), 0, s, static_cast<const __bf16*>(src),
                       static_cast<float*>(dst), n);
  else {
    set_error("unsupported cast %d -> %d", src_dtype, dst_dtype);
    return SEL_ERR_UNSUPPORTED;
  }
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

}  // extern "C"
