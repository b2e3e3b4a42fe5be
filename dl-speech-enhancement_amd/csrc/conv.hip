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

#include "conv_common.h"

namespace sel {
namespace conv {


constexpr int CK = 32;  // channels per reduction chunk

template <typename T> struct Pitch;
template <> struct Pitch<float> { static constexpr int v = 36; };   // 144 B rows: conflict-free b128
template <> struct Pitch<__bf16> { static constexpr int v = 40; };  // 80 B rows: conflict-free b128



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

template <typename T> struct Vec16;
template <> struct Vec16<float> { static constexpr int n = 4; };
template <> struct Vec16<__bf16> { static constexpr int n = 8; };

// Forward primitive.  Per 32-channel chunk: stage the input rows (with halo) and
// the packed weights of ALL K taps once, one barrier pair, then K x TM x TN MFMAs
// per wave.  Epilogue goes through LDS so every lane stores/loads 16 B vectors.
template <typename TI, typename TO, int BM, int BN>
__global__ __launch_bounds__(256) void k_conv_fwd(Args a, const TI* __restrict__ in,
                                                  const TI* __restrict__ wp,
                                                  const float* __restrict__ bias,
                                                  const TO* __restrict__ aux,
                                                  const TO* __restrict__ res, TO* __restrict__ out) {
  constexpr int P = Pitch<TI>::v;
  constexpr int TM = BM / 32, TN = BN / 32;  // 16x16 tiles per wave (2x2 waves)
  constexpr int OP = BN + 4;                 // fp32 epilogue tile pitch
  extern __shared__ __align__(16) unsigned char smem[];
  const int halo = (a.K - 1) * a.dil;
  const int span = BM + halo;
  TI* xs = reinterpret_cast<TI*>(smem);
  TI* ws = xs + span * P;  // [K][BN][P]

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int64_t m0 = int64_t(blockIdx.x) * BM;
  const int n0 = blockIdx.y * BN;
  const int64_t g0 = m0 - a.pad;

  // per-lane output rows: local row and time index inside its sample
  int lr[TM], tt[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    lr[i] = wm * (BM / 2) + i * 16 + (lane & 15);
    const int64_t m = m0 + lr[i];
    tt[i] = m < a.rows ? int(m % a.T) : -(1 << 30);
  }

  floatx4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  for (int c0 = 0; c0 < a.C; c0 += CK) {
    __syncthreads();
    stage_rows<TI>(in, a, g0, span, c0, xs, a.in_elu != 0);
    for (int k = 0; k < a.K; ++k) stage_w<TI, BN>(wp, a, n0, k, c0, ws + k * BN * P);
    __syncthreads();
    for (int k = 0; k < a.K; ++k) {
      const TI* wk = ws + k * BN * P;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        int ti = tt[i] + k * a.dil - a.pad;
        bool valid = ti >= 0 && ti < a.T;
        int xr = lr[i] + k * a.dil;
        if (!valid && a.pad_mode == SEL_PAD_REPLICATE && tt[i] >= 0) {
          const int tc = ti < 0 ? 0 : a.T - 1;
          xr = lr[i] + a.pad + tc - tt[i];
          valid = true;
        }
        const TI* xrow = xs + (valid ? xr : 0) * P;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int nc = wn * (BN / 2) + j * 16 + (lane & 15);
          mma_chunk(acc[i][j], xrow, wk + nc * P, lane, valid);
        }
      }
    }
  }

  // epilogue: accumulators -> LDS (fp32) -> 16-B vectors with bias / ELU' / residual
  __syncthreads();
  float* ot = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = wn * (BN / 2) + j * 16 + (lane & 15);
#pragma unroll
      for (int e = 0; e < 4; ++e) ot[(wm * (BM / 2) + i * 16 + 4 * (lane >> 4) + e) * OP + col] = acc[i][j][e];
    }
  __syncthreads();
  constexpr int V = Vec16<TO>::n;
  const bool vec_ok = (a.N % V) == 0;
  for (int idx = threadIdx.x; idx < BM * (BN / V); idx += blockDim.x) {
    const int r = idx / (BN / V), cv = (idx % (BN / V)) * V;
    const int64_t m = m0 + r;
    const int n = n0 + cv;
    if (m >= a.rows || n >= a.N) continue;
    const int64_t o = m * a.N + n;
    float v[V];
#pragma unroll
    for (int e = 0; e < V; ++e) {
      const int ne = n + e;
      const float bv = (bias && a.bias_period && ne < a.N) ? bias[ne % a.bias_period] : 0.f;
      v[e] = ot[r * OP + cv + e] + bv;
    }
    if (vec_ok) {
      if (aux) {
        TO av[V];
        *reinterpret_cast<uint4*>(av) = *reinterpret_cast<const uint4*>(aux + o);
#pragma unroll
        for (int e = 0; e < V; ++e) v[e] *= elu_grad(to_f(av[e]));
      }
      if (res) {
        TO rv[V];
        *reinterpret_cast<uint4*>(rv) = *reinterpret_cast<const uint4*>(res + o);
#pragma unroll
        for (int e = 0; e < V; ++e) v[e] += to_f(rv[e]);
      }
      TO ov[V];
#pragma unroll
      for (int e = 0; e < V; ++e) ov[e] = from_f<TO>(v[e]);
      *reinterpret_cast<uint4*>(out + o) = *reinterpret_cast<uint4*>(ov);
    } else {
      for (int e = 0; e < V && n + e < a.N; ++e) {
        float x = v[e];
        if (aux) x *= elu_grad(to_f(aux[o + e]));
        if (res) x += to_f(res[o + e]);
        out[o + e] = from_f<TO>(x);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// fp32 forward primitive on sample-aligned tiles (the reference-precision path;
// also every fp32 dgrad, as the forward of the adjoint descriptor).  BM x BN
// output tile, 4 waves of (BM / WM) x 32, v_mfma_f32_16x16x4_f32.  Per
// 16-channel chunk the input span (tile + halo, ELU applied once, zero- or
// replicate-filled per sample: no masks in the MFMA loop) and the weights of
// all K taps are staged in LDS (80-B rows: conflict-free 16-B fragment reads;
// 16 instead of 32 channels keeps the K = 7 stage at 46 KB, 3 workgroups per
// CU, where the generic kernel's 82 KB allowed one), and the next chunk's
// rows and weights are fetched into registers (16-B loads) during this
// chunk's MFMAs.  Epilogue as k_conv_fwd (bias, ELU'(aux), residual, in that
// order) through an fp32 LDS tile.
constexpr int FF_CK = 16, FF_P = 20, FF_HALO = 64;
// v or zeros, component-wise (a ternary on the float4 struct makes hipcc select
// between two ADDRESSES: both operands go to scratch memory)
__device__ __forceinline__ float4 keep4(bool ok, const float4& v) {
  return make_float4(ok ? v.x : 0.f, ok ? v.y : 0.f, ok ? v.z : 0.f, ok ? v.w : 0.f);
}
template <int BM, int BN>
constexpr int ff_xv() { return ((BM + FF_HALO) * (FF_CK / 4) + 255) / 256; }
template <int KM, int BM, int BN>
__global__ __launch_bounds__(256) void k_conv_fwd_f32(Args a, const float* __restrict__ in,
                                                      const float* __restrict__ wp, const float* __restrict__ bias,
                                                      const float* __restrict__ aux, const float* __restrict__ res,
                                                      float* __restrict__ out) {
  constexpr int WN = BN / 32, WM = 4 / WN, TM = BM / WM / 16, TN = 2;
  constexpr int XV = ff_xv<BM, BN>();
  constexpr int WV = (KM * BN * (FF_CK / 4) + 255) / 256;
  extern __shared__ __align__(16) unsigned char smem[];
  float* const xs = reinterpret_cast<float*>(smem);      // [BM + halo][FF_P]
  float* const ws = xs + (BM + FF_HALO) * FF_P;          // [K][BN][FF_P]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int tps = (a.T + BM - 1) / BM;
  const int64_t b = blockIdx.x / tps;
  const int t0 = int(blockIdx.x - b * tps) * BM;
  const int n0 = blockIdx.y * BN;
  const int span = BM + (a.K - 1) * a.dil;
  const float* __restrict__ xb = in + b * a.T * int64_t(a.C);

  // raw loads and their predicates: the zero select happens in put(), after
  // the next chunk's MFMAs (a select right behind a load waits for it)
  floatx4 xr[XV], wr[WV];
  bool xok[XV];
  auto fetch = [&](int c0) {
#pragma unroll
    for (int u = 0; u < XV; ++u) {
      const int v = tid + u * 256;
      const int r = v >> 2, c = c0 + (v & 3) * 4;
      int ti = t0 - a.pad + r;
      bool ok = r < span;
      if (ti < 0 || ti >= a.T) {
        if (a.pad_mode == SEL_PAD_ZERO) ok = false;
        ti = ti < 0 ? 0 : a.T - 1;
      }
      // unconditional load of a clamped (valid) row: a load under a
      // per-element condition becomes a branch with its own vmcnt(0) wait
      xr[u] = *reinterpret_cast<const floatx4*>(xb + int64_t(ti) * a.C + c);
      xok[u] = ok;
    }
#pragma unroll
    for (int u = 0; u < WV; ++u) {
      const int v = tid + u * 256;
      const int q = v & 3, row = v >> 2;  // row = k * BN + n
      const int k = row / BN, n = row % BN;
      const int kc = k < a.K ? k : a.K - 1;  // taps past K: never stored
      wr[u] = *reinterpret_cast<const floatx4*>(wp + (int64_t(n0 + n) * a.K + kc) * a.C + c0 + 4 * q);
    }
  };
  auto put = [&]() {
#pragma unroll
    for (int u = 0; u < XV; ++u) {
      const int v = tid + u * 256;
      const int r = v >> 2;
      const bool ok = xok[u];
      floatx4 x = floatx4{ok ? xr[u][0] : 0.f, ok ? xr[u][1] : 0.f, ok ? xr[u][2] : 0.f, ok ? xr[u][3] : 0.f};
      if (a.in_elu) x = floatx4{elu(x[0]), elu(x[1]), elu(x[2]), elu(x[3])};
      if (r < BM + FF_HALO) *reinterpret_cast<floatx4*>(xs + r * FF_P + (v & 3) * 4) = x;
    }
#pragma unroll
    for (int u = 0; u < WV; ++u) {
      const int v = tid + u * 256;
      // (the stage holds K, not KM, taps)
      if ((v >> 2) < a.K * BN) *reinterpret_cast<floatx4*>(ws + (v >> 2) * FF_P + (v & 3) * 4) = wr[u];
    }
  };

  floatx4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  const int arow = wm * (BM / WM) + (lane & 15);
  const int g4 = 4 * (lane >> 4);
  fetch(0);
  for (int c0 = 0; c0 < a.C; c0 += FF_CK) {
    __syncthreads();  // every wave is done with the previous chunk
    put();
    __syncthreads();
    if (c0 + FF_CK < a.C) fetch(c0 + FF_CK);
    for (int k = 0; k < a.K; ++k) {
      float4 av[TM], bv[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) av[i] = *reinterpret_cast<const float4*>(xs + (arow + 16 * i + k * a.dil) * FF_P + g4);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bv[j] = *reinterpret_cast<const float4*>(ws + (k * BN + wn * 32 + 16 * j + (lane & 15)) * FF_P + g4);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i].x, bv[j].x, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i].y, bv[j].y, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i].z, bv[j].z, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i].w, bv[j].w, acc[i][j], 0, 0, 0);
        }
    }
  }
  // epilogue: accumulators -> LDS (fp32) -> 16-B vectors with bias / ELU' / residual
  constexpr int OP = BN + 4;
  __syncthreads();
  float* ot = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = wn * 32 + j * 16 + (lane & 15);
#pragma unroll
      for (int e = 0; e < 4; ++e) ot[(wm * (BM / WM) + i * 16 + g4 + e) * OP + col] = acc[i][j][e];
    }
  __syncthreads();
  const int mrows = a.T - t0 < BM ? a.T - t0 : BM;
  for (int idx = tid; idx < BM * (BN / 4); idx += 256) {
    const int r = idx / (BN / 4), cv = (idx % (BN / 4)) * 4;
    if (r >= mrows) continue;
    const int64_t o = (b * a.T + t0 + r) * a.N + n0 + cv;
    float v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int ne = n0 + cv + e;
      const float bv = (bias && a.bias_period) ? bias[ne % a.bias_period] : 0.f;
      v[e] = ot[r * OP + cv + e] + bv;
    }
    if (aux) {
      const float4 av = *reinterpret_cast<const float4*>(aux + o);
      v[0] *= elu_grad(av.x), v[1] *= elu_grad(av.y), v[2] *= elu_grad(av.z), v[3] *= elu_grad(av.w);
    }
    if (res) {
      const float4 rv = *reinterpret_cast<const float4*>(res + o);
      v[0] += rv.x, v[1] += rv.y, v[2] += rv.z, v[3] += rv.w;
    }
    *reinterpret_cast<float4*>(out + o) = make_float4(v[0], v[1], v[2], v[3]);
  }
}

// ---------------------------------------------------------------------------
// bf16 forward primitive (the hot one).  Per 32-channel chunk the input rows
// [m0 - pad, m0 + BM + (K-1)*dil - pad) are staged ONCE (ELU applied once per
// element) together with the packed weights of all K taps; the K taps then
// re-read the staged rows at shifted offsets (implicit GEMM).  The next
// chunk's rows/weights are fetched into registers while the current chunk's
// MFMAs run (T14 issue-early / write-late), and all global loads are branch-free
// (clamped address + select; requires C % 32 == 0) so hipcc emits no per-element
// fallback waits.  MFMA: v_mfma_f32_32x32x16_bf16; staged rows are 80 B apart,
// which makes its 16-B fragment reads bank-conflict free.
// ---------------------------------------------------------------------------
// residual-unit kernels' occupancy targets (waves per SIMD the register
// allocation must allow)
#ifndef SEL_W_RU32F
#define SEL_W_RU32F 3
#endif
#ifndef SEL_W_RU32F128
#define SEL_W_RU32F128 4
#endif
#ifndef SEL_W_RU32B
#define SEL_W_RU32B 3
#endif
#ifndef SEL_W_RU32W
#define SEL_W_RU32W 2
#endif
#ifndef SEL_W_RU64F
#define SEL_W_RU64F 2
#endif
#ifndef SEL_W_RU64B
#define SEL_W_RU64B 2
#endif
constexpr int F4_P = 40;  // staged row pitch (bf16 elements) = 80 B


template <int BM, int BN, int WAVES_M, int KMAX, typename TO>
__global__ __launch_bounds__(256) void k_conv_fwd_bf16(Args a, const __bf16* __restrict__ in,
                                                       const __bf16* __restrict__ wp,
                                                       const float* __restrict__ bias,
                                                       const TO* __restrict__ aux, const TO* __restrict__ res,
                                                       TO* __restrict__ out, int ncol) {
  constexpr int P = F4_P;
  constexpr int WAVES_N = 4 / WAVES_M;
  constexpr int WTM = BM / WAVES_M, WTN = BN / WAVES_N;
  constexpr int TM = WTM / 32, TN = WTN / 32;
  constexpr int XV = ((BM + F4_HALOMAX) * 4 + 255) / 256;
  constexpr int WV = (KMAX * BN * 4 + 255) / 256;
  extern __shared__ __align__(16) unsigned char smem[];
  __bf16* const xs = reinterpret_cast<__bf16*>(smem);
  const int halo = (a.K - 1) * a.dil;
  const int span = BM + halo;
  __bf16* const ws = xs + span * P;  // [k][BN][P]

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  // sample-aligned tiles: every output row of the block belongs to sample b, so
  // the causal zero / replicate padding is resolved once while staging and the
  // MFMA loop needs no per-tap row validity (blocks past T are clipped at store)
  const int tps = (a.T + BM - 1) / BM;
  int64_t mt;
  int nt;
  xcd_tile(ncol, mt, nt);
  const int64_t b = mt / tps;
  const int t0 = int(mt % tps) * BM;
  const int64_t m0 = b * a.T + t0;
  const int mrows = a.T - t0 < BM ? a.T - t0 : BM;
  const int n0 = nt * BN;
  const int nchunk = a.C / CK;

  // staging row r <-> input time t0 - pad + r of sample b; per-thread source
  // pointers computed once (chunks only add the channel offset)
  const __bf16* xsrc[XV];
  bool xok[XV];
#pragma unroll
  for (int u = 0; u < XV; ++u) {
    const int r = (tid + u * 256) >> 2;
    int ti = t0 - a.pad + r;
    const bool inside = ti >= 0 && ti < a.T;
    xok[u] = r < span && (inside || a.pad_mode == SEL_PAD_REPLICATE);
    ti = ti < 0 ? 0 : (ti >= a.T ? a.T - 1 : ti);
    xsrc[u] = in + (b * a.T + ti) * a.C + ((tid + u * 256) & 3) * 8;
  }
  const __bf16* wsrc[WV];
  bool wok[WV];
#pragma unroll
  for (int u = 0; u < WV; ++u) {
    const int v = tid + u * 256;
    const int k = v / (BN * 4), n = (v >> 2) % BN;
    const bool ok = k < a.K && n0 + n < a.N;
    wok[u] = ok;
    wsrc[u] = wp + (int64_t(ok ? n0 + n : 0) * a.K + (ok ? k : 0)) * a.C + (v & 3) * 8;
  }
  uint4 xr[XV], wr[WV];
  auto load = [&](int c0) {
#pragma unroll
    for (int u = 0; u < XV; ++u) xr[u] = *reinterpret_cast<const uint4*>(xsrc[u] + c0);  // masked in store()
#pragma unroll
    for (int u = 0; u < WV; ++u) wr[u] = *reinterpret_cast<const uint4*>(wsrc[u] + c0);
  };
  auto store = [&]() {
#pragma unroll
    for (int u = 0; u < XV; ++u) {
      const int v = tid + u * 256;
      if ((v >> 2) >= span) continue;
      // zero-fill AFTER the wait: masking right at the load would make hipcc wait
      // on the load there (vmcnt(0)) and serialise the register prefetch
      uint4 val = xok[u] ? xr[u] : make_uint4(0, 0, 0, 0);
      if (a.in_elu) {
        val = elu8(val);
      }
      *reinterpret_cast<uint4*>(xs + (v >> 2) * P + (v & 3) * 8) = val;
    }
#pragma unroll
    for (int u = 0; u < WV; ++u) {
      const int v = tid + u * 256;
      const int k = v / (BN * 4), n = (v >> 2) % BN;
      const uint4 val = wok[u] ? wr[u] : make_uint4(0, 0, 0, 0);
      if (k < a.K) *reinterpret_cast<uint4*>(ws + (k * BN + n) * P + (v & 3) * 8) = val;
    }
  };

  // per-lane output row of each 32-row tile -> its staged-row offset
  int lr[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) lr[i] = (wm * WTM + i * 32 + (lane & 31)) * P;

  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  load(0);
  for (int ch = 0; ch < nchunk; ++ch) {
    if (ch) __syncthreads();
    store();
    __syncthreads();
    if (ch + 1 < nchunk) load((ch + 1) * CK);
    for (int k = 0; k < a.K; ++k) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {  // two K=16 halves of the 32-channel chunk
        const int co = 16 * h + 8 * (lane >> 5);
        bf16x8 bf[TN];
#pragma unroll
        for (int j = 0; j < TN; ++j)
          bf[j] = *reinterpret_cast<const bf16x8*>(ws + (k * BN + wn * WTN + j * 32 + (lane & 31)) * P + co);
        const int kofs = k * a.dil * P + co;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const bf16x8 af = *reinterpret_cast<const bf16x8*>(xs + lr[i] + kofs);
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bf[j], af, acc[i][j], 0, 0, 0);
        }
      }
    }
  }

  // epilogue straight from the accumulators (operands were swapped, so C/D is
  // out^T): lane -> output row m = lane & 31 of its 32-row tile, element r ->
  // n = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5): four runs of 4 consecutive
  // channels, each stored as one 8-B (bf16) / 16-B (fp32) vector.
  const bool bias_vec = bias && a.bias_period && (a.bias_period % 4) == 0;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int r = wm * WTM + i * 32 + (lane & 31);
    if (r >= mrows) continue;
    const int64_t m = m0 + r;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int n = n0 + wn * WTN + j * 32 + 8 * g + 4 * (lane >> 5);
        if (n >= a.N) continue;
        const int64_t o = m * a.N + n;
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = acc[i][j][4 * g + e];
        if (bias_vec) {
          const float4 bv = *reinterpret_cast<const float4*>(bias + (n % a.bias_period));
          v[0] += bv.x, v[1] += bv.y, v[2] += bv.z, v[3] += bv.w;
        } else if (bias && a.bias_period) {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (n + e < a.N) v[e] += bias[(n + e) % a.bias_period];
        }
        if (a.N % 4 == 0) {
          if (aux) {
            TO av[4];
            if constexpr (sizeof(TO) == 2) *reinterpret_cast<uint2*>(av) = *reinterpret_cast<const uint2*>(aux + o);
            else *reinterpret_cast<uint4*>(av) = *reinterpret_cast<const uint4*>(aux + o);
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] *= elu_grad_fast(to_f(av[e]));
          }
          if (res) {
            TO rv[4];
            if constexpr (sizeof(TO) == 2) *reinterpret_cast<uint2*>(rv) = *reinterpret_cast<const uint2*>(res + o);
            else *reinterpret_cast<uint4*>(rv) = *reinterpret_cast<const uint4*>(res + o);
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] += to_f(rv[e]);
          }
          TO ov[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) ov[e] = from_f<TO>(v[e]);
          if constexpr (sizeof(TO) == 2) *reinterpret_cast<uint2*>(out + o) = *reinterpret_cast<uint2*>(ov);
          else *reinterpret_cast<uint4*>(out + o) = *reinterpret_cast<uint4*>(ov);
        } else {
          for (int e = 0; e < 4 && n + e < a.N; ++e) {
            float x = v[e];
            if (aux) x *= elu_grad_fast(to_f(aux[o + e]));
            if (res) x += to_f(res[o + e]);
            out[o + e] = from_f<TO>(x);
          }
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Warp-specialised bf16 forward for the wide layers at few rows (256 output
// channels at T = 400 x 64 clips: the RU256 k7 forwards and dgrads, the
// 640 -> 256 phase-view strided conv).  The tiled kernel above runs those at
// 2 waves per SIMD with staging (ELU + LDS stores) and MFMAs in separate
// barrier phases: SQ counters show the matrix pipe busy 28% of the kernel and
// ~3,700 VALU instructions per wave, as many issue cycles as its MFMAs
// (profiles/r2_ws_conv.md).  Here one 256 x 128 tile per CU, 12 waves:
//   waves 0-7  consumers: 4 x 2 grid of 64 x 64 wave tiles; per 16-channel
//              chunk K taps x 4 MFMAs, the next tap's fragments read while the
//              current tap's MFMAs run;
//   waves NC..NC+3 producers: global -> LDS DMA (global_load_lds_dwordx4) of the
//              input span and the K weight slices three chunks ahead into a
//              4-slot LDS ring, then the input ELU in place one chunk ahead;
//   all 12:    the epilogue, through an fp32 LDS tile with row-contiguous 16-B
//              global accesses.
// One barrier per chunk.  LDS rows are 32 B (16 channels) with the 16-B slot
// XOR-swizzled by row bit 3 (conflict-free ds_read_b128 for both MFMA operands);
// the DMA destination is lane-linear, so the swizzle is applied to the SOURCE
// address.  Padding rows are DMA'd from a zero buffer.
// Measured limits (block stamps, tools/ws_probe.py): consumers alone run the
// main loop at ~75% of the MFMA pipe (2.1 GHz); the producers' DMA into LDS
// costs the consumers ~900 cycles per chunk and lowers the clock to ~1.87 GHz,
// the in-place ELU ~3 us per launch; one wave of 256 tiles leaves the prologue
// and the epilogue (~2 us fwd, ~4 us with aux + res) exposed.
// ---------------------------------------------------------------------------
constexpr int WS_BM = 256, WS_BN = 128, WS_CK = 16, WS_NBUF = 4;
constexpr int WS_RPI = 1024 / (WS_CK * 2);    // LDS rows per 1-KB DMA piece
constexpr int WS_SPR = WS_CK / 8;             // 16-B slots per LDS row
constexpr int WS_XROWS = WS_BM + F4_HALOMAX;  // staged input rows per chunk (multiple of WS_RPI)
constexpr int WS_CMAX = 4096;                 // input channels the zero source covers
constexpr int WS_EP = WS_BN + 4;              // fp32 epilogue tile pitch (conflict-free 16-B writes)

__device__ __attribute__((aligned(64))) __bf16 g_ws_zero[WS_CMAX];

// XOR pattern of LDS row `row`'s 16-B slots: conflict-free ds_read_b128 of 16
// consecutive rows per lane group for both row widths (brute-force checked)
__device__ __forceinline__ int ws_swzbits(int row) { return WS_CK == 16 ? (row >> 3) & 1 : (row >> 2) & 3; }
// element offset of 16-B slot `slot` of LDS row `row` (WS_CK channels)
__device__ __forceinline__ int ws_swz(int row, int slot) { return row * WS_CK + ((slot ^ ws_swzbits(row)) << 3); }

inline size_t ws_buf_bytes(int K) { return (size_t(WS_XROWS) + size_t(K) * WS_BN) * WS_CK * 2; }
// CPB chunks per barrier: the ring has 4 * CPB slots and slots free CPB at a time
inline size_t ws_lds_bytes(int K, int cpb = 1) {
  return std::max(size_t(WS_NBUF) * cpb * ws_buf_bytes(K), size_t(WS_BM) * WS_EP * sizeof(float));
}



// DMA piece of producer wave pw's u-th slot: q = 4u + pw, clamped to the last piece
template <int TI>
__device__ __forceinline__ int ws_piece(int u, int pw) {
  return u * 4 + pw < TI ? u * 4 + pw : TI - 1;
}

// In-place input ELU of producer wave pw's input pieces (q = 4u + pw < XI) of
// one ring slot: each lane rewrites exactly the 16 B its own DMA wrote, so this
// wave's vmcnt wait alone orders it (elementwise, so the swizzle does not
// matter).  Inline-asm LDS access: hipcc would put vmcnt(0) before a plain LDS
// read while DMAs are in flight, draining the next chunk's prefetch too.
template <int PW>
__device__ __forceinline__ void ws_elu_pieces(unsigned char* lane_base, int pw, int xi) {
#pragma unroll
  for (int u = 0; u < PW; ++u) {
    const int q = u * 4 + pw;
    if (q >= xi) break;
    const unsigned addr = unsigned(reinterpret_cast<uintptr_t>(lane_base + q * 1024));
    bf16x8 val;
    asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(val) : "v"(addr) : "memory");
    val = __builtin_bit_cast(bf16x8, elu8(__builtin_bit_cast(uint4, val)));
    asm volatile("ds_write_b128 %0, %1" : : "v"(addr), "v"(val) : "memory");
  }
}

template <int KT, typename TO, int NC, int CPB>
__global__ __launch_bounds__((NC + 4) * 64) void k_conv_ws_bf16(Args a, const __bf16* __restrict__ in,
                                                      const __bf16* __restrict__ wp,
                                                      const float* __restrict__ bias, const TO* __restrict__ aux,
                                                      const TO* __restrict__ res, TO* __restrict__ out, int ncol,
                                                      int dbg) {
  constexpr int BM = WS_BM, BN = WS_BN;
  // NC consumer waves as 4 x 2 (64 x 64 each) or 2 x 2 (128 x 64: six fragment
  // reads per eight MFMAs instead of four per four)
  static_assert(NC == 8 || NC == 4, "consumer waves");
  constexpr int NT = (NC + 4) * 64;
  constexpr int TM = 16 / NC, TN = 2, WTM = 32 * TM, WTN = 64;
  constexpr int XI = WS_XROWS / WS_RPI;  // DMA pieces (1 KB) per chunk: input span
  constexpr int WI = KT * BN / WS_RPI;   // weight slices
  constexpr int TI = XI + WI;
  constexpr int PW = (TI + 3) / 4;   // per producer wave (the last one repeats its final piece)
  constexpr int BUF = (WS_XROWS + KT * BN) * WS_CK;  // bf16 elements per ring slot
  extern __shared__ __align__(16) unsigned char smem[];
  __bf16* const lds = reinterpret_cast<__bf16*>(smem);
  const int halo = (KT - 1) * a.dil;
  const int span = BM + halo;

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // diagnostic (tune key 13 bit 3): per-block start / end stamps (100 MHz
  // realtime) and hardware ids into the output buffer instead of results
  const uint64_t t_start = (dbg & 8) ? __builtin_amdgcn_s_memrealtime() : 0;
  const uint64_t c_start = (dbg & 8) ? __builtin_amdgcn_s_memtime() : 0;
  uint64_t t_loop = 0;
  const int tps = (a.T + BM - 1) / BM;
  int64_t mt;
  int nt;
  xcd_tile(ncol, mt, nt);
  const int64_t b = mt / tps;
  const int t0 = int(mt % tps) * BM;
  const int64_t m0 = b * a.T + t0;
  const int mrows = a.T - t0 < BM ? a.T - t0 : BM;
  const int n0 = nt * BN;
  const int nchunk = a.C / WS_CK;

  if (wave >= NC) {
    // ---------------- producers ----------------
    const int pw = wave - NC;
    // DMA piece q (1 KB) goes to producer wave q % 4 (the input pieces, which
    // get the ELU pass, spread over all four); a wave short of PW repeats its last
    const __bf16* src[PW];
#pragma unroll
    for (int u = 0; u < PW; ++u) {
      const int q = ws_piece<TI>(u, pw);
      if (q < XI) {
        const int R = q * WS_RPI + lane / WS_SPR, ls = (lane % WS_SPR) ^ ws_swzbits(R);
        int ti = t0 - a.pad + R;
        const bool valid =
            R < span && (a.seq_pitch > 0 ? ti >= 0 && ti < a.T && ti % a.seq_pitch < a.tin_valid
                                         : (ti >= 0 && ti < a.tin_valid) || a.pad_mode == SEL_PAD_REPLICATE);
        // flat tiling: ti is a row of the whole row space (b == 0) and `valid`
        // already keeps it in range; only the per-sequence form clamps into
        // the sequence (replicate pad)
        if (a.seq_pitch == 0) ti = ti < 0 ? 0 : (ti >= a.tin_valid ? a.tin_valid - 1 : ti);
        src[u] = valid ? in + (b * a.tin_pitch + ti) * a.ldx + 8 * ls : g_ws_zero + 8 * ls;
      } else {
        const int R = (q - XI) * WS_RPI + lane / WS_SPR, ls = (lane % WS_SPR) ^ ws_swzbits(R);
        const int k = R / BN, n = R % BN;
        src[u] = wp + (int64_t(n0 + n) * KT + k) * a.C + 8 * ls;
      }
    }
    auto issue = [&](int ch) {
      unsigned char* const base = smem + (ch % (WS_NBUF * CPB)) * (BUF * 2);
#pragma unroll
      for (int u = 0; u < PW; ++u) {
        const int q = ws_piece<TI>(u, pw);
        if ((dbg & 32) && q < XI) continue;   // diagnostic: no input DMA (tune key 13 bit 5)
        if ((dbg & 64) && q >= XI) continue;  // diagnostic: no weight DMA (tune key 13 bit 6)
        const int off = q < XI ? q * 1024 : WS_XROWS * WS_CK * 2 + (q - XI) * 1024;
        __builtin_amdgcn_global_load_lds((const void*)(src[u] + ch * WS_CK), (lds_ptr_t)(base + off), 16, 0, 0);
      }
    };
      const int xi_used = (span + WS_RPI - 1) / WS_RPI;  // input pieces holding rows < span (the rest stay zero)
    auto elu_pass = [&](int ch) __attribute__((always_inline)) {
      ws_elu_pieces<PW>(smem + (ch % (WS_NBUF * CPB)) * (BUF * 2) + lane * 16, pw, xi_used);
    };
    // stages of CPB chunks, one barrier per stage
    const int nst = (nchunk + CPB - 1) / CPB;
    if (dbg & 1) {  // diagnostic: consumers alone (tune key 13 bit 0)
      for (int st = 0; st <= nst; ++st) __syncthreads();
    } else {
    // ring of NB = 4 CPB slots, prefetch distance D = NB - CPB chunks (slots are
    // released a stage at a time); wait_chunk(n): chunk landed with n younger
    // chunks still allowed in flight
    constexpr int NB = WS_NBUF * CPB, D = NB - CPB;
    static_assert(D >= 1 && 2 * CPB * PW < 64, "ring depth / vmcnt range");
    auto wait_chunk = [&](int younger) __attribute__((always_inline)) {
      if (younger >= 4 && 2 * CPB >= 4) ws_wait_vm<(2 * CPB >= 4 ? 4 * PW : 0)>();
      else if (younger == 3 && 2 * CPB >= 3) ws_wait_vm<(2 * CPB >= 3 ? 3 * PW : 0)>();
      else if (younger >= 2) ws_wait_vm<2 * PW>();
      else if (younger == 1) ws_wait_vm<PW>();
      else ws_wait_vm<0>();
    };
    for (int c = 0; c < D && c < nchunk; ++c) issue(c);
    // stage 0 landed (its last chunk with the younger ones in flight), then its ELU
    wait_chunk(std::min(D, nchunk) - std::min(CPB, nchunk));
    if (a.in_elu && !(dbg & 16))  // bit 4: diagnostic without the ELU pass
      for (int c = 0; c < CPB && c < nchunk; ++c) elu_pass(c);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    for (int st = 0; st < nst; ++st) {
      // issue first: the slots of stage st-1 were released by the last barrier,
      // and the count below assumes chunks up to min(st CPB + D + CPB - 1,
      // nchunk - 1) are out
      const int c0 = st * CPB;
      for (int c = c0 + D; c < c0 + D + CPB && c < nchunk; ++c) issue(c);
      if (c0 + CPB < nchunk) {
        // stage st+1 landed (later chunks may still be in flight), then its ELU
        const int issued = std::min(c0 + D + CPB, nchunk) - 1;
        const int need = std::min(c0 + 2 * CPB, nchunk) - 1;
        wait_chunk(issued - need);
        if (a.in_elu && !(dbg & 16))
          for (int c = c0 + CPB; c < c0 + 2 * CPB && c < nchunk; ++c) elu_pass(c);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
    }
  } else {
  // ---------------- consumers ----------------
  const int wm = wave >> 1, wn = wave & 1;
  const int hl = lane >> 5;
  int arow[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) arow[i] = wm * WTM + i * 32 + (lane & 31);
  int boff[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) boff[j] = WS_XROWS * WS_CK + ws_swz(wn * WTN + j * 32 + (lane & 31), hl);

  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  __syncthreads();
  // consumers outrank the producers in the SIMD's issue arbitration (tune key
  // 13 bit 7 = diagnostic without)
  if (!(dbg & 128)) __builtin_amdgcn_s_setprio(2);
  for (int ch = 0; ch < nchunk; ++ch) {
    // one barrier per stage of CPB chunks (after its last chunk)
    const bool stage_end = (ch + 1) % CPB == 0 || ch + 1 == nchunk;
    if (dbg & 2) {  // diagnostic: producers alone (tune key 13 bit 1)
      if (stage_end) __syncthreads();
      continue;
    }
    const __bf16* const xb = lds + (ch % (WS_NBUF * CPB)) * BUF;
    bf16x8 fa[2][TM], fb[2][TN];
    constexpr int NS = KT * (WS_CK / 16);  // (tap, 16-channel half) steps
    // slot bit 1 <-> element offset bit 4 (row * 32 keeps bits 0-4 clear)
    auto fetch = [&](int st, int q) {
      const int k = st / (WS_CK / 16), h = st % (WS_CK / 16);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        fb[q][j] = *reinterpret_cast<const bf16x8*>(xb + ((boff[j] + k * BN * WS_CK) ^ (16 * h)));
#pragma unroll
      for (int i = 0; i < TM; ++i)
        fa[q][i] = *reinterpret_cast<const bf16x8*>(xb + ws_swz(arow[i] + k * a.dil, 2 * h + hl));
    };
    for (int rep = 0; rep < ((dbg & 256) ? 2 : 1); ++rep) {  // bit 8: diagnostic double MFMA work
    fetch(0, 0);
#pragma unroll
    for (int st = 0; st < NS; ++st) {
      // pin the order: the next step's fragment reads go out before this step's MFMAs
      if (st + 1 < NS) fetch(st + 1, (st + 1) & 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fb[st & 1][j], fa[st & 1][i], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    }
    if (stage_end) __syncthreads();
  }

  __builtin_amdgcn_s_setprio(0);
  if (dbg & 8) {
    if (tid == 0) t_loop = __builtin_amdgcn_s_memrealtime();
  }
  if (!(dbg & 4)) {
    // accumulators -> fp32 tile [BM][BN + 4] over the (drained) ring: lane ->
    // row lane & 31 of its 32-row tile, element r -> column (r & 3) + 8 (r >> 2)
    // + 4 (lane >> 5), i.e. four 16-B runs per accumulator
    float* const tile = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int r = wm * WTM + i * 32 + (lane & 31);
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          floatx4 v4;
#pragma unroll
          for (int e = 0; e < 4; ++e) v4[e] = acc[i][j][4 * g + e];
          *reinterpret_cast<floatx4*>(tile + r * WS_EP + wn * WTN + j * 32 + 8 * g + 4 * hl) = v4;
        }
    }
  }
  }
  if (dbg & 4) return;  // diagnostic: no epilogue (tune key 13 bit 2)
  __syncthreads();

  // epilogue by all NC + 4 waves: 8 consecutive channels per thread, row-contiguous
  // 16-B global accesses (aux / res fetched for every vector first)
  struct alignas(16) V8 { TO v[8]; };
  constexpr int EV = (BM * BN / 8 + NT - 1) / NT;
  const float* const tile = reinterpret_cast<const float*>(smem);
  const int nvec = mrows * (BN / 8);
  V8 av[EV], rv[EV];
#pragma unroll
  for (int u = 0; u < EV; ++u) {
    const int v = tid + u * NT;
    if (v >= nvec) break;
    const int64_t o = (m0 + (v >> 4)) * a.ldo + n0 + (v & 15) * 8;
    if (aux) av[u] = *reinterpret_cast<const V8*>(aux + o);
    if (res) rv[u] = *reinterpret_cast<const V8*>(res + o);
  }
#pragma unroll
  for (int u = 0; u < EV; ++u) {
    const int v = tid + u * NT;
    if (v >= nvec) break;
    const int row = v >> 4, c8 = (v & 15) * 8;
    const int64_t o = (m0 + row) * a.ldo + n0 + c8;
    const floatx4 lo = *reinterpret_cast<const floatx4*>(tile + row * WS_EP + c8);
    const floatx4 hi = *reinterpret_cast<const floatx4*>(tile + row * WS_EP + c8 + 4);
    float x[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    if (a.epi) {
      // discriminator epilogue (k_dconv_mfma order): + bias, + res, * LeakyReLU'(aux),
      // LeakyReLU; rows past the computed ones are the next layer's zero padding
      const bool valid = (a.seq_pitch > 0 ? (t0 + row) % a.seq_pitch : t0 + row) < a.tout_valid;
      float bv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if (bias) {
        const floatx4 b0 = *reinterpret_cast<const floatx4*>(bias + n0 + c8);
        const floatx4 b1 = *reinterpret_cast<const floatx4*>(bias + n0 + c8 + 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) bv[e] = b0[e], bv[e + 4] = b1[e];
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float y = 0.f;
        if (valid) {
          y = x[e];
          if (bias) y += bv[e];
          if (res) y += to_f(rv[u].v[e]);
          if (aux) y *= to_f(av[u].v[e]) > 0.f ? 1.f : a.slope;
          if (a.act) y = y > 0.f ? y : y * a.slope;
        }
        x[e] = y;
      }
    } else {
    if (bias && a.bias_period) {
      if (a.bias_period % 8 == 0) {
        const float* const bp = bias + (n0 + c8) % a.bias_period;
        const floatx4 b0 = *reinterpret_cast<const floatx4*>(bp), b1 = *reinterpret_cast<const floatx4*>(bp + 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) x[e] += b0[e], x[e + 4] += b1[e];
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) x[e] += bias[(n0 + c8 + e) % a.bias_period];
      }
    }
    if (aux) {
#pragma unroll
      for (int e = 0; e < 8; ++e) x[e] *= elu_grad_fast(to_f(av[u].v[e]));
    }
    if (res) {
#pragma unroll
      for (int e = 0; e < 8; ++e) x[e] += to_f(rv[u].v[e]);
    }
    }
    V8 ov;
#pragma unroll
    for (int e = 0; e < 8; ++e) ov.v[e] = from_f<TO>(x[e]);
    *reinterpret_cast<V8*>(out + o) = ov;
  }
  if ((dbg & 8) && bias && !a.bias_period) {
    // diagnostic (tune key 13 bit 3): per-block stamps into a scratch "bias"
    // buffer: realtime (100 MHz) start / main-loop end / block end, shader
    // clock start / end, HW_ID, XCC_ID
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      uint64_t* st = reinterpret_cast<uint64_t*>(const_cast<float*>(bias)) +
                     8 * (int64_t(blockIdx.y) * gridDim.x + blockIdx.x);
      st[0] = t_start;
      st[1] = t_loop;
      st[2] = __builtin_amdgcn_s_memrealtime();
      st[3] = c_start;
      st[4] = __builtin_amdgcn_s_memtime();
      st[5] = uint64_t(__builtin_amdgcn_s_getreg(4 | (31 << 11)));   // HW_ID
      st[6] = uint64_t(__builtin_amdgcn_s_getreg(20 | (31 << 11)));  // XCC_ID
    }
  }
}

// ---------------------------------------------------------------------------
// Eight-wave form of the warp-specialised kernel (k_conv_ws8).  Same LDS ring
// layout, swizzle, DMA sources and (chunk, tap) MFMA order as k_conv_ws_bf16,
// hence bit-identical outputs, but:
//   - no producer waves: each of the 8 waves issues its share of the chunk's
//     1-KB DMA pieces (q = 8u + wave) and ELUs the input pieces it DMA'd;
//   - 128 x 64 per wave (4 x 2 MFMA tiles of 32 x 32): six fragment reads per
//     eight MFMAs instead of four per four, at 2 waves per SIMD with the
//     256-VGPR budget the 128 accumulators need;
//   - block tiles of 256 x 256 (the MPD's 512 / 1024-wide layers: half the
//     weight-slice DMA per flop of a 256 x 128 tile) or 512 x 128 (the 128-wide
//     k7 dgrads at T = 2000: 4 tiles per sample, 256 per launch);
//   - a 3-slot ring: chunk c + 2 is issued while chunk c is computed, chunk
//     c + 1 is waited for (counted vmcnt, never 0 while a later chunk is in
//     flight) after the first tap of chunk c, one raw barrier per chunk.
// The LDS image per chunk is what the 12-wave kernel's producers build, so
// the DMA and the ELU are unchanged; the LDS reads per flop fall by a quarter
// and the DMA'd weight bytes per flop by up to a half.
// ---------------------------------------------------------------------------
template <int KT, int BM, int BN, int HALO, int TM = 4>
struct Ws8 {
  static constexpr int WTM = 32 * TM;               // wave tile rows (x 64 columns)
  static constexpr int WM = BM / WTM, WN = BN / 64;  // wave grid
  static_assert(WM * WN == 8 && BM % 128 == 0, "eight wave tiles");
  static constexpr int XROWS = BM + HALO;           // staged input rows per chunk
  static constexpr int XI = XROWS / WS_RPI;         // input pieces (1 KB = 32 rows x 16 channels)
  static constexpr int WI = KT * BN / WS_RPI;       // weight pieces
  static constexpr int TI = XI + WI;
  static constexpr int PW = (TI + 7) / 8;           // pieces per wave per chunk
  static constexpr int NB = 3;                      // ring slots
  static constexpr int BUF = (XROWS + KT * BN) * WS_CK;  // bf16 elements per slot
  static constexpr int EP = BN + 4;                 // fp32 epilogue pitch (conflict-free 16-B writes)
  static constexpr size_t RING = size_t(NB) * BUF * 2;
  // epilogue pass rows: 256 where that fp32 tile fits over the ring (the 512 x
  // 128 tiles: 2 passes instead of 4, half the exposed aux / res load latency)
  static constexpr int PR = (BM >= 256 && size_t(256) * EP * 4 <= RING) ? 256 : 128;
  static constexpr size_t EPI = size_t(PR) * EP * 4;
  static constexpr size_t LDS = RING > EPI ? RING : EPI;
  static_assert(XROWS % WS_RPI == 0 && WI * WS_RPI == KT * BN && LDS <= 160 * 1024, "LDS");
  static_assert(2 * PW < 64, "vmcnt range");
};

template <int PW>
__device__ __forceinline__ void ws8_elu_pieces(unsigned char* slot, int lane, int wave, int xi) {
#pragma unroll
  for (int u = 0; u < PW; ++u) {
    const int q = u * 8 + wave;
    if (q >= xi) break;
    const unsigned addr = unsigned(reinterpret_cast<uintptr_t>(slot + q * 1024 + lane * 16));
    bf16x8 val;
    asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(val) : "v"(addr) : "memory");
    val = __builtin_bit_cast(bf16x8, elu8(__builtin_bit_cast(uint4, val)));
    asm volatile("ds_write_b128 %0, %1" : : "v"(addr), "v"(val) : "memory");
  }
}

template <int KT, typename TO, int BM, int BN, int HALO, int TM>
__global__ __launch_bounds__(512) void k_conv_ws8(Args a, const __bf16* __restrict__ in,
                                                  const __bf16* __restrict__ wp, const float* __restrict__ bias,
                                                  const TO* __restrict__ aux, const TO* __restrict__ res,
                                                  TO* __restrict__ out, int ncol, int dbg) {
  // dbg (tune key 13, diagnostics only): bit 0 = no DMA in the loop, bit 1 =
  // no MFMAs, bit 2 = no barriers in the loop, bit 3 = no epilogue
  using G = Ws8<KT, BM, BN, HALO, TM>;
  constexpr int PW = G::PW, XI = G::XI, TI = G::TI, NB = G::NB, BUF = G::BUF, XROWS = G::XROWS;
  extern __shared__ __align__(16) unsigned char smem[];
  __bf16* const lds = reinterpret_cast<__bf16*>(smem);
  const int span = BM + (KT - 1) * a.dil;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tps = (a.T + BM - 1) / BM;
  int64_t mt;
  int nt;
  xcd_tile(ncol, mt, nt);
  const int64_t b = mt / tps;
  const int t0 = int(mt % tps) * BM;
  const int64_t m0 = b * a.T + t0;
  const int mrows = a.T - t0 < BM ? a.T - t0 : BM;
  const int n0 = nt * BN;
  const int nchunk = a.C / WS_CK;

  // this wave's DMA pieces q = 8u + wave (past the last piece: the last one again)
  const __bf16* src[PW];
#pragma unroll
  for (int u = 0; u < PW; ++u) {
    const int q = u * 8 + wave < TI ? u * 8 + wave : TI - 1;
    if (q < XI) {
      const int R = q * WS_RPI + lane / WS_SPR, ls = (lane % WS_SPR) ^ ws_swzbits(R);
      int ti = t0 - a.pad + R;
      const bool valid =
          R < span && (a.seq_pitch > 0 ? ti >= 0 && ti < a.T && ti % a.seq_pitch < a.tin_valid
                                       : (ti >= 0 && ti < a.tin_valid) || a.pad_mode == SEL_PAD_REPLICATE);
      if (a.seq_pitch == 0) ti = ti < 0 ? 0 : (ti >= a.tin_valid ? a.tin_valid - 1 : ti);
      src[u] = valid ? in + (b * a.tin_pitch + ti) * a.ldx + 8 * ls : g_ws_zero + 8 * ls;
    } else {
      const int R = (q - XI) * WS_RPI + lane / WS_SPR, ls = (lane % WS_SPR) ^ ws_swzbits(R);
      const int k = R / BN, n = R % BN;
      src[u] = wp + (int64_t(n0 + n) * KT + k) * a.C + 8 * ls;
    }
  }
  auto issue = [&](int ch) __attribute__((always_inline)) {
    unsigned char* const base = smem + (ch % NB) * (BUF * 2);
#pragma unroll
    for (int u = 0; u < PW; ++u) {
      const int q = u * 8 + wave < TI ? u * 8 + wave : TI - 1;
      const int off = q < XI ? q * 1024 : XROWS * WS_CK * 2 + (q - XI) * 1024;
      __builtin_amdgcn_global_load_lds((const void*)(src[u] + ch * WS_CK), (lds_ptr_t)(base + off), 16, 0, 0);
    }
  };
  const int xi_used = (span + WS_RPI - 1) / WS_RPI;  // input pieces holding rows < span
  auto elu_pass = [&](int ch) __attribute__((always_inline)) {
    ws8_elu_pieces<PW>(smem + (ch % NB) * (BUF * 2), lane, wave, xi_used);
  };

  const int wm = wave / G::WN, wn = wave % G::WN;
  const int hl = lane >> 5;
  int arow[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) arow[i] = wm * G::WTM + i * 32 + (lane & 31);
  int boff[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) boff[j] = XROWS * WS_CK + ws_swz(wn * 64 + j * 32 + (lane & 31), hl);
  floatx16 acc[TM][2];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  // prologue: chunks 0 and 1 in flight, chunk 0 landed (and ELU'd) before the first barrier
  constexpr int D = NB - 1;
  for (int c = 0; c < D && c < nchunk; ++c) issue(c);
  if (nchunk > 1) ws_wait_vm<PW>();
  else ws_wait_vm<0>();
  if (a.in_elu) elu_pass(0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  for (int ch = 0; ch < nchunk; ++ch) {
    // chunk ch - 1's slot is free (every wave passed the barrier after reading it)
    if (ch + D < nchunk && !(dbg & 1)) issue(ch + D);
    const __bf16* const xb = lds + (ch % NB) * BUF;
    bf16x8 fa[2][TM], fb[2][2];
    auto fetch = [&](int k, int q) __attribute__((always_inline)) {
#pragma unroll
      for (int j = 0; j < 2; ++j) fb[q][j] = *reinterpret_cast<const bf16x8*>(xb + boff[j] + k * BN * WS_CK);
#pragma unroll
      for (int i = 0; i < TM; ++i) fa[q][i] = *reinterpret_cast<const bf16x8*>(xb + ws_swz(arow[i] + k * a.dil, hl));
    };
    fetch(0, 0);
#pragma unroll
    for (int k = 0; k < KT; ++k) {
      if (k + 1 < KT) fetch(k + 1, (k + 1) & 1);
      __builtin_amdgcn_sched_barrier(0);
      if (!(dbg & 2)) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fb[k & 1][j], fa[k & 1][i], acc[i][j], 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
      if (k == 0 && ch + 1 < nchunk) {
        // chunk ch + 1 landed (chunk ch + 2, when issued above, still in flight), then its ELU
        if (ch + D < nchunk && !(dbg & 1)) ws_wait_vm<PW>();
        else ws_wait_vm<0>();
        if (a.in_elu) elu_pass(ch + 1);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (!(dbg & 4)) __builtin_amdgcn_s_barrier();
  }
  if (dbg & 8) return;

  // epilogue in BM / PR passes of PR rows: the waves whose rows fall in pass p
  // write their accumulators into an fp32 [PR][BN + 4] tile over the (drained)
  // ring, then all 8 waves run row-contiguous 16-B accesses (the 12-wave
  // kernel's epilogue)
  struct alignas(16) V8 { TO v[8]; };
  constexpr int PR = G::PR, BNV = BN / 8, EV = PR * BNV / 512, NP = BM / PR;
  float* const tile = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    if (wm * G::WTM / PR == p) {
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int r = wm * G::WTM % PR + i * 32 + (lane & 31);
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            floatx4 v4;
#pragma unroll
            for (int e = 0; e < 4; ++e) v4[e] = acc[i][j][4 * g + e];
            *reinterpret_cast<floatx4*>(tile + r * G::EP + wn * 64 + j * 32 + 8 * g + 4 * hl) = v4;
          }
      }
    }
    __syncthreads();
    const int prow = p * PR;
#pragma unroll
    for (int u = 0; u < EV; ++u) {
      const int v = tid + u * 512;
      const int row = v / BNV, c8 = (v % BNV) * 8;
      if (prow + row >= mrows) continue;
      const int64_t o = (m0 + prow + row) * a.ldo + n0 + c8;
      V8 av, rv;
      if (aux) av = *reinterpret_cast<const V8*>(aux + o);
      if (res) rv = *reinterpret_cast<const V8*>(res + o);
      const floatx4 lo = *reinterpret_cast<const floatx4*>(tile + row * G::EP + c8);
      const floatx4 hi = *reinterpret_cast<const floatx4*>(tile + row * G::EP + c8 + 4);
      float x[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      if (a.epi) {
        const bool valid = (a.seq_pitch > 0 ? (t0 + prow + row) % a.seq_pitch : t0 + prow + row) < a.tout_valid;
        float bv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        if (bias) {
          const floatx4 b0 = *reinterpret_cast<const floatx4*>(bias + n0 + c8);
          const floatx4 b1 = *reinterpret_cast<const floatx4*>(bias + n0 + c8 + 4);
#pragma unroll
          for (int e = 0; e < 4; ++e) bv[e] = b0[e], bv[e + 4] = b1[e];
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float y = 0.f;
          if (valid) {
            y = x[e];
            if (bias) y += bv[e];
            if (res) y += to_f(rv.v[e]);
            if (aux) y *= to_f(av.v[e]) > 0.f ? 1.f : a.slope;
            if (a.act) y = y > 0.f ? y : y * a.slope;
          }
          x[e] = y;
        }
      } else {
        if (bias && a.bias_period) {
          if (a.bias_period % 8 == 0) {
            const float* const bp = bias + (n0 + c8) % a.bias_period;
            const floatx4 b0 = *reinterpret_cast<const floatx4*>(bp), b1 = *reinterpret_cast<const floatx4*>(bp + 4);
#pragma unroll
            for (int e = 0; e < 4; ++e) x[e] += b0[e], x[e + 4] += b1[e];
          } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) x[e] += bias[(n0 + c8 + e) % a.bias_period];
          }
        }
        if (aux) {
#pragma unroll
          for (int e = 0; e < 8; ++e) x[e] *= elu_grad_fast(to_f(av.v[e]));
        }
        if (res) {
#pragma unroll
          for (int e = 0; e < 8; ++e) x[e] += to_f(rv.v[e]);
        }
      }
      V8 ov;
#pragma unroll
      for (int e = 0; e < 8; ++e) ov.v[e] = from_f<TO>(x[e]);
      *reinterpret_cast<V8*>(out + o) = ov;
    }
    if (p + 1 < NP) __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// Weight-stationary streaming conv for the thin layers (32/64/96 input and
// 32/64 output channels: the residual-unit convs at T = 24000 / 8000, their
// dgrads, the first strided layer and the last transposed layer's dgrad).
// These are HBM-bound, yet the tiled kernel above re-stages every tap of the
// weight slice for each 128-row tile (for a 64x64 k7 layer, 3x the tile's
// activation bytes through L2 and LDS), and its neighbouring tiles land on
// different XCDs, so the causal halo is re-fetched from HBM (rocprofv3 PMC:
// 1.85x the algorithmic read bytes at 32 channels, profiles/r1_c3_pmc_traffic.md).
// Here each wave keeps the MFMA A-fragments of its 32-channel output slice
// for ALL taps and input channels in VGPRs (K*C/16 fragments, loaded once
// per block), and the block streams a CONTIGUOUS range of sample-aligned
// R-row tiles (the halo re-read hits the block's own XCD L2):
//   stage rows + causal halo (ELU applied, padding resolved) in LDS
//   -> K*C/16*TM MFMAs per wave while the next tile's rows are in flight
//   -> accumulators -> LDS (fp32) -> one fully coalesced 16-B epilogue pass
//      (bias, ELU'(aux), residual) over the tile's contiguous output rows.
// ---------------------------------------------------------------------------
template <int C, int N, int K, int R, bool E = false>
struct Thin {
  static constexpr int PLANES = C / 32;
  // NS output slices of 32 channels, RG row groups; at N = 96 the fourth
  // wave has no slice (it stages and runs the epilogue only)
  static constexpr int NS = N / 32, RG = 4 / NS;
  static constexpr int WR = R / RG, TM = WR / 32;
  static constexpr int SPAN = R + F4_HALOMAX;
  static constexpr int CV = C / 8;  // 16-B vectors per staged row
  static constexpr int XV = (SPAN * CV + 255) / 256;
  static constexpr int OP = N + 4;  // fp32 out-tile pitch (conflict-free b128)
  static constexpr size_t LDS_STAGE = size_t(PLANES) * SPAN * F4_P * 2;
  static constexpr size_t LDS_OUT = size_t(R) * OP * 4;
  static constexpr size_t LDS = LDS_STAGE > LDS_OUT ? LDS_STAGE : LDS_OUT;
  // E: epilogue-operand prefetch, EJ 16-B vectors per lane and operand held
  // in VGPRs across the MFMA phase (costs up to 8*EJ VGPRs, i.e. occupancy on
  // some instances: chosen per instance, kThinEpfDefault), plus the split
  // tile loop (separate staging and out tiles in LDS) where both fit in 64 KB
  static constexpr int EJ = (R * (N / 8) + 255) / 256;
  static constexpr bool EPF = E && EJ <= 8;
  static constexpr bool SPLIT = EPF && LDS_STAGE + LDS_OUT <= 64 * 1024;
  static constexpr size_t LDS_TOTAL = SPLIT ? LDS_STAGE + LDS_OUT : LDS;
  static_assert(N == 32 || N == 64 || N == 96 || N == 128, "thin kernel: N in {32, 64, 96, 128}");
  static_assert(C % 32 == 0 && WR % 32 == 0, "thin kernel tiling");
  static_assert(LDS <= 64 * 1024, "thin kernel LDS");
};

template <int C, int N, int K, int R, bool E>
__global__ __launch_bounds__(256) void k_conv_thin_bf16(Args a, const __bf16* __restrict__ in,
                                                        const __bf16* __restrict__ wp,
                                                        const float* __restrict__ bias,
                                                        const __bf16* __restrict__ aux,
                                                        const __bf16* __restrict__ res, __bf16* __restrict__ out,
                                                        int tiles_per_block, int epi_pf) {
  using G = Thin<C, N, K, R, E>;
  constexpr int P = F4_P;
  constexpr int CV = G::CV;
  extern __shared__ __align__(16) unsigned char smem[];
  __bf16* const xs = reinterpret_cast<__bf16*>(smem);  // [PLANES][SPAN][P]
  // [R][OP] fp32 out tile: aliases xs, or follows it when the tile loop is split
  float* const ot = reinterpret_cast<float*>(smem + (G::SPLIT ? G::LDS_STAGE : 0));
  const bool split = G::SPLIT && (epi_pf & 2);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ns = wave % G::NS, rg = wave / G::NS;
  const int span = R + (K - 1) * a.dil;
  const int tps = (a.T + R - 1) / R;
  const int64_t ntiles = (a.rows / a.T) * tps;
  // XCD-contiguous tile ranges: the grid is a multiple of 8 and block b runs on
  // XCD b % 8, so virtual block (b % 8) * (grid / 8) + b / 8 gives each XCD one
  // contiguous run of tiles, walked in dispatch order -> a tile's causal halo
  // was just fetched into the same L2 by its predecessor
  const int64_t vb = int64_t(blockIdx.x % 8) * (gridDim.x / 8) + blockIdx.x / 8;
  const int64_t tile0 = vb * tiles_per_block;
  const int64_t tile_end = tile0 + tiles_per_block < ntiles ? tile0 + tiles_per_block : ntiles;
  if (tile0 >= tile_end) return;  // block-uniform

  // A fragments of output slice ns: wf[k][g] = Wp[n][k][16g + 8*(lane>>5) .. +8]
  bf16x8 wf[K][C / 16];
  {
    const __bf16* wrow = wp + int64_t(ns * 32 + (lane & 31)) * K * C + 8 * (lane >> 5);
#pragma unroll
    for (int k = 0; k < K; ++k)
#pragma unroll
      for (int g = 0; g < C / 16; ++g) wf[k][g] = *reinterpret_cast<const bf16x8*>(wrow + k * C + 16 * g);
  }
  ws_wait_vm<0>();  // weights landed: the tile loop's MFMAs then wait on no request of the loop

  uint4 xr[G::XV];
  bool xok[G::XV];
  // branch-free buffer loads (Ru32Stage::load): rows past the span, zero-padded
  // rows and a dead request (live = false) read nothing and return zeros
  auto load = [&](int64_t tile, bool live) {
    const int64_t b = tile / tps;
    const int t0 = int(tile % tps) * R;
    const __amdgpu_buffer_rsrc_t rs = ru_rsrc(in + b * a.T * C, int64_t(a.T) * C);
#pragma unroll
    for (int u = 0; u < G::XV; ++u) {
      const int v = tid + u * 256;
      const int r = v / CV, c = (v % CV) * 8;
      int ti = t0 - a.pad + r;
      const bool inside = ti >= 0 && ti < a.T;
      xok[u] = r < span && (inside || a.pad_mode == SEL_PAD_REPLICATE);
      ti = ti < 0 ? 0 : (ti >= a.T ? a.T - 1 : ti);
      xr[u] = ru_bload(rs, live && xok[u] ? (ti * C + c) * 2 : RU_OOB);
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int u = 0; u < G::XV; ++u) {
      const int v = tid + u * 256;
      const int r = v / CV, c = (v % CV) * 8;
      if (r >= span) continue;
      uint4 val = xok[u] ? xr[u] : make_uint4(0, 0, 0, 0);
      if (a.in_elu) {
        val = elu8(val);
      }
      *reinterpret_cast<uint4*>(xs + ((c >> 5) * G::SPAN + r) * P + (c & 31)) = val;
    }
  };

  // the bias over this kernel's N output channels in LDS (bs[n] = bias[n % period]):
  // a global bias load in the epilogue would wait behind the next tile's request
  __shared__ __align__(16) float bs[N];
  const bool has_bias = bias && a.bias_period;
  if (has_bias && tid < N) bs[tid] = bias[tid % a.bias_period];
  load(tile0, true);
  if (split) {
    store();
    __syncthreads();
    if (tile0 + 1 < tile_end) load(tile0 + 1, true);
  }
  for (int64_t tile = tile0; tile < tile_end; ++tile) {
    if (!split) {
      __syncthreads();  // the previous tile's epilogue is done with ot (= xs)
      store();
      __syncthreads();
      load(tile + 1 < tile_end ? tile + 1 : tile, tile + 1 < tile_end);  // unconditional: exact counts
    }

    // this tile's epilogue operands (ELU'(aux), residual), fetched before the
    // MFMA phase so their HBM latency hides behind it instead of stalling the
    // epilogue (N <= 64: <= 8 16-B vectors per lane per operand)
    const int64_t eb = tile / tps;
    const int et0 = int(tile % tps) * R;
    const int emrows = a.T - et0 < R ? a.T - et0 : R;
    const int64_t eobase = (eb * a.T + et0) * N;
    uint4 apf[G::EPF ? G::EJ : 1], rpf[G::EPF ? G::EJ : 1];
    if constexpr (G::EPF) {
      if (epi_pf & 1) {
#pragma unroll
        for (int j = 0; j < G::EJ; ++j) {
          const int idx = tid + j * 256, r = idx / (N / 8), n = (idx % (N / 8)) * 8;
          const int64_t o = eobase + int64_t(r) * N + n;
          if (aux && r < emrows) apf[j] = *reinterpret_cast<const uint4*>(aux + o);
          if (res && r < emrows) rpf[j] = *reinterpret_cast<const uint4*>(res + o);
        }
      }
    }

    const bool mma_wave = G::NS * G::RG == 4 || rg < G::RG;  // wave-uniform
    floatx16 acc[G::TM];
#pragma unroll
    for (int i = 0; i < G::TM; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][e] = 0.f;
    const __bf16* xw = xs + ((mma_wave ? rg : 0) * G::WR + (lane & 31)) * P + 8 * (lane >> 5);
    if (mma_wave) {
#pragma unroll
      for (int k = 0; k < K; ++k) {
#pragma unroll
        for (int g = 0; g < C / 16; ++g) {
          const __bf16* xb = xw + ((g >> 1) * G::SPAN + k * a.dil) * P + 16 * (g & 1);
#pragma unroll
          for (int i = 0; i < G::TM; ++i) {
            const bf16x8 xf = *reinterpret_cast<const bf16x8*>(xb + i * 32 * P);
            acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[k][g], xf, acc[i], 0, 0, 0);
          }
        }
      }
    }

    // accumulators (out^T: lane -> row, element r -> channel) -> fp32 tile in LDS
    __syncthreads();  // every wave is done reading xs (split: and the last epilogue with ot)
    if (mma_wave) {
#pragma unroll
      for (int i = 0; i < G::TM; ++i) {
        const int row = rg * G::WR + i * 32 + (lane & 31);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int n = ns * 32 + 8 * g + 4 * (lane >> 5);
          *reinterpret_cast<floatx4*>(ot + row * G::OP + n) =
              floatx4{acc[i][4 * g], acc[i][4 * g + 1], acc[i][4 * g + 2], acc[i][4 * g + 3]};
        }
      }
    }
    // split loop: the next tile is staged beside this tile's out tile, so a
    // tile costs two barriers and its epilogue overlaps the next MFMA phase
    if (split && tile + 1 < tile_end) store();
    __syncthreads();
    if (split && tile + 2 < tile_end) load(tile + 2, true);

    // coalesced epilogue: a sample-aligned tile's output rows are contiguous in HBM
    const int64_t b = tile / tps;
    const int t0 = int(tile % tps) * R;
    const int mrows = a.T - t0 < R ? a.T - t0 : R;
    const int64_t obase = (b * a.T + t0) * N;
    constexpr int GN = N / 8;
    auto epilogue = [&](int idx, const uint4* apv, const uint4* rpv) {
      const int r = idx / GN, n = (idx % GN) * 8;
      const floatx4 lo = *reinterpret_cast<const floatx4*>(ot + r * G::OP + n);
      const floatx4 hi = *reinterpret_cast<const floatx4*>(ot + r * G::OP + n + 4);
      float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      if (has_bias) {
        const floatx4 b0 = *reinterpret_cast<const floatx4*>(bs + n);
        const floatx4 b1 = *reinterpret_cast<const floatx4*>(bs + n + 4);
        v[0] += b0[0], v[1] += b0[1], v[2] += b0[2], v[3] += b0[3];
        v[4] += b1[0], v[5] += b1[1], v[6] += b1[2], v[7] += b1[3];
      }
      const int64_t o = obase + int64_t(r) * N + n;
      // explicit roundings (no FMA contraction): every instance, and the fused
      // residual-unit kernels, produce the same bits
      if (aux) {
        uint4 raw = apv ? *apv : *reinterpret_cast<const uint4*>(aux + o);
        const __bf16* av = reinterpret_cast<const __bf16*>(&raw);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = __fmul_rn(v[e], elu_grad_fast(float(av[e])));
      }
      if (res) {
        uint4 raw = rpv ? *rpv : *reinterpret_cast<const uint4*>(res + o);
        const __bf16* rv = reinterpret_cast<const __bf16*>(&raw);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = __fadd_rn(v[e], float(rv[e]));
      }
      uint4 ov;
      __bf16* op = reinterpret_cast<__bf16*>(&ov);
#pragma unroll
      for (int e = 0; e < 8; ++e) op[e] = __bf16(v[e]);
      *reinterpret_cast<uint4*>(out + o) = ov;
    };
    if (G::EPF && (epi_pf & 1)) {
#pragma unroll
      for (int j = 0; j < (G::EPF ? G::EJ : 1); ++j)
        if (tid + j * 256 < mrows * GN) epilogue(tid + j * 256, &apf[j], &rpf[j]);
    } else {
      for (int idx = tid; idx < mrows * GN; idx += 256) epilogue(idx, nullptr, nullptr);
    }
  }
}

// ---------------------------------------------------------------------------
// Fused residual-unit forward for the thin layers (residual_unit.py:43-46 with
// conv1 = causal K-tap dilated C->C, conv2 = 1x1 C->C, no bias in AudioDec):
//   h   = conv1(ELU(x))                       -> HBM (saved for the backward)
//   out = x + conv2(ELU(h))                   -> HBM
// One pass over the tile: conv1 as in k_conv_thin_bf16 (weights in VGPRs,
// ELU at staging), its accumulators -> fp32 tile in LDS -> coalesced h store
// AND ELU(bf16(h)) staged straight into a second LDS tile that feeds conv2's
// MFMAs (its weights also in VGPRs); the residual is re-read from L2 in the
// final coalesced epilogue.  vs. two primitive calls this drops the h re-read
// and one x re-read from HBM (5 -> 3 activation-sized tensors per unit).
// ---------------------------------------------------------------------------
template <int C, int K, int R>
struct RuThin {
  using G = Thin<C, C, K, R>;
  static constexpr size_t LDS_HS = size_t(G::PLANES) * R * F4_P * 2;
  static constexpr size_t LDS = G::LDS + LDS_HS;
  static_assert(LDS <= 64 * 1024, "fused residual unit LDS");
};

template <int C, int K, int R>
__global__ __launch_bounds__(256) void k_ru_thin_bf16(Args a, const __bf16* __restrict__ in,
                                                      const __bf16* __restrict__ w1p, const float* __restrict__ b1,
                                                      const __bf16* __restrict__ w2p, const float* __restrict__ b2,
                                                      __bf16* __restrict__ hout, __bf16* __restrict__ out,
                                                      int tiles_per_block) {
  using G = Thin<C, C, K, R>;
  constexpr int P = F4_P;
  constexpr int CV = G::CV;
  constexpr int N = C;
  extern __shared__ __align__(16) unsigned char smem[];
  __bf16* const xs = reinterpret_cast<__bf16*>(smem);                   // [PLANES][SPAN][P]
  float* const ot = reinterpret_cast<float*>(smem);                     // [R][OP], aliases xs
  __bf16* const hs = reinterpret_cast<__bf16*>(smem + G::LDS);          // [PLANES][R][P]

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ns = wave % G::NS, rg = wave / G::NS;
  const int span = R + (K - 1) * a.dil;
  const int tps = (a.T + R - 1) / R;
  const int64_t ntiles = (a.rows / a.T) * tps;
  const int64_t vb = int64_t(blockIdx.x % 8) * (gridDim.x / 8) + blockIdx.x / 8;
  const int64_t tile0 = vb * tiles_per_block;
  const int64_t tile_end = tile0 + tiles_per_block < ntiles ? tile0 + tiles_per_block : ntiles;
  if (tile0 >= tile_end) return;  // block-uniform

  bf16x8 wf[K][C / 16], wf2[C / 16];
  {
    const __bf16* wrow = w1p + int64_t(ns * 32 + (lane & 31)) * K * C + 8 * (lane >> 5);
#pragma unroll
    for (int k = 0; k < K; ++k)
#pragma unroll
      for (int g = 0; g < C / 16; ++g) wf[k][g] = *reinterpret_cast<const bf16x8*>(wrow + k * C + 16 * g);
    const __bf16* wrow2 = w2p + int64_t(ns * 32 + (lane & 31)) * C + 8 * (lane >> 5);
#pragma unroll
    for (int g = 0; g < C / 16; ++g) wf2[g] = *reinterpret_cast<const bf16x8*>(wrow2 + 16 * g);
  }

  uint4 xr[G::XV];
  bool xok[G::XV];
  auto load = [&](int64_t tile) {
    const int64_t b = tile / tps;
    const int t0 = int(tile % tps) * R;
#pragma unroll
    for (int u = 0; u < G::XV; ++u) {
      const int v = tid + u * 256;
      const int r = v / CV, c = (v % CV) * 8;
      int ti = t0 - a.pad + r;
      xok[u] = r < span && ti >= 0 && ti < a.T;
      ti = ti < 0 ? 0 : (ti >= a.T ? a.T - 1 : ti);
      if ((u * 256) / CV < span) xr[u] = *reinterpret_cast<const uint4*>(in + (b * a.T + ti) * C + c);
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int u = 0; u < G::XV; ++u) {
      const int v = tid + u * 256;
      const int r = v / CV, c = (v % CV) * 8;
      if (r >= span) continue;
      uint4 val = xok[u] ? xr[u] : make_uint4(0, 0, 0, 0);
      val = elu8(val);
      *reinterpret_cast<uint4*>(xs + ((c >> 5) * G::SPAN + r) * P + (c & 31)) = val;
    }
  };
  // accumulators (out^T: lane -> row, element -> channel) -> fp32 tile in LDS
  auto acc_to_ot = [&](const floatx16 (&acc)[G::TM]) {
#pragma unroll
    for (int i = 0; i < G::TM; ++i) {
      const int row = rg * G::WR + i * 32 + (lane & 31);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int n = ns * 32 + 8 * g + 4 * (lane >> 5);
        *reinterpret_cast<floatx4*>(ot + row * G::OP + n) =
            floatx4{acc[i][4 * g], acc[i][4 * g + 1], acc[i][4 * g + 2], acc[i][4 * g + 3]};
      }
    }
  };
  constexpr int GN = N / 8;

  load(tile0);
  for (int64_t tile = tile0; tile < tile_end; ++tile) {
    __syncthreads();  // the previous tile's epilogue is done with ot (= xs)
    store();
    __syncthreads();
    if (tile + 1 < tile_end) load(tile + 1);
    const int64_t b = tile / tps;
    const int t0 = int(tile % tps) * R;
    const int mrows = a.T - t0 < R ? a.T - t0 : R;
    const int64_t obase = (b * a.T + t0) * N;

    // conv1
    floatx16 acc[G::TM];
#pragma unroll
    for (int i = 0; i < G::TM; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][e] = 0.f;
    {
      const __bf16* xw = xs + (rg * G::WR + (lane & 31)) * P + 8 * (lane >> 5);
#pragma unroll
      for (int k = 0; k < K; ++k)
#pragma unroll
        for (int g = 0; g < C / 16; ++g) {
          const __bf16* xb = xw + ((g >> 1) * G::SPAN + k * a.dil) * P + 16 * (g & 1);
#pragma unroll
          for (int i = 0; i < G::TM; ++i)
            acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[k][g], *reinterpret_cast<const bf16x8*>(xb + i * 32 * P),
                                                             acc[i], 0, 0, 0);
        }
    }
    __syncthreads();  // every wave is done reading xs
    acc_to_ot(acc);
    __syncthreads();
    // h epilogue: + b1, store h (bf16), stage ELU(h) for conv2
    for (int idx = tid; idx < R * GN; idx += 256) {
      const int r = idx / GN, n = (idx % GN) * 8;
      const floatx4 lo = *reinterpret_cast<const floatx4*>(ot + r * G::OP + n);
      const floatx4 hi = *reinterpret_cast<const floatx4*>(ot + r * G::OP + n + 4);
      float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      if (b1) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += b1[n + e];
      }
      uint4 hv, ev;
      __bf16* hp = reinterpret_cast<__bf16*>(&hv);
      __bf16* ep = reinterpret_cast<__bf16*>(&ev);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        hp[e] = __bf16(v[e]);
        ep[e] = __bf16(elu_fast(float(hp[e])));
      }
      if (r < mrows) *reinterpret_cast<uint4*>(hout + obase + int64_t(r) * N + n) = hv;
      *reinterpret_cast<uint4*>(hs + ((n >> 5) * R + r) * P + (n & 31)) = ev;
    }
    __syncthreads();
    // conv2 (1x1)
#pragma unroll
    for (int i = 0; i < G::TM; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][e] = 0.f;
    {
      const __bf16* hw = hs + (rg * G::WR + (lane & 31)) * P + 8 * (lane >> 5);
#pragma unroll
      for (int g = 0; g < C / 16; ++g) {
        const __bf16* hb = hw + (g >> 1) * R * P + 16 * (g & 1);
#pragma unroll
        for (int i = 0; i < G::TM; ++i)
          acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf2[g], *reinterpret_cast<const bf16x8*>(hb + i * 32 * P),
                                                           acc[i], 0, 0, 0);
      }
    }
    acc_to_ot(acc);  // ot is free: the h epilogue read it before the last barrier
    __syncthreads();
    for (int idx = tid; idx < mrows * GN; idx += 256) {
      const int r = idx / GN, n = (idx % GN) * 8;
      const floatx4 lo = *reinterpret_cast<const floatx4*>(ot + r * G::OP + n);
      const floatx4 hi = *reinterpret_cast<const floatx4*>(ot + r * G::OP + n + 4);
      float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      if (b2) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += b2[n + e];
      }
      const int64_t o = obase + int64_t(r) * N + n;
      uint4 raw = *reinterpret_cast<const uint4*>(in + o);
      const __bf16* rv = reinterpret_cast<const __bf16*>(&raw);
      uint4 ov;
      __bf16* op = reinterpret_cast<__bf16*>(&ov);
#pragma unroll
      for (int e = 0; e < 8; ++e) op[e] = __bf16(v[e] + float(rv[e]));
      *reinterpret_cast<uint4*>(out + o) = ov;
    }
  }
}

// ---------------------------------------------------------------------------
// Residual unit at 32 channels, forward and backward in ONE launch each, with
// the 1x1 conv done in registers (residual_unit.py:43-46; conv1 = causal k7
// dilated 32 -> 32, conv2 = 1x1 32 -> 32, both with bias in AudioDec).
//
// A wave owns 32-row sub-tiles of a sample-aligned R-row tile and all 32
// channels of them.  conv1's accumulators (lane -> row, element e -> channel
// (e & 3) + 8 (e >> 2) + 4 (lane >> 5)) are packed to bf16 and re-laid out with
// two v_permlane32_swap per channel-group pair into 8-consecutive-channel
// vectors: exactly the B operand of the next 32x32x16 MFMA AND one 16-B
// store.  So h goes to HBM (saved for the backward) and ELU(h) straight into
// conv2's MFMAs without an LDS round trip or a block barrier; the only shared
// stage is the input tile with its causal halo.  HBM per row: forward reads x
// and writes h, out (3 tensors instead of 5 over two launches); backward
// reads g (grad of out), h, x and writes gx (+ gh for the weight gradient):
// 4-5 tensors instead of 7 over two launches.
//
// Same MFMA order, same bf16 rounding points and the same epilogue arithmetic
// as the two-launch primitive path, so the results are bit-identical to it
// (test_gpu_conv.py::test_resunit32_*).
// ---------------------------------------------------------------------------
constexpr int RU_C = 32, RU_K = 7;

// acc (one 32x32 MFMA result) -> bf16, re-laid out: frag[kc] = channels
// 16 kc + 8 (lane >> 5) .. +8 of this lane's row (T21 of the HIP guide)
// Global stores of the fused residual-unit kernels' outputs (h, out, gh, gx:
// written once, read by a later launch).  SEL_RU_NT=1 builds them as streaming
// (non-temporal) stores, the |X| kernel's lever (A/B library: make nt).
#ifndef SEL_RU_NT
#define SEL_RU_NT 0
#endif
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void ru_store(__bf16* p, bf16x8 v) {
  if constexpr (SEL_RU_NT) __builtin_nontemporal_store(__builtin_bit_cast(u32x4, v), reinterpret_cast<u32x4*>(p));
  else *reinterpret_cast<bf16x8*>(p) = v;
}

// branch-free output store into a buffer resource (ru_rsrc): a row outside the
// tile's valid rows takes RU_OOB and is dropped by the hardware.  Every wave
// then issues the same number of stores per tile, so the compiler counts the
// next tile's prefetch exactly (a conditional store made the staging wait at
// the top of the next tile fall back to vmcnt(0), i.e. wait for these stores'
// completion too).
// AUX: the store's cache policy (2 = nt, streaming).  Judged inside the
// profiled step (tools/ru_bench.py re-reads its own inputs, which favours
// anything that keeps them cached): nt pays on k_ru32_fwd's h rows (read
// again only by the backward), and loses on outputs the next kernel reads
// (k_ru32_bwd's gx) or on rows two waves write in halves (k_ru64_fwd's h)
// k_ru32_fwd's h rows (read again only by the backward, much later) leave as
// nt stores: 71.7-72.5 -> 69.1-69.5 us per unit inside the profiled C3 step;
// nt on both h and out measured 1.5-2x slower, nt on out alone neutral
// (A/B builds: SEL_RU_FWD_*NT)
#ifndef SEL_RU_FWD_HNT
#define SEL_RU_FWD_HNT 2
#endif
#ifndef SEL_RU_FWD_ONT
#define SEL_RU_FWD_ONT 0
#endif
// k_ru32_bwd's gx rows: plain stores.  nt measured 86 -> 79 us per unit in
// tools/ru_bench.py but 87.4-88.0 -> 90.8-91.0 us inside the profiled C3 step
// (the next layer's backward reads gx right away); A/B builds: SEL_RU32B_GXNT=2
#ifndef SEL_RU32B_GXNT
#define SEL_RU32B_GXNT 0
#endif
template <int AUX = 0>
__device__ __forceinline__ void ru_bstore(__amdgpu_buffer_rsrc_t rs, int byte_off, bf16x8 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rs, byte_off, 0, AUX);
}

// N dropped stores (a zero-byte region; distinct offsets so that the compiler
// keeps them apart) after a tile loop's first prefetch: the loop issues N
// output stores after each later prefetch, so both paths into the staging
// waits carry the same count and the compiler leaves those stores pending
template <int N>
__device__ __forceinline__ void ru_dummy_stores(const __bf16* base) {
  const __amdgpu_buffer_rsrc_t rz = ru_rsrc(base, 0);
  const bf16x8 z = {};
#pragma unroll
  for (int i = 0; i < N; ++i) ru_bstore(rz, 16 * i, z);
}

__device__ __forceinline__ void ru_acc_to_frags(const float (&v)[16], bf16x8 (&frag)[2]) {
  unsigned pk[8];
#pragma unroll
  for (int q = 0; q < 8; ++q)
    pk[q] = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2{v[2 * q], v[2 * q + 1]}), bf16x2));
  // group g = elements 4g..4g+3 = pk[2g], pk[2g+1]; swap pairs (0,1) and (2,3)
#pragma unroll
  for (int pr = 0; pr < 2; ++pr) {
    unsigned a0 = pk[4 * pr], a1 = pk[4 * pr + 1], b0 = pk[4 * pr + 2], b1 = pk[4 * pr + 3];
    const auto r0 = __builtin_amdgcn_permlane32_swap(a0, b0, false, false);
    const auto r1 = __builtin_amdgcn_permlane32_swap(a1, b1, false, false);
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 w = {r0[0], r1[0], r0[1], r1[1]};
    frag[pr] = __builtin_bit_cast(bf16x8, w);
  }
}

// ---------------------------------------------------------------------------
// Pointwise (1x1) conv for the 256-wide residual units at T = 400
// (residual_unit.py:43-46's conv2 forward, out = x + W ELU(h), and its dgrad,
// gh = ELU'(h) * W^T g).  The tiled kernel ran them as 8 dependent
// 32-channel chunk steps per 64 x 128 tile (one global-load latency per
// step): 19 us per launch for 39 MB, 2 TB/s.  Here one workgroup per CU owns
// a contiguous range of rows:
//   - N/32 waves; wave w holds the MFMA fragments of output columns
//     [32w, 32w + 32) for all C input channels in VGPRs;
//   - a pass over up to SUB 32-row sub-tiles requests everything up front,
//     in use order: sub-tile 0's rows and epilogue operands, the weights,
//     then the later sub-tiles (all row-contiguous 16-B pieces);
//   - per sub-tile: wait for its own rows only, ELU them into its LDS slice,
//     barrier, C/16 MFMAs per wave with every fragment read ahead,
//     accumulators -> fp32 LDS tile, barrier, and a row-contiguous epilogue
//     (bias, ELU'(aux), residual; 16-B stores), overlapping the arrival of
//     the later sub-tiles;
//   - every access is a buffer access over the block's own row range, so rows
//     past it read zeros and their stores are dropped (no tail masking).
// Same MFMA (32x32x16, weights as the first operand), same channel order and
// the same epilogue roundings as k_conv_fwd_bf16: bit-identical outputs for
// one epilogue operand (the residual-unit forms).
// ---------------------------------------------------------------------------
template <int C, int N>
struct Pw {
  static constexpr int WAVES = N / 32;
  static constexpr int THREADS = WAVES * 64;
  static constexpr int R = 32;                       // rows per sub-tile (one 32x32 MFMA tile)
  static constexpr int SUB = 4;                      // sub-tiles per pass
  static constexpr int RB = R * SUB;                 // rows per pass
  static constexpr int PITCH = C + 8;                // LDS row pitch (bf16): conflict-free b128 reads
  static constexpr int OP = N + 4;                   // fp32 out-tile pitch
  static constexpr int XV = R * (C / 8) / THREADS;   // 16-B input pieces per thread per sub-tile
  static constexpr int EV = R * (N / 8) / THREADS;   // 16-B output pieces per thread per sub-tile
  static constexpr size_t LDS_X = size_t(RB) * PITCH * 2;
  static constexpr size_t LDS = LDS_X + size_t(R) * OP * 4;
  static_assert(XV >= 1 && R * (C / 8) % THREADS == 0 && EV >= 1 && R * (N / 8) % THREADS == 0, "pw pieces");
};

#ifndef SEL_W_PW
#define SEL_W_PW 2
#endif
// timing ablations (diagnostic builds only, tools/pw_abl.sh): 1 no weight
// loads, 2 no MFMAs, 4 no epilogue operand loads, 8 no output stores
#ifndef SEL_PW_ABL
#define SEL_PW_ABL 0
#endif

template <int C, int N, bool ELU, bool AUX, bool RES>
__global__ __launch_bounds__((N / 32) * 64) __attribute__((amdgpu_waves_per_eu(SEL_W_PW))) void k_pw_bf16(
    Args a, const __bf16* __restrict__ in, const __bf16* __restrict__ wp, const float* __restrict__ bias,
    const __bf16* __restrict__ aux, const __bf16* __restrict__ res, __bf16* __restrict__ out, int rows_per_block) {
  using G = Pw<C, N>;
  constexpr int R = G::R, SUB = G::SUB, PITCH = G::PITCH, OP = G::OP, T = G::THREADS;
  extern __shared__ __align__(16) unsigned char smem[];
  __bf16* const xs = reinterpret_cast<__bf16*>(smem);             // [RB][PITCH]
  float* const ot = reinterpret_cast<float*>(smem + G::LDS_X);    // [R][OP]
  __shared__ __align__(16) float bs[N];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t r0 = int64_t(blockIdx.x) * rows_per_block;
  if (r0 >= a.rows) return;  // block-uniform
  const int nrows = int(a.rows - r0 < rows_per_block ? a.rows - r0 : rows_per_block);

  const __amdgpu_buffer_rsrc_t rin = ru_rsrc(in + r0 * C, int64_t(nrows) * C);
  const __amdgpu_buffer_rsrc_t rout = ru_rsrc(out + r0 * N, int64_t(nrows) * N);
  const __amdgpu_buffer_rsrc_t raux = ru_rsrc(AUX ? aux + r0 * N : out, AUX ? int64_t(nrows) * N : 0);
  const __amdgpu_buffer_rsrc_t rres = ru_rsrc(RES ? res + r0 * N : out, RES ? int64_t(nrows) * N : 0);

  // the bias over the N columns (bs[n] = bias[n % period]) goes to LDS after
  // the first sub-tile's requests; its value is requested here
  const bool has_bias = bias && a.bias_period;
  const float bval = has_bias && tid < N ? bias[tid % a.bias_period] : 0.f;

  // input piece u of a sub-tile: row v / (C/8), channels (v % (C/8)) * 8;
  // output piece j: row v / (N/8), channels (v % (N/8)) * 8 (v = tid + u*T)
  uint4 xr[SUB][G::XV], ar[SUB][G::EV], rr[SUB][G::EV];
  auto request = [&](int p0, int s) {
#pragma unroll
    for (int u = 0; u < G::XV; ++u) {
      const int v = tid + u * T;
      xr[s][u] = ru_bload(rin, ((p0 + s * R + v / (C / 8)) * C + (v % (C / 8)) * 8) * 2);
    }
#pragma unroll
    for (int j = 0; j < G::EV; ++j) {
      const int v = tid + j * T;
      const int off = ((p0 + s * R + v / (N / 8)) * N + (v % (N / 8)) * 8) * 2;
      if constexpr (SEL_PW_ABL & 4) {
        ar[s][j] = make_uint4(off, 7u, 9u, 11u);
        rr[s][j] = make_uint4(off ^ 5, 3u, 1u, 13u);
      } else {
        if constexpr (AUX) ar[s][j] = ru_bload(raux, off);
        if constexpr (RES) rr[s][j] = ru_bload(rres, off);
      }
    }
  };
  // weight fragments of this wave's 32 output columns: wf[g] = Wp[n][16g + 8*(lane>>5) .. +8]
  bf16x8 wf[C / 16];
  const __bf16* const wrow = wp + int64_t(wave * 32 + (lane & 31)) * C + 8 * (lane >> 5);

  for (int p0 = 0; p0 < nrows; p0 += G::RB) {
    if (p0) __syncthreads();  // the previous pass is done with xs / ot
    request(p0, 0);
#pragma unroll
    for (int g = 0; g < C / 16; ++g) {
      if constexpr (SEL_PW_ABL & 1) wf[g] = __builtin_bit_cast(bf16x8, make_uint4(lane * 7u + g, g, lane, 3u));
      else wf[g] = *reinterpret_cast<const bf16x8*>(wrow + 16 * g);
    }
#pragma unroll
    for (int s = 1; s < SUB; ++s) request(p0, s);
    if (tid < N) bs[tid] = bval;  // visible after the first sub-tile's barrier

#pragma unroll
    for (int s = 0; s < SUB; ++s) {
      if (p0 + s * R >= nrows) break;  // block-uniform
      // sub-tile s's rows -> its own LDS slice
#pragma unroll
      for (int u = 0; u < G::XV; ++u) {
        const int v = tid + u * T;
        const uint4 val = ELU ? elu8(xr[s][u]) : xr[s][u];
        *reinterpret_cast<uint4*>(xs + (s * R + v / (C / 8)) * PITCH + (v % (C / 8)) * 8) = val;
      }
      __syncthreads();
      // every fragment of the sub-tile requested before the first MFMA
      const __bf16* xb = xs + (s * R + (lane & 31)) * PITCH + 8 * (lane >> 5);
      bf16x8 xf[C / 16];
#pragma unroll
      for (int g = 0; g < C / 16; ++g) xf[g] = *reinterpret_cast<const bf16x8*>(xb + 16 * g);
      __builtin_amdgcn_sched_barrier(0);
      floatx16 acc;
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[e] = 0.f;
      if constexpr (SEL_PW_ABL & 2) {
#pragma unroll
        for (int g = 0; g < C / 16; ++g) acc[g] = float(xf[g][0]) + float(wf[g][1]);
      } else {
#pragma unroll
        for (int g = 0; g < C / 16; ++g) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[g], xf[g], acc, 0, 0, 0);
      }
      // accumulators (out^T: lane -> row, element 4q + e -> channel 32w + 8q + 4*(lane>>5) + e)
      // -> fp32 tile; the previous sub-tile's epilogue reads ended before this
      // sub-tile's barrier
#pragma unroll
      for (int q = 0; q < 4; ++q)
        *reinterpret_cast<floatx4*>(ot + (lane & 31) * OP + wave * 32 + 8 * q + 4 * (lane >> 5)) =
            floatx4{acc[4 * q], acc[4 * q + 1], acc[4 * q + 2], acc[4 * q + 3]};
      __syncthreads();
#pragma unroll
      for (int j = 0; j < G::EV; ++j) {
        const int v = tid + j * T, r = v / (N / 8), n = (v % (N / 8)) * 8;
        const floatx4 lo = *reinterpret_cast<const floatx4*>(ot + r * OP + n);
        const floatx4 hi = *reinterpret_cast<const floatx4*>(ot + r * OP + n + 4);
        float x[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        if (has_bias) {
          const floatx4 b0 = *reinterpret_cast<const floatx4*>(bs + n);
          const floatx4 b1 = *reinterpret_cast<const floatx4*>(bs + n + 4);
          x[0] += b0[0], x[1] += b0[1], x[2] += b0[2], x[3] += b0[3];
          x[4] += b1[0], x[5] += b1[1], x[6] += b1[2], x[7] += b1[3];
        }
        if constexpr (AUX) {
          const __bf16* av = reinterpret_cast<const __bf16*>(&ar[s][j]);
#pragma unroll
          for (int e = 0; e < 8; ++e) x[e] = __fmul_rn(x[e], elu_grad_fast(float(av[e])));
        }
        if constexpr (RES) {
          const __bf16* rv = reinterpret_cast<const __bf16*>(&rr[s][j]);
#pragma unroll
          for (int e = 0; e < 8; ++e) x[e] = __fadd_rn(x[e], float(rv[e]));
        }
        bf16x8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = __bf16(x[e]);
        if (!(SEL_PW_ABL & 8) || x[0] == 1234.5f)
          ru_bstore(rout, ((p0 + s * R + r) * N + n) * 2, o);
      }
    }
  }
}

template <int R>
struct Ru32 {
  static constexpr int P = F4_P;
  static constexpr int SPAN = R + F4_HALOMAX;   // staged rows (tile + max halo)
  static constexpr int XV = (SPAN * 4 + 255) / 256;
  static constexpr int TM = R / 128;            // 32-row sub-tiles per wave
  static constexpr size_t LDS_FWD = size_t(SPAN + R) * P * 2;  // ELU(x) span + raw tile rows
  static constexpr size_t LDS_BWD = 3 * size_t(SPAN) * P * 2;  // g, gh and h tiles
  static_assert(R % 128 == 0, "ru32 tile rows");
};

// stage `span` rows of a 32-channel tensor starting at sample row t0 + off
// (rows outside [0, T) -> zero) into registers / LDS (optionally ELU'd)
template <int R>
struct Ru32Stage {
  uint4 r[Ru32<R>::XV];
  bool ok[Ru32<R>::XV];
  // Buffer loads over sample b: rows outside [0, T), past the span or of a
  // dead request (live = false: no next tile) take an out-of-range offset and
  // return zeros without touching memory.  No branch around any load, so the
  // compiler counts this request exactly and later waits in the tile loop do
  // not fall back to vmcnt(0) behind it.
  __device__ __forceinline__ void load(const Args& a, const __bf16* __restrict__ src, int64_t b, int t0, int off,
                                       int span, bool live = true) {
    const __amdgpu_buffer_rsrc_t rs = ru_rsrc(src + b * a.T * RU_C, a.T * RU_C);
#pragma unroll
    for (int u = 0; u < Ru32<R>::XV; ++u) {
      const int v = threadIdx.x + u * 256;
      const int row = v >> 2, c = (v & 3) * 8;
      const int ti = t0 + off + row;
      ok[u] = row < span && ti >= 0 && ti < a.T;
      r[u] = ru_bload(rs, live && ok[u] ? (ti * RU_C + c) * 2 : RU_OOB);
      // program order pinned: the same order from the prologue and the tile
      // loop, so the staging waits count both paths into them exactly
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  // raw != nullptr: rows [raw_off, raw_off + R) are also stored un-ELU'd into raw
  __device__ __forceinline__ void store(__bf16* xs, int span, bool elu, __bf16* raw = nullptr, int raw_off = 0,
                                        int pitch = F4_P) {
#pragma unroll
    for (int u = 0; u < Ru32<R>::XV; ++u) {
      const int v = threadIdx.x + u * 256;
      const int row = v >> 2, c = (v & 3) * 8;
      if (row >= span) continue;
      uint4 val = ok[u] ? r[u] : make_uint4(0, 0, 0, 0);
      if (raw && row >= raw_off && row < raw_off + R) *reinterpret_cast<uint4*>(raw + (row - raw_off) * F4_P + c) = val;
      if (elu) {
        val = elu8(val);
      }
      *reinterpret_cast<uint4*>(xs + row * pitch + c) = val;
    }
  }
};

// XCD-contiguous tile range of this block (as k_conv_thin_bf16)
__device__ __forceinline__ bool ru_tiles(int64_t ntiles, int tiles_per_block, int64_t& t_begin, int64_t& t_end) {
  const int64_t vb = int64_t(blockIdx.x % 8) * (gridDim.x / 8) + blockIdx.x / 8;
  t_begin = vb * tiles_per_block;
  t_end = t_begin + tiles_per_block < ntiles ? t_begin + tiles_per_block : ntiles;
  return t_begin < t_end;
}

// A fragments of a packed [32][K][32] weight (row n = lane & 31, channels 16 g + 8 (lane >> 5))
template <int K>
__device__ __forceinline__ void ru_wfrags(const __bf16* __restrict__ wp, bf16x8 (&wf)[K][2]) {
  const int lane = threadIdx.x & 63;
  const __bf16* wrow = wp + int64_t(lane & 31) * K * RU_C + 8 * (lane >> 5);
#pragma unroll
  for (int k = 0; k < K; ++k)
#pragma unroll
    for (int g = 0; g < 2; ++g) wf[k][g] = *reinterpret_cast<const bf16x8*>(wrow + k * RU_C + 16 * g);
}

template <int R>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(R == 128 ? SEL_W_RU32F128 : SEL_W_RU32F))) void k_ru32_fwd(Args a, const __bf16* __restrict__ x,
                                                  const __bf16* __restrict__ w1p, const float* __restrict__ b1,
                                                  const __bf16* __restrict__ w2p, const float* __restrict__ b2,
                                                  __bf16* __restrict__ hout, __bf16* __restrict__ out,
                                                  int tiles_per_block, int dbg) {
  using G = Ru32<R>;
  constexpr int P = G::P;
  extern __shared__ __align__(16) unsigned char smem[];
  __bf16* const xs = reinterpret_cast<__bf16*>(smem);  // [SPAN][P]: ELU(x) rows t0 - pad ..
  __bf16* const xr = xs + G::SPAN * P;                 // [R][P]: raw x rows t0 .. (the residual)
  const int lane = threadIdx.x & 63, hl = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int span = R + a.pad;
  const int tps = (a.T + R - 1) / R;
  int64_t tile0, tile_end;
  if (!ru_tiles((a.rows / a.T) * tps, tiles_per_block, tile0, tile_end)) return;

  bf16x8 wf[RU_K][2], w2f[1][2];
  ru_wfrags<RU_K>(w1p, wf);
  ru_wfrags<1>(w2p, w2f);
  ws_wait_vm<0>();  // weights landed: the tile loop's waits then count only its own loads

  // both biases staged in LDS once (k_ru64_fwd)
  __shared__ __align__(16) float bsm[2][RU_C];
  if (threadIdx.x < 2 * RU_C) {
    const int i = threadIdx.x;
    const float* bp = i < RU_C ? b1 : b2;
    bsm[i / RU_C][i % RU_C] = bp ? bp[i % RU_C] : 0.f;
  }
  Ru32Stage<R> st;
  st.load(a, x, tile0 / tps, int(tile0 % tps) * R, -a.pad, span);
  ru_dummy_stores<4 * G::TM>(out);  // the loop's h / out stores after each prefetch
  for (int64_t tile = tile0; tile < tile_end; ++tile) {
    const int64_t b = tile / tps;
    const int t0 = int(tile % tps) * R;
    const int mrows = a.T - t0 < R ? a.T - t0 : R;
    __syncthreads();  // every wave is done with the previous tile's rows
    st.store(xs, span, true, xr, a.pad);
    __syncthreads();
    {  // unconditional (a dead request loads nothing): exact counts
      const bool live = tile + 1 < tile_end;
      const int64_t nt = live ? tile + 1 : tile;
      st.load(a, x, nt / tps, int(nt % tps) * R, -a.pad, span, live);
    }
    // every sub-tile computes and stores (rows past T to RU_OOB): a fixed count
    // of stores per tile keeps the next tile's staging wait exact (ru_bstore)
    const __amdgpu_buffer_rsrc_t rh = ru_rsrc(hout + b * a.T * RU_C, int64_t(a.T) * RU_C);
    const __amdgpu_buffer_rsrc_t ro = ru_rsrc(out + b * a.T * RU_C, int64_t(a.T) * RU_C);
#pragma unroll
    for (int i = 0; i < G::TM; ++i) {
      const int lr = wave * (R / 4) + i * 32 + (lane & 31);  // this lane's row in the tile
      const bool valid = lr < mrows;
      const int off = ((t0 + lr) * RU_C + 8 * hl) * 2;
      floatx16 acc;
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[e] = 0.f;
      const __bf16* xw = xs + lr * P + 8 * hl;
#pragma unroll
      for (int k = 0; k < RU_K; ++k)
#pragma unroll
        for (int g = 0; g < 2; ++g)
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[k][g], *reinterpret_cast<const bf16x8*>(xw + k * a.dil * P + 16 * g),
                                                        acc, 0, 0, 0);
      // h = conv1 + b1 -> bf16 -> HBM, ELU(h) -> conv2
      // bias in accumulator order: element group q = channels 8 q + 4 hl .. +4
      float v[16];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const floatx4 bq = *reinterpret_cast<const floatx4*>(&bsm[0][8 * q + 4 * hl]);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[4 * q + e] = acc[4 * q + e] + bq[e];
      }
      bf16x8 hf[2];
      ru_acc_to_frags(v, hf);
      const bool hst = valid && !(dbg & 1);  // tune key 15 bit 0: diagnostic without the h store
      ru_bstore<SEL_RU_FWD_HNT>(rh, hst ? off : RU_OOB, hf[0]);
      ru_bstore<SEL_RU_FWD_HNT>(rh, hst ? off + 32 : RU_OOB, hf[1]);
      floatx16 acc2;
#pragma unroll
      for (int e = 0; e < 16; ++e) acc2[e] = 0.f;
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        const bf16x8 ef = __builtin_bit_cast(bf16x8, elu8(__builtin_bit_cast(uint4, hf[g])));
        acc2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w2f[0][g], ef, acc2, 0, 0, 0);
      }
      // out = conv2 + b2 + x (the residual in accumulator order: 4 runs of 4 channels)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint2 xres = *reinterpret_cast<const uint2*>(xr + lr * P + 8 * q + 4 * hl);
        const __bf16* rv = reinterpret_cast<const __bf16*>(&xres);
        const floatx4 bq = *reinterpret_cast<const floatx4*>(&bsm[1][8 * q + 4 * hl]);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[4 * q + e] = acc2[4 * q + e] + bq[e] + float(rv[e]);
      }
      bf16x8 of[2];
      ru_acc_to_frags(v, of);
      const bool ost = valid && !(dbg & 2);  // bit 1: diagnostic without the out store
      ru_bstore<SEL_RU_FWD_ONT>(ro, ost ? off : RU_OOB, of[0]);
      ru_bstore<SEL_RU_FWD_ONT>(ro, ost ? off + 32 : RU_OOB, of[1]);
    }
  }
}

// k_ru32_fwd at four blocks per CU (tune key 70 = 1; round 6): the conv1
// weights live in LDS (one A-fragment ds_read_b128 per MFMA instead of 56
// VGPRs), ELU(x) rows are 64 B with their 16-B slots XOR-swizzled by
// (row >> 2) & 3 (the 16 rows of every ds_read_b128 lane group hit 16 distinct
// bank groups), and the residual rows are re-read from global memory (staged
// one tile earlier: L2-hot) instead of a raw LDS plane.  35 KB of LDS and at
// most 128 VGPRs: four blocks per CU instead of three keep a third more tiles'
// loads in flight.  Same operands, MFMA order and epilogue as k_ru32_fwd:
// bit-identical.
constexpr int RU4_WP = RU_K * RU_C + 8;  // bf16 pitch of a W1 row in LDS (464 B: conflict-free A reads)
__device__ __forceinline__ int ru4_swz(int row) { return (row >> 2) & 3; }

template <int R>
struct Ru32F4 {
  static constexpr int SPAN = R + F4_HALOMAX;
  static constexpr int TM = R / 128;
  static constexpr size_t LDS = size_t(SPAN) * RU_C * 2 + size_t(RU_C) * RU4_WP * 2;
};

template <int R>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void k_ru32_fwd4(
    Args a, const __bf16* __restrict__ x, const __bf16* __restrict__ w1p, const float* __restrict__ b1,
    const __bf16* __restrict__ w2p, const float* __restrict__ b2, __bf16* __restrict__ hout,
    __bf16* __restrict__ out, int tiles_per_block) {
  using G = Ru32F4<R>;
  extern __shared__ __align__(16) unsigned char smem[];
  __bf16* const xs = reinterpret_cast<__bf16*>(smem);  // [SPAN][32]: ELU(x) rows t0 - pad .., swizzled slots
  __bf16* const wsm = xs + G::SPAN * RU_C;             // [32][RU4_WP]: W1 rows (packed [n][k][c])
  const int lane = threadIdx.x & 63, hl = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int span = R + a.pad;
  const int tps = (a.T + R - 1) / R;
  int64_t tile0, tile_end;
  if (!ru_tiles((a.rows / a.T) * tps, tiles_per_block, tile0, tile_end)) return;

  for (int i = threadIdx.x; i < RU_C * RU_K * RU_C / 8; i += 256) {
    const int n = i / (RU_K * RU_C / 8), r = i % (RU_K * RU_C / 8);
    *reinterpret_cast<uint4*>(wsm + n * RU4_WP + 8 * r) =
        *reinterpret_cast<const uint4*>(w1p + int64_t(n) * RU_K * RU_C + 8 * r);
  }
  bf16x8 w2f[1][2];
  ru_wfrags<1>(w2p, w2f);
  ws_wait_vm<0>();  // weights landed: the tile loop's waits then count only its own loads

  __shared__ __align__(16) float bsm[2][RU_C];
  if (threadIdx.x < 2 * RU_C) {
    const int i = threadIdx.x;
    const float* bp = i < RU_C ? b1 : b2;
    bsm[i / RU_C][i % RU_C] = bp ? bp[i % RU_C] : 0.f;
  }
  const __bf16* const wrow = wsm + (lane & 31) * RU4_WP + 8 * hl;
  Ru32Stage<R> st;
  st.load(a, x, tile0 / tps, int(tile0 % tps) * R, -a.pad, span);
  ru_dummy_stores<4 * G::TM>(out);  // the loop's h / out stores after each prefetch
  for (int64_t tile = tile0; tile < tile_end; ++tile) {
    const int64_t b = tile / tps;
    const int t0 = int(tile % tps) * R;
    const int mrows = a.T - t0 < R ? a.T - t0 : R;
    __syncthreads();  // every wave is done with the previous tile's rows (and W1 / biases staged)
#pragma unroll
    for (int u = 0; u < Ru32<R>::XV; ++u) {
      const int v = threadIdx.x + u * 256;
      const int row = v >> 2, slot = v & 3;
      if (row >= span) continue;
      const uint4 val = elu8(st.ok[u] ? st.r[u] : make_uint4(0, 0, 0, 0));
      *reinterpret_cast<uint4*>(xs + row * RU_C + 8 * (slot ^ ru4_swz(row))) = val;
    }
    __syncthreads();
    {  // unconditional (a dead request loads nothing): exact counts
      const bool live = tile + 1 < tile_end;
      const int64_t nt = live ? tile + 1 : tile;
      st.load(a, x, nt / tps, int(nt % tps) * R, -a.pad, span, live);
    }
    const __amdgpu_buffer_rsrc_t rh = ru_rsrc(hout + b * a.T * RU_C, int64_t(a.T) * RU_C);
    const __amdgpu_buffer_rsrc_t ro = ru_rsrc(out + b * a.T * RU_C, int64_t(a.T) * RU_C);
#pragma unroll
    for (int i = 0; i < G::TM; ++i) {
      const int lr = wave * (R / 4) + i * 32 + (lane & 31);  // this lane's row in the tile
      const bool valid = lr < mrows;
      const int off = ((t0 + lr) * RU_C + 8 * hl) * 2;
      // the residual rows (raw x), requested before conv1: branch-free, clamped row
      const int64_t orow = (b * a.T + t0 + (valid ? lr : 0)) * RU_C;
      uint2 xres[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) xres[q] = *reinterpret_cast<const uint2*>(x + orow + 8 * q + 4 * hl);
      floatx16 acc;
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[e] = 0.f;
#pragma unroll
      for (int k = 0; k < RU_K; ++k) {
        const int row = lr + k * a.dil;
#pragma unroll
        for (int g = 0; g < 2; ++g) {
          const bf16x8 af = *reinterpret_cast<const bf16x8*>(wrow + k * RU_C + 16 * g);
          const bf16x8 bf = *reinterpret_cast<const bf16x8*>(xs + row * RU_C + 8 * ((2 * g + hl) ^ ru4_swz(row)));
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bf, acc, 0, 0, 0);
        }
      }
      float v[16];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const floatx4 bq = *reinterpret_cast<const floatx4*>(&bsm[0][8 * q + 4 * hl]);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[4 * q + e] = acc[4 * q + e] + bq[e];
      }
      bf16x8 hf[2];
      ru_acc_to_frags(v, hf);
      ru_bstore<SEL_RU_FWD_HNT>(rh, valid ? off : RU_OOB, hf[0]);
      ru_bstore<SEL_RU_FWD_HNT>(rh, valid ? off + 32 : RU_OOB, hf[1]);
      floatx16 acc2;
#pragma unroll
      for (int e = 0; e < 16; ++e) acc2[e] = 0.f;
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        const bf16x8 ef = __builtin_bit_cast(bf16x8, elu8(__builtin_bit_cast(uint4, hf[g])));
        acc2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w2f[0][g], ef, acc2, 0, 0, 0);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const __bf16* rv = reinterpret_cast<const __bf16*>(&xres[q]);
        const floatx4 bq = *reinterpret_cast<const floatx4*>(&bsm[1][8 * q + 4 * hl]);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[4 * q + e] = acc2[4 * q + e] + bq[e] + float(rv[e]);
      }
      bf16x8 of[2];
      ru_acc_to_frags(v, of);
      ru_bstore<SEL_RU_FWD_ONT>(ro, valid ? off : RU_OOB, of[0]);
      ru_bstore<SEL_RU_FWD_ONT>(ro, valid ? off + 32 : RU_OOB, of[1]);
    }
  }
}

// Residual unit at 64 channels, forward in ONE launch (round 3): the 32-channel
// scheme with the 1x1 still fed from registers, but a wave computes conv1 for
// one 32-channel output slice only (all 64 x 7 input fragments of its slice in
// VGPRs, as k_conv_thin_bf16), so the 1x1 (all 64 h channels of a row) needs
// the partner wave's slice: each wave writes ELU(bf16(h)) of its rows and slice
// to a [2][R][P] LDS tile in the 1x1's B-fragment order, one block barrier, and
// every wave reads its four fragments back.  Waves = 2 row groups x 2 slices.
// h and out leave from the re-laid-out fragments as 16-B stores; the residual
// rows (raw x) are requested before conv1 (L2-hot: the tile was just staged).
// Same MFMA order, rounding points and epilogue arithmetic as the two thin
// launches (k7 then 1x1), so the results are bit-identical to them.
template <int R>
struct Ru64 {
  static constexpr int C = 64, K = 7, P = F4_P;
  static constexpr int SPAN = R + F4_HALOMAX;
  static constexpr int CV = C / 8;
  static constexpr int XV = (SPAN * CV + 255) / 256;
  static constexpr int WR = R / 2;  // rows per row group
  static constexpr int TM = WR / 32;
  // ELU(x) span planes + ELU(h) planes + raw x tile planes (the residual)
  static constexpr size_t LDS = size_t(2) * (SPAN + 2 * R) * P * 2;
  static_assert(R % 64 == 0, "ru64 tile rows");
};

template <int R>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(SEL_W_RU64F))) void k_ru64_fwd(Args a, const __bf16* __restrict__ x,
                                                  const __bf16* __restrict__ w1p, const float* __restrict__ b1,
                                                  const __bf16* __restrict__ w2p, const float* __restrict__ b2,
                                                  __bf16* __restrict__ hout, __bf16* __restrict__ out,
                                                  int tiles_per_block) {
  using G = Ru64<R>;
  constexpr int P = G::P, C = G::C, K = G::K, CV = G::CV;
  extern __shared__ __align__(16) unsigned char smem[];
  __bf16* const xs = reinterpret_cast<__bf16*>(smem);  // [2][SPAN][P]: ELU(x) rows t0 - pad ..
  __bf16* const hs = xs + 2 * G::SPAN * P;             // [2][R][P]: ELU(h) rows t0 ..
  __bf16* const xraw = hs + 2 * R * P;                 // [2][R][P]: raw x rows t0 .. (the residual)
  const int tid = threadIdx.x, lane = tid & 63, hl = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ns = wave & 1, rg = wave >> 1;
  const int span = R + a.pad;
  const int tps = (a.T + R - 1) / R;
  int64_t tile0, tile_end;
  if (!ru_tiles((a.rows / a.T) * tps, tiles_per_block, tile0, tile_end)) return;

  bf16x8 wf[K][C / 16], wf2[C / 16];
  {
    const __bf16* wrow = w1p + int64_t(ns * 32 + (lane & 31)) * K * C + 8 * hl;
#pragma unroll
    for (int k = 0; k < K; ++k)
#pragma unroll
      for (int g = 0; g < C / 16; ++g) wf[k][g] = *reinterpret_cast<const bf16x8*>(wrow + k * C + 16 * g);
    const __bf16* wrow2 = w2p + int64_t(ns * 32 + (lane & 31)) * C + 8 * hl;
#pragma unroll
    for (int g = 0; g < C / 16; ++g) wf2[g] = *reinterpret_cast<const bf16x8*>(wrow2 + 16 * g);
  }
  ws_wait_vm<0>();  // weights landed: the tile loop's waits then count only its own loads
  // biases in accumulator order (element group q = channels ns*32 + 8q + 4hl .. +4),
  // read where used (L1-hot; registers are what bounds this kernel's occupancy)
  // both biases staged in LDS once (zeros when absent): a global bias load in
  // the tile loop would wait behind the next tile's prefetch (memory counters
  // retire in order)
  __shared__ __align__(16) float bsm[2][C];
  for (int i = tid; i < 2 * C; i += 256) {
    const float* bp = i < C ? b1 : b2;
    bsm[i / C][i % C] = bp ? bp[i % C] : 0.f;
  }
  auto bias_q = [&](int which, int q) { return *reinterpret_cast<const floatx4*>(&bsm[which][ns * 32 + 8 * q + 4 * hl]); };

  uint4 xr[G::XV];
  bool xok[G::XV];
  auto load = [&](int64_t tile, bool live) {
    const int64_t b = tile / tps;
    const int t0 = int(tile % tps) * R;
    const __amdgpu_buffer_rsrc_t rs = ru_rsrc(x + b * a.T * C, int64_t(a.T) * C);
#pragma unroll
    for (int u = 0; u < G::XV; ++u) {
      const int v = tid + u * 256;
      const int r = v / CV, c = (v % CV) * 8;
      const int ti = t0 - a.pad + r;
      xok[u] = r < span && ti >= 0 && ti < a.T;
      xr[u] = ru_bload(rs, live && xok[u] ? (ti * C + c) * 2 : RU_OOB);  // Ru32Stage::load
      __builtin_amdgcn_sched_barrier(0);  // program order pinned (Ru32Stage::load)
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int u = 0; u < G::XV; ++u) {
      const int v = tid + u * 256;
      const int r = v / CV, c = (v % CV) * 8;
      if (r >= span) continue;
      const uint4 raw = xok[u] ? xr[u] : make_uint4(0, 0, 0, 0);
      if (r >= a.pad && r < a.pad + R) *reinterpret_cast<uint4*>(xraw + ((c >> 5) * R + r - a.pad) * P + (c & 31)) = raw;
      *reinterpret_cast<uint4*>(xs + ((c >> 5) * G::SPAN + r) * P + (c & 31)) = elu8(raw);
    }
  };

  load(tile0, true);
  ru_dummy_stores<4 * G::TM>(out);  // the loop's h / out stores after each prefetch
  for (int64_t tile = tile0; tile < tile_end; ++tile) {
    const int64_t b = tile / tps;
    const int t0 = int(tile % tps) * R;
    const int mrows = a.T - t0 < R ? a.T - t0 : R;
    __syncthreads();  // every wave is done with the previous tile's xs / hs
    store();
    __syncthreads();
    // the next tile's rows (no other global load in the tile loop: the
    // residual rows come from the staged raw planes)
    load(tile + 1 < tile_end ? tile + 1 : tile, tile + 1 < tile_end);  // unconditional: exact counts

    // conv1 (k_conv_thin_bf16 order: taps, 16-channel chunks, sub-tiles)
    floatx16 acc[G::TM];
#pragma unroll
    for (int i = 0; i < G::TM; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][e] = 0.f;
    const __bf16* xw = xs + (rg * G::WR + (lane & 31)) * P + 8 * hl;
#pragma unroll
    for (int k = 0; k < K; ++k)
#pragma unroll
      for (int g = 0; g < C / 16; ++g) {
        const __bf16* xb = xw + ((g >> 1) * G::SPAN + k * a.dil) * P + 16 * (g & 1);
#pragma unroll
        for (int i = 0; i < G::TM; ++i)
          acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[k][g], *reinterpret_cast<const bf16x8*>(xb + i * 32 * P),
                                                           acc[i], 0, 0, 0);
      }
    // every sub-tile stores (rows past T to RU_OOB): a fixed count of stores per
    // tile keeps the next tile's staging wait exact (ru_bstore)
    const __amdgpu_buffer_rsrc_t rh = ru_rsrc(hout + b * a.T * C, int64_t(a.T) * C);
    const __amdgpu_buffer_rsrc_t ro = ru_rsrc(out + b * a.T * C, int64_t(a.T) * C);
    // h = conv1 + b1 -> bf16 -> HBM; ELU(h) -> the 1x1's LDS tile (plane ns)
#pragma unroll
    for (int i = 0; i < G::TM; ++i) {
      const int lr = rg * G::WR + i * 32 + (lane & 31);
      float v[16];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const floatx4 bq = bias_q(0, q);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[4 * q + e] = acc[i][4 * q + e] + bq[e];
      }
      bf16x8 hf[2];
      ru_acc_to_frags(v, hf);
      const int off = ((t0 + lr) * C + ns * 32 + 8 * hl) * 2;
      // (plain stores: nt on these h rows, whose 128-B lines the two
      // channel-slice waves write in halves, measured 60 -> 79 us)
      ru_bstore(rh, lr < mrows ? off : RU_OOB, hf[0]);
      ru_bstore(rh, lr < mrows ? off + 32 : RU_OOB, hf[1]);
#pragma unroll
      for (int g = 0; g < 2; ++g)
        *reinterpret_cast<uint4*>(hs + (ns * R + lr) * P + 16 * g + 8 * hl) = elu8(__builtin_bit_cast(uint4, hf[g]));
    }
    __syncthreads();
    // out = x + conv2(ELU(h)) + b2 (k_conv_thin_bf16 epilogue order: + bias, then the residual)
#pragma unroll
    for (int i = 0; i < G::TM; ++i) {
      const int lr = rg * G::WR + i * 32 + (lane & 31);
      floatx16 acc2;
#pragma unroll
      for (int e = 0; e < 16; ++e) acc2[e] = 0.f;
      const __bf16* hw = hs + lr * P + 8 * hl;
#pragma unroll
      for (int g = 0; g < C / 16; ++g)
        acc2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf2[g], *reinterpret_cast<const bf16x8*>(hw + (g >> 1) * R * P + 16 * (g & 1)),
                                                       acc2, 0, 0, 0);
      float v[16];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint2 xres = *reinterpret_cast<const uint2*>(xraw + (ns * R + lr) * P + 8 * q + 4 * hl);
        const __bf16* rv = reinterpret_cast<const __bf16*>(&xres);
        const floatx4 bq = bias_q(1, q);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[4 * q + e] = __fadd_rn(acc2[4 * q + e] + bq[e], float(rv[e]));
      }
      bf16x8 of[2];
      ru_acc_to_frags(v, of);
      const int off = ((t0 + lr) * C + ns * 32 + 8 * hl) * 2;
      ru_bstore(ro, lr < mrows ? off : RU_OOB, of[0]);
      ru_bstore(ro, lr < mrows ? off + 32 : RU_OOB, of[1]);
    }
  }
}

// Residual unit at 64 channels, backward in ONE launch (the k_ru32_bwd scheme
// with 32-channel output slices per wave, as k_ru64_fwd): g (grad of out) is
// staged over the tile + anti-causal halo; gh = (W2^T g) * ELU'(h) per (32-row
// sub-tile, slice) into a [2][SPAN][P] LDS tile (and HBM for the weight
// gradient); after one barrier gx = conv1^T(gh) * ELU'(x) + g per (row group,
// slice) from the dgrad-packed weights in VGPRs.  Same MFMA order, rounding
// points and epilogue arithmetic as the two thin adjoint launches (1x1 with
// ELU'(h), then k7 with ELU'(x) + g): bit-identical to them.
template <int R>
struct Ru64B {
  static constexpr int C = 64, K = 7, P = F4_P;
  static constexpr int SPAN = R + F4_HALOMAX;
  static constexpr int CV = C / 8;
  static constexpr int XV = (SPAN * CV + 255) / 256;
  static constexpr int WR = R / 2;
  static constexpr int TM = WR / 32;
  static constexpr int NSUBMAX = (SPAN + 31) / 32;
  static constexpr int UPW = (NSUBMAX * 2 + 3) / 4;  // gh (sub-tile, slice) units per wave
  static constexpr size_t LDS = size_t(4) * SPAN * P * 2;  // g planes + gh planes
};

template <int R>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(SEL_W_RU64B))) void k_ru64_bwd(
    Args a, const __bf16* __restrict__ g, const __bf16* __restrict__ h, const __bf16* __restrict__ x,
    const __bf16* __restrict__ wd1, const __bf16* __restrict__ wd2, __bf16* __restrict__ ghout,
    __bf16* __restrict__ gx, int tiles_per_block) {
  using G = Ru64B<R>;
  constexpr int P = G::P, C = G::C, K = G::K, CV = G::CV;
  extern __shared__ __align__(16) unsigned char smem[];
  __bf16* const gs = reinterpret_cast<__bf16*>(smem);  // [2][SPAN][P]: g rows t0 ..
  __bf16* const ghs = gs + 2 * G::SPAN * P;            // [2][SPAN][P]: gh rows t0 ..
  const int tid = threadIdx.x, lane = tid & 63, hl = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ns = wave & 1, rg = wave >> 1;
  const int halo = (K - 1) * a.dil;
  const int span = R + halo;
  const int nsub = (span + 31) / 32;
  const int tps = (a.T + R - 1) / R;
  int64_t tile0, tile_end;
  if (!ru_tiles((a.rows / a.T) * tps, tiles_per_block, tile0, tile_end)) return;

  bf16x8 wf[K][C / 16];  // the 1x1 adjoint's fragments are read per gh unit (L1-hot)
  {
    const __bf16* wrow = wd1 + int64_t(ns * 32 + (lane & 31)) * K * C + 8 * hl;
#pragma unroll
    for (int k = 0; k < K; ++k)
#pragma unroll
      for (int q = 0; q < C / 16; ++q) wf[k][q] = *reinterpret_cast<const bf16x8*>(wrow + k * C + 16 * q);
  }
  // the 1x1 adjoint's weights [C][C] in LDS (rows padded to W2P: 16-B reads of
  // 32 rows x 2 lane halves spread over the banks); a per-unit global load in
  // the gh phase waited behind every request before it (memory counters
  // retire in order)
  constexpr int W2P = C + 8;
  __shared__ __align__(16) __bf16 w2s[C * W2P];
  for (int i = tid; i < C * C / 8; i += 256) {
    const int n = i / (C / 8), c8 = (i % (C / 8)) * 8;
    *reinterpret_cast<bf16x8*>(w2s + n * W2P + c8) = *reinterpret_cast<const bf16x8*>(wd2 + int64_t(n) * C + c8);
  }
  ws_wait_vm<0>();  // weights landed: the tile loop's waits then count only its own loads

  uint4 xr[G::XV];
  bool xok[G::XV];
  auto load = [&](int64_t tile, bool live) {  // g rows t0 .. t0 + span (rows >= T: zero; Ru32Stage::load)
    const int64_t b = tile / tps;
    const int t0 = int(tile % tps) * R;
    const __amdgpu_buffer_rsrc_t rs = ru_rsrc(g + b * a.T * C, int64_t(a.T) * C);
#pragma unroll
    for (int u = 0; u < G::XV; ++u) {
      const int v = tid + u * 256;
      const int r = v / CV, c = (v % CV) * 8;
      const int ti = t0 + r;
      xok[u] = r < span && ti < a.T;
      xr[u] = ru_bload(rs, live && xok[u] ? (ti * C + c) * 2 : RU_OOB);
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int u = 0; u < G::XV; ++u) {
      const int v = tid + u * 256;
      const int r = v / CV, c = (v % CV) * 8;
      if (r >= span) continue;
      *reinterpret_cast<uint4*>(gs + ((c >> 5) * G::SPAN + r) * P + (c & 31)) = xok[u] ? xr[u] : make_uint4(0, 0, 0, 0);
    }
  };

  load(tile0, true);
  for (int64_t tile = tile0; tile < tile_end; ++tile) {
    const int64_t b = tile / tps;
    const int t0 = int(tile % tps) * R;
    const int mrows = a.T - t0 < R ? a.T - t0 : R;
    __syncthreads();  // every wave is done with the previous tile's gs / ghs
    store();
    __syncthreads();
    // h rows of a gh unit (the ELU'(h) factor), one unit ahead of its MFMAs
    auto load_h = [&](int unit, uint2 (&hq)[4]) {
      const int sb = unit >> 1, sl = unit & 1;
      const int ti = t0 + sb * 32 + (lane & 31);
      const bool inside = unit < 2 * nsub && ti < a.T;
      const int64_t orow = (b * a.T + (inside ? ti : 0)) * C + sl * 32;
#pragma unroll
      for (int q = 0; q < 4; ++q)
        hq[q] = inside ? *reinterpret_cast<const uint2*>(h + orow + 8 * q + 4 * hl) : make_uint2(0, 0);
    };
    // every gh unit's h rows requested up front (one latency per tile, not one per unit)
    uint2 hall[G::UPW][4];
#pragma unroll
    for (int uu = 0; uu < G::UPW; ++uu) load_h(wave + 4 * uu, hall[uu]);
    // x rows of this wave's gx sub-tiles (the ELU'(x) factor), requested before
    // the gh phase so their HBM latency hides behind it
    uint2 xpre[G::TM][4];
#pragma unroll
    for (int i = 0; i < G::TM; ++i) {
      const int lr = rg * G::WR + i * 32 + (lane & 31);
      const bool in = lr < mrows;
      const int64_t orow = (b * a.T + t0 + (in ? lr : 0)) * C + ns * 32 + 4 * hl;
#pragma unroll
      for (int q = 0; q < 4; ++q) xpre[i][q] = in ? *reinterpret_cast<const uint2*>(x + orow + 8 * q) : make_uint2(0, 0);
    }

    // gh = (W2^T g) * ELU'(h), units u = (sub-tile, slice) round-robin over the waves
#pragma unroll
    for (int uu = 0; uu < G::UPW; ++uu) {
      const int unit = wave + 4 * uu;
      if (unit >= 2 * nsub) break;  // wave-uniform
      const int sb = unit >> 1, sl = unit & 1;
      const int lr = sb * 32 + (lane & 31);
      const int ti = t0 + lr;
      const bool inside = ti < a.T;
      const int64_t orow = (b * a.T + (inside ? ti : 0)) * C + sl * 32;
      uint2 hq[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) hq[q] = hall[uu][q];
      // the slice-sl weights of the 1x1 adjoint: rows n = sl*32 + (lane & 31), from LDS
      bf16x8 w2q[C / 16];
      {
        const __bf16* wr2 = w2s + (sl * 32 + (lane & 31)) * W2P + 8 * hl;
#pragma unroll
        for (int q = 0; q < C / 16; ++q) w2q[q] = *reinterpret_cast<const bf16x8*>(wr2 + 16 * q);
      }
      floatx16 acc;
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[e] = 0.f;
      const __bf16* gw = gs + lr * P + 8 * hl;
#pragma unroll
      for (int q = 0; q < C / 16; ++q)
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w2q[q], *reinterpret_cast<const bf16x8*>(gw + (q >> 1) * G::SPAN * P + 16 * (q & 1)),
                                                      acc, 0, 0, 0);
      float v[16];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const __bf16* hv = reinterpret_cast<const __bf16*>(&hq[q]);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[4 * q + e] = __fmul_rn(acc[4 * q + e], elu_grad_fast(float(hv[e])));
      }
      bf16x8 ghf[2];
      ru_acc_to_frags(v, ghf);
      if (lr < span) {
        *reinterpret_cast<bf16x8*>(ghs + (sl * G::SPAN + lr) * P + 8 * hl) = ghf[0];
        *reinterpret_cast<bf16x8*>(ghs + (sl * G::SPAN + lr) * P + 16 + 8 * hl) = ghf[1];
      }
      if (ghout && lr < mrows) {
        ru_store(ghout + orow + 8 * hl, ghf[0]);
        ru_store(ghout + orow + 16 + 8 * hl, ghf[1]);
      }
    }
    __syncthreads();
    // the next tile's g rows, requested after the gh phase: its h / x / weight
    // loads then wait only for each other (memory counters retire in order),
    // and this request has the gx phase to land
    load(tile + 1 < tile_end ? tile + 1 : tile, tile + 1 < tile_end);  // unconditional: exact counts
    // gx = conv1^T(gh) * ELU'(x) + g (k_conv_thin_bf16 order: taps, chunks, sub-tiles)
    floatx16 acc[G::TM];
#pragma unroll
    for (int i = 0; i < G::TM; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][e] = 0.f;
    const __bf16* hw = ghs + (rg * G::WR + (lane & 31)) * P + 8 * hl;
#pragma unroll
    for (int k = 0; k < K; ++k)
#pragma unroll
      for (int q = 0; q < C / 16; ++q) {
        const __bf16* hb = hw + ((q >> 1) * G::SPAN + k * a.dil) * P + 16 * (q & 1);
#pragma unroll
        for (int i = 0; i < G::TM; ++i)
          acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[k][q], *reinterpret_cast<const bf16x8*>(hb + i * 32 * P),
                                                           acc[i], 0, 0, 0);
      }
#pragma unroll
    for (int i = 0; i < G::TM; ++i) {
      const int lr = rg * G::WR + i * 32 + (lane & 31);
      if (__builtin_amdgcn_readfirstlane(rg * G::WR + i * 32) >= mrows) break;
      const bool valid = lr < mrows;
      const int64_t orow = (b * a.T + t0 + (valid ? lr : 0)) * C + ns * 32;
      float v[16];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint2 graw = *reinterpret_cast<const uint2*>(gs + (ns * G::SPAN + lr) * P + 8 * q + 4 * hl);
        const __bf16* xv = reinterpret_cast<const __bf16*>(&xpre[i][q]);
        const __bf16* gv = reinterpret_cast<const __bf16*>(&graw);
#pragma unroll
        for (int e = 0; e < 4; ++e)
          v[4 * q + e] = __fadd_rn(__fmul_rn(acc[i][4 * q + e], elu_grad_fast(float(xv[e]))), float(gv[e]));
      }
      bf16x8 of[2];
      ru_acc_to_frags(v, of);
      if (valid) {
        ru_store(gx + orow + 8 * hl, of[0]);
        ru_store(gx + orow + 16 + 8 * hl, of[1]);
      }
    }
  }
}

// Backward: gh = (W2^T g) * ELU'(h) over the tile + its anti-causal halo (the
// adjoint of the causal conv reads rows t .. t + 6 dil), in registers -> LDS
// (and HBM when the weight gradient needs it); gx = conv1^T(gh) * ELU'(x) + g.
// wd1 / wd2 are the dgrad-packed weights of the primitive path.
template <int R>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(R == 128 ? SEL_W_RU32B : 1))) void k_ru32_bwd(Args a, const __bf16* __restrict__ g,
                                                  const __bf16* __restrict__ h, const __bf16* __restrict__ x,
                                                  const __bf16* __restrict__ wd1, const __bf16* __restrict__ wd2,
                                                  __bf16* __restrict__ ghout, __bf16* __restrict__ gx,
                                                  int tiles_per_block) {
  using G = Ru32<R>;
  constexpr int P = G::P;
  extern __shared__ __align__(16) unsigned char smem[];
  __bf16* const gs = reinterpret_cast<__bf16*>(smem);  // [SPAN][P]: g rows t0 ..
  __bf16* const ghs = gs + G::SPAN * P;                // [SPAN][P]: gh rows t0 ..
  __bf16* const hs = ghs + G::SPAN * P;                // [SPAN][P]: h rows t0 .. (the ELU'(h) factor)
  const int lane = threadIdx.x & 63, hl = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int halo = (RU_K - 1) * a.dil;
  const int span = R + halo;
  const int nsub = (span + 31) / 32;  // gh sub-tiles (tile + halo)
  const int tps = (a.T + R - 1) / R;
  int64_t tile0, tile_end;
  if (!ru_tiles((a.rows / a.T) * tps, tiles_per_block, tile0, tile_end)) return;

  bf16x8 wf[RU_K][2], w2f[1][2];
  ru_wfrags<RU_K>(wd1, wf);
  ru_wfrags<1>(wd2, w2f);
  ws_wait_vm<0>();  // weights landed: the tile loop's waits then count only its own loads

  // g and h rows staged one tile ahead (k_ru32_bwdw): the gh phase reads h from
  // LDS instead of waiting on a request made at the top of the tile
  Ru32Stage<R> st, sh;
  st.load(a, g, tile0 / tps, int(tile0 % tps) * R, 0, span);
  sh.load(a, h, tile0 / tps, int(tile0 % tps) * R, 0, span);
  ru_dummy_stores<2 * G::TM>(gx);  // the loop's gx stores after each prefetch
  for (int64_t tile = tile0; tile < tile_end; ++tile) {
    const int64_t b = tile / tps;
    const int t0 = int(tile % tps) * R;
    const int mrows = a.T - t0 < R ? a.T - t0 : R;
    __syncthreads();  // every wave is done with the previous tile's g / gh rows
    st.store(gs, span, false);
    sh.store(hs, span, false);
    __syncthreads();
    // the x rows of this wave's gx sub-tiles (ELU'(x)), requested up front (their
    // latency hides behind the gh phase)
    constexpr int NSUB_W = (G::SPAN / 32 + 3) / 4;  // gh sub-tiles per wave (max)
    uint2 xpre[G::TM][4];
#pragma unroll
    for (int i = 0; i < G::TM; ++i) {
      const int lr = wave * (R / 4) + i * 32 + (lane & 31);
      const bool in = lr < mrows;
      const int64_t orow = (b * a.T + t0 + (in ? lr : 0)) * RU_C;
#pragma unroll
      for (int q = 0; q < 4; ++q) xpre[i][q] = in ? *reinterpret_cast<const uint2*>(x + orow + 8 * q + 4 * hl) : make_uint2(0, 0);
    }
    // gh for rows t0 .. t0 + span (rows >= T: g staged as zero -> gh = 0)
#pragma unroll
    for (int j = 0; j < NSUB_W; ++j) {
      const int sb = wave + 4 * j;
      if (sb >= nsub) break;
      const int lr = sb * 32 + (lane & 31);
      floatx16 acc;
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[e] = 0.f;
      const __bf16* gw = gs + lr * P + 8 * hl;
#pragma unroll
      for (int c = 0; c < 2; ++c)
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w2f[0][c], *reinterpret_cast<const bf16x8*>(gw + 16 * c), acc, 0, 0, 0);
      const int ti = t0 + lr;
      const bool inside = ti < a.T;
      const int64_t orow = (b * a.T + (inside ? ti : 0)) * RU_C;
      uint2 hq[4];  // h rows (zero past T), as staged
#pragma unroll
      for (int q = 0; q < 4; ++q) hq[q] = *reinterpret_cast<const uint2*>(hs + lr * P + 8 * q + 4 * hl);
      float v[16];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const __bf16* hv = reinterpret_cast<const __bf16*>(&hq[q]);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[4 * q + e] = acc[4 * q + e] * elu_grad_fast(float(hv[e]));
      }
      bf16x8 ghf[2];
      ru_acc_to_frags(v, ghf);
      if (lr < span) {
        *reinterpret_cast<bf16x8*>(ghs + lr * P + 8 * hl) = ghf[0];
        *reinterpret_cast<bf16x8*>(ghs + lr * P + 16 + 8 * hl) = ghf[1];
      }
      if (ghout && lr < mrows) {
        ru_store(ghout + orow + 8 * hl, ghf[0]);
        ru_store(ghout + orow + 16 + 8 * hl, ghf[1]);
      }
    }
    __syncthreads();
    // the next tile's g rows, requested after the gh phase (k_ru64_bwd)
    {  // unconditional (a dead request loads nothing): exact counts
      const bool live = tile + 1 < tile_end;
      const int64_t nt = live ? tile + 1 : tile;
      st.load(a, g, nt / tps, int(nt % tps) * R, 0, span, live);
      sh.load(a, h, nt / tps, int(nt % tps) * R, 0, span, live);
    }
    // every sub-tile stores (rows past T to RU_OOB): a fixed count of stores per
    // tile keeps the next tile's staging waits exact (ru_bstore)
    const __amdgpu_buffer_rsrc_t rgx = ru_rsrc(gx + b * a.T * RU_C, int64_t(a.T) * RU_C);
#pragma unroll
    for (int i = 0; i < G::TM; ++i) {
      const int lr = wave * (R / 4) + i * 32 + (lane & 31);
      floatx16 acc;
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[e] = 0.f;
      const __bf16* hw = ghs + lr * P + 8 * hl;
#pragma unroll
      for (int k = 0; k < RU_K; ++k)
#pragma unroll
        for (int c = 0; c < 2; ++c)
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[k][c], *reinterpret_cast<const bf16x8*>(hw + k * a.dil * P + 16 * c),
                                                        acc, 0, 0, 0);
      const bool valid = lr < mrows;
      float v[16];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint2 graw = *reinterpret_cast<const uint2*>(gs + lr * P + 8 * q + 4 * hl);
        const __bf16* xv = reinterpret_cast<const __bf16*>(&xpre[i][q]);
        const __bf16* gv = reinterpret_cast<const __bf16*>(&graw);
#pragma unroll
        for (int e = 0; e < 4; ++e)
          v[4 * q + e] = __fadd_rn(__fmul_rn(acc[4 * q + e], elu_grad_fast(float(xv[e]))), float(gv[e]));
      }
      bf16x8 of[2];
      ru_acc_to_frags(v, of);
      const int off = ((t0 + lr) * RU_C + 8 * hl) * 2;
      ru_bstore<SEL_RU32B_GXNT>(rgx, valid ? off : RU_OOB, of[0]);
      ru_bstore<SEL_RU32B_GXNT>(rgx, valid ? off + 32 : RU_OOB, of[1]);
    }
  }
}

// ---------------------------------------------------------------------------
// Single-input-channel layers (the encoder's first conv 1->32 k7, and the dgrad
// of the decoder's last conv 32->1 k7): an implicit GEMM with a reduction of
// only K taps would leave MFMA idle and stage a 1-wide tile, so this is a
// streaming kernel instead: one output row per thread, K input samples, N x K
// FMAs against LDS-broadcast weights, 16-B vector stores of the N outputs.
// ---------------------------------------------------------------------------
constexpr int C1_NMAX = 64;
constexpr int C1_KMAX = 8;
constexpr int C1_TR = 256;    // rows per sample-aligned tile (weight gradient)
// rows per tile of the forward kernel: 768 (round 6; was 1024).  One resident
// round is 1024 workgroups at C3: 64 x 24000 rows in 1024-row tiles are 1536
// tiles, so half the workgroups ran two and the launch took two tile times;
// 768-row tiles are 2048 tiles, two per workgroup, 1.5 (1024-row) tile times
constexpr int C1F_TR = 768;
constexpr int C1_HALO = 64;   // max (K-1)*dil

// Stage act(x) for input times [t0 - pad, t0 - pad + C1_TR + halo) of sample b as
// fp32 in LDS, causal zero / replicate padding resolved here.
__device__ __forceinline__ void c1_stage(const Args& a, const __bf16* __restrict__ in, int64_t b, int t0,
                                         float* xs) {
  const int span = C1_TR + (a.K - 1) * a.dil;
  for (int r = threadIdx.x; r < span; r += 256) {
    int ti = t0 - a.pad + r;
    const bool inside = ti >= 0 && ti < a.T;
    const bool ok = inside || a.pad_mode == SEL_PAD_REPLICATE;
    ti = ti < 0 ? 0 : (ti >= a.T ? a.T - 1 : ti);
    const float v = float(in[b * a.T + ti]);
    xs[r] = ok ? (a.in_elu ? elu_fast(v) : v) : 0.f;
  }
}

// Thread = (8-wide output group g, row lane rl): its 8 x K weights live in
// registers; per row it reads K staged samples and writes one 16-B vector, the
// NG lanes of a row together writing the row's contiguous N outputs.
// TI = float (the reference-precision path): exact expm1 / exp in the ELU and
// ELU' (the bf16 build rounds its result to bf16 and uses the hardware exp)
template <typename TI>
__device__ __forceinline__ float c1_act(float v) {
  if constexpr (sizeof(TI) == 4) return elu(v);
  else return elu_fast(v);
}
template <typename TI>
__device__ __forceinline__ float c1_act_grad(float v) {
  if constexpr (sizeof(TI) == 4) return elu_grad(v);
  else return elu_grad_fast(v);
}
template <typename TI, typename TO, int TR>
__global__ __launch_bounds__(256) void k_conv_c1(Args a, const TI* __restrict__ in,
                                                 const TI* __restrict__ wp, const float* __restrict__ bias,
                                                 const TO* __restrict__ aux, const TO* __restrict__ res,
                                                 TO* __restrict__ out) {
  __shared__ float xs[TR + C1_HALO];
  constexpr int PV = (TR + C1_HALO + 255) / 256;  // staged samples per thread
  constexpr int V = Vec16<TO>::n;  // outputs per vector store (8 bf16 / 4 fp32)
  const int NG = a.N / V;
  const int tid = threadIdx.x, grp = tid % NG, rl = tid / NG, nrl = 256 / NG;
  float w[V][C1_KMAX], bs[V];
#pragma unroll
  for (int e = 0; e < V; ++e) {
    const int n = grp * V + e;
    bs[e] = (bias && a.bias_period) ? bias[n % a.bias_period] : 0.f;
#pragma unroll
    for (int k = 0; k < C1_KMAX; ++k) w[e][k] = k < a.K ? to_f(wp[n * a.K + k]) : 0.f;
  }
  const int tps = (a.T + TR - 1) / TR;
  const int64_t ntiles = (a.rows / a.T) * tps;
  // the next tile's samples are fetched into registers while this tile is
  // computed and stored (one resident round of workgroups walks the tiles)
  const int span = TR + (a.K - 1) * a.dil;
  float pre[PV];
  auto fetch = [&](int64_t tile) {
    const int64_t b = tile / tps;
    const int t0 = int(tile % tps) * TR;
#pragma unroll
    for (int u = 0; u < PV; ++u) {
      const int r = threadIdx.x + 256 * u;
      int ti = t0 - a.pad + r;
      const bool ok = r < span && ((ti >= 0 && ti < a.T) || a.pad_mode == SEL_PAD_REPLICATE);
      ti = ti < 0 ? 0 : (ti >= a.T ? a.T - 1 : ti);
      const float v = ok ? to_f(in[b * a.T + ti]) : 0.f;
      pre[u] = ok && a.in_elu ? c1_act<TI>(v) : v;
    }
  };
  if (int64_t(blockIdx.x) < ntiles) fetch(blockIdx.x);
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int64_t b = tile / tps;
    const int t0 = int(tile % tps) * TR;
    __syncthreads();
#pragma unroll
    for (int u = 0; u < PV; ++u)
      if (threadIdx.x + 256 * u < span) xs[threadIdx.x + 256 * u] = pre[u];
    __syncthreads();
    if (tile + gridDim.x < ntiles) fetch(tile + gridDim.x);
    const int rows = a.T - t0 < TR ? a.T - t0 : TR;
    for (int r = rl; r < rows; r += nrl) {
      float v[V];
#pragma unroll
      for (int e = 0; e < V; ++e) v[e] = bs[e];
#pragma unroll
      for (int k = 0; k < C1_KMAX; ++k) {
        if (k >= a.K) break;
        const float x = xs[r + k * a.dil];
#pragma unroll
        for (int e = 0; e < V; ++e) v[e] = fmaf(w[e][k], x, v[e]);
      }
      const int64_t o = (b * a.T + t0 + r) * a.N + grp * V;
      if (aux) {
        TO av[V];
        *reinterpret_cast<uint4*>(av) = *reinterpret_cast<const uint4*>(aux + o);
#pragma unroll
        for (int e = 0; e < V; ++e) v[e] *= c1_act_grad<TI>(to_f(av[e]));
      }
      if (res) {
        TO rv[V];
        *reinterpret_cast<uint4*>(rv) = *reinterpret_cast<const uint4*>(res + o);
#pragma unroll
        for (int e = 0; e < V; ++e) v[e] += to_f(rv[e]);
      }
      TO ov[V];
#pragma unroll
      for (int e = 0; e < V; ++e) ov[e] = from_f<TO>(v[e]);
      *reinterpret_cast<uint4*>(out + o) = *reinterpret_cast<uint4*>(ov);
    }
  }
}

// Weight gradient of a single-input-channel layer: gWp[n][k] = sum_m g[m][n] *
// act(x[row(m, k)]) and the bias sums.  Thread = (8-wide n group, row lane);
// each block walks its contiguous range of sample-aligned 256-row tiles with the
// samples staged in LDS, then reduces its lanes (shuffles, LDS over waves) into
// one partial per block.
// 8 consecutive gout values of one row: one 16-B load (bf16) or two (fp32)
struct F8 {
  float4 lo, hi;
};
template <typename TI> struct G8;
template <> struct G8<__bf16> {
  using type = uint4;
  static __device__ __forceinline__ type load(const __bf16* p) { return *reinterpret_cast<const uint4*>(p); }
  static __device__ __forceinline__ void get(const type& v, float (&f)[8]) {
    const __bf16* h = reinterpret_cast<const __bf16*>(&v);
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] = float(h[e]);
  }
};
template <> struct G8<float> {
  using type = F8;
  static __device__ __forceinline__ type load(const float* p) {
    return F8{*reinterpret_cast<const float4*>(p), *reinterpret_cast<const float4*>(p + 4)};
  }
  static __device__ __forceinline__ void get(const type& v, float (&f)[8]) {
    f[0] = v.lo.x, f[1] = v.lo.y, f[2] = v.lo.z, f[3] = v.lo.w;
    f[4] = v.hi.x, f[5] = v.hi.y, f[6] = v.hi.z, f[7] = v.hi.w;
  }
};

template <typename TI, int NG>  // 1, 2, 4 or 8 n-groups (N / 8)
__global__ __launch_bounds__(256) void k_wgrad_c1(Args a, const TI* __restrict__ gout,
                                                  const TI* __restrict__ in, int64_t tiles_per_split,
                                                  float* __restrict__ part, float* __restrict__ bpart) {
  __shared__ float xs[C1_TR + C1_HALO];
  __shared__ float red[4][C1_NMAX * (C1_KMAX + 1)];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int grp = tid % NG, rl = tid / NG, nrl = 256 / NG;
  const int tps = (a.T + C1_TR - 1) / C1_TR;
  const int64_t ntiles = (a.rows / a.T) * tps;
  const int64_t tb = int64_t(blockIdx.x) * tiles_per_split;
  const int64_t te = tb + tiles_per_split < ntiles ? tb + tiles_per_split : ntiles;
  float acc[8][C1_KMAX], bsum[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    bsum[e] = 0.f;
#pragma unroll
    for (int k = 0; k < C1_KMAX; ++k) acc[e][k] = 0.f;
  }
  // the next tile's samples are fetched into registers while this tile is
  // reduced; this tile's gout rows are requested together before the FMAs
  const int span = C1_TR + (a.K - 1) * a.dil;
  float pre[2];
  auto fetch = [&](int64_t tile) {
    const int64_t b = tile / tps;
    const int t0 = int(tile % tps) * C1_TR;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int r = threadIdx.x + 256 * u;
      int ti = t0 - a.pad + r;
      const bool ok = r < span && ((ti >= 0 && ti < a.T) || a.pad_mode == SEL_PAD_REPLICATE);
      ti = ti < 0 ? 0 : (ti >= a.T ? a.T - 1 : ti);
      const float v = ok ? to_f(in[b * a.T + ti]) : 0.f;
      pre[u] = ok && a.in_elu ? c1_act<TI>(v) : v;
    }
  };
  constexpr int MAXR = C1_TR * NG / 256;  // rows per thread and tile
  // this tile's gout rows (next tile's: requested before this tile's FMAs)
  using GV = typename G8<TI>::type;
  GV gq[MAXR];
  auto fetch_g = [&](int64_t tile) {
    const int64_t b = tile / tps;
    const int t0 = int(tile % tps) * C1_TR;
    const int rows = a.T - t0 < C1_TR ? a.T - t0 : C1_TR;
#pragma unroll
    for (int j = 0; j < MAXR; ++j) {
      const int r = rl + j * nrl;
      if (j * nrl < C1_TR && r < rows)
        gq[j] = G8<TI>::load(gout + (b * a.T + t0 + r) * a.N + grp * 8);
    }
  };
  if (tb < te) {
    fetch(tb);
    fetch_g(tb);
  }
  for (int64_t tile = tb; tile < te; ++tile) {
    const int t0 = int(tile % tps) * C1_TR;
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 2; ++u)
      if (threadIdx.x + 256 * u < span) xs[threadIdx.x + 256 * u] = pre[u];
    __syncthreads();
    if (tile + 1 < te) fetch(tile + 1);
    const int rows = a.T - t0 < C1_TR ? a.T - t0 : C1_TR;
    GV gc[MAXR];
#pragma unroll
    for (int j = 0; j < MAXR; ++j) gc[j] = gq[j];
    if (tile + 1 < te) fetch_g(tile + 1);
#pragma unroll
    for (int j = 0; j < MAXR; ++j) {
      const int r = rl + j * nrl;
      if (j * nrl >= C1_TR || r >= rows) break;
      float gv[8];
      G8<TI>::get(gc[j], gv);
      float xv[C1_KMAX];
#pragma unroll
      for (int k = 0; k < C1_KMAX; ++k) xv[k] = k < a.K ? xs[r + k * a.dil] : 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float g = gv[e];
        bsum[e] += g;
#pragma unroll
        for (int k = 0; k < C1_KMAX; ++k) acc[e][k] = fmaf(g, xv[k], acc[e][k]);
      }
    }
  }
  // lanes of one wave with the same n group differ in the bits >= log2(NG)
#pragma unroll
  for (int e = 0; e < 8; ++e) {
#pragma unroll
    for (int k = 0; k <= C1_KMAX; ++k) {
      float v = k < C1_KMAX ? acc[e][k] : bsum[e];
      for (int o = 32; o >= NG; o >>= 1) v += __shfl_xor(v, o, 64);
      if (lane < NG) red[wave][(grp * 8 + e) * (C1_KMAX + 1) + k] = v;
    }
  }
  __syncthreads();
  for (int i = tid; i < a.N * (C1_KMAX + 1); i += 256) {
    const int n = i / (C1_KMAX + 1), k = i % (C1_KMAX + 1);
    const float v = red[0][i] + red[1][i] + red[2][i] + red[3][i];
    if (k < a.K) part[int64_t(blockIdx.x) * a.N * a.K + n * a.K + k] = v;
    else if (k == C1_KMAX && bpart) bpart[int64_t(blockIdx.x) * a.N + n] = v;
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

// fp32 weight gradient on sample-aligned 64-row tiles (the reference-precision
// path; the generic k_conv_wgrad above remains for other shapes).  One
// workgroup owns 64 output channels (16 per wave) x 32 input channels x all K
// taps and a contiguous range of 64-row tiles that never cross a sample, so
// the causal halo is zero- or replicate-filled while staging and the MFMA loop
// has no per-row address arithmetic or masks.  The next tile's g and x rows
// are fetched (16-B loads) into registers while the current tile's MFMAs run.
// MFMA v_mfma_f32_16x16x4_f32: A = g^T (lane: n = l & 15, row 4q + l >> 4),
// B = ELU(x) rows shifted by the tap (col c = l & 15); the 4 rows of one
// k-step are 80 / 48 floats apart in LDS (distinct 16-bank groups).
constexpr int WF_BM = 64, WF_XR = 128;
// NB output x CB input channels per workgroup: (64, 32), or (32, 64) / (32, 32)
// for the 32-wide layers (a 64-wide block would leave two of its waves on
// absent output channels); waves = (NB / 16) along n x the rest along c, each
// 16 n x CT 16-wide c tiles x all taps.  Row pitches NB + 16 / CB + 16 floats
// put the 4 rows of one k-step in distinct 16-bank groups.
template <int KM, int NB, int CB>
__global__ __launch_bounds__(256) void k_wgrad_f32(Args a, const float* __restrict__ gout,
                                                   const float* __restrict__ in, int tps, int64_t n_tiles,
                                                   int tiles_per_split, float* __restrict__ part,
                                                   float* __restrict__ bpart) {
  constexpr int GP = NB + 16, XP = CB + 16;
  constexpr int WN = NB / 16, WC = 4 / WN, CT = CB / (16 * WC);
  constexpr int G4 = NB / 4, GRP = 256 / G4, GI = WF_BM / GRP;   // gout float4 per row, rows per pass, passes
  constexpr int X4 = CB / 4, XRP = 256 / X4, XI = WF_XR / XRP;   // input float4 per row, rows per pass, passes
  static_assert(WN * WC == 4 && CT >= 1, "wave layout");
  __shared__ __align__(16) float gs[WF_BM * GP];
  __shared__ __align__(16) float xs[WF_XR * XP];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave % WN, wc = wave / WN;
  const int n0 = blockIdx.x * NB, c0 = blockIdx.y * CB;
  const int split = blockIdx.z;
  const int64_t tb = int64_t(split) * tiles_per_split;
  const int64_t te = tb + tiles_per_split < n_tiles ? tb + tiles_per_split : n_tiles;
  const int span = WF_BM + (a.K - 1) * a.dil;
  const bool want_bias = bpart != nullptr && c0 == 0;

  floatx4 acc[KM][CT];
#pragma unroll
  for (int k = 0; k < KM; ++k)
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) acc[k][ct] = floatx4{0.f, 0.f, 0.f, 0.f};
  float bsum = 0.f;

  // raw loads of clamped (valid) addresses and their predicates; the zero
  // select happens in put() (a load under a per-element condition is a branch
  // with a vmcnt(0) wait, and a select right behind a load waits for it)
  float4 gr[GI], xr[XI];
  bool gok[GI], xok[XI];
  auto fetch = [&](int64_t tile) {
    const int64_t b = tile / tps;
    const int t0 = int(tile - b * tps) * WF_BM;
#pragma unroll
    for (int i = 0; i < GI; ++i) {
      const int r = i * GRP + tid / G4, n = n0 + (tid % G4) * 4;
      const int t = t0 + r;
      const int tc = t < a.T ? t : a.T - 1, nc = n < a.N ? n : a.N - 4;
      gr[i] = *reinterpret_cast<const float4*>(gout + (b * a.T + tc) * a.N + nc);
      gok[i] = t < a.T && n < a.N;
    }
#pragma unroll
    for (int i = 0; i < XI; ++i) {
      const int r = i * XRP + tid / X4, c = c0 + (tid % X4) * 4;
      int ti = t0 - a.pad + r;
      bool ok = r < span && c < a.C;
      if (ti < 0 || ti >= a.T) {
        if (a.pad_mode == SEL_PAD_ZERO) ok = false;
        ti = ti < 0 ? 0 : a.T - 1;
      }
      xr[i] = *reinterpret_cast<const float4*>(in + (b * a.T + ti) * a.C + (c < a.C ? c : a.C - 4));
      xok[i] = ok;
    }
  };
  auto put = [&]() {
#pragma unroll
    for (int i = 0; i < GI; ++i)
      *reinterpret_cast<float4*>(gs + (i * GRP + tid / G4) * GP + (tid % G4) * 4) = keep4(gok[i], gr[i]);
#pragma unroll
    for (int i = 0; i < XI; ++i) {
      float4 v = keep4(xok[i], xr[i]);
      if (a.in_elu) v = make_float4(elu(v.x), elu(v.y), elu(v.z), elu(v.w));
      *reinterpret_cast<float4*>(xs + (i * XRP + tid / X4) * XP + (tid % X4) * 4) = v;
    }
  };

  if (tb < te) fetch(tb);
  const float* gcol = gs + wn * 16 + (lane & 15);
  const float* xcol = xs + wc * CT * 16 + (lane & 15);
  for (int64_t tile = tb; tile < te; ++tile) {
    __syncthreads();  // the previous tile's MFMAs are done with gs / xs
    put();
    __syncthreads();
    if (tile + 1 < te) fetch(tile + 1);
    if (want_bias && tid < NB)
      for (int r = 0; r < WF_BM; ++r) bsum += gs[r * GP + tid];
#pragma unroll 2
    for (int q = 0; q < WF_BM / 4; ++q) {
      const int r = 4 * q + (lane >> 4);
      const float av = gcol[r * GP];
#pragma unroll
      for (int k = 0; k < KM; ++k) {
        if (k >= a.K) break;
        const float* xrow = xcol + (r + k * a.dil) * XP;
#pragma unroll
        for (int ct = 0; ct < CT; ++ct)
          acc[k][ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, xrow[16 * ct], acc[k][ct], 0, 0, 0);
      }
    }
  }
  // partials: part[split][n][k][c] (C/D: col = c (lane & 15), row = n (4 (lane >> 4) + e))
  float* pdst = part + int64_t(split) * a.N * a.K * a.C;
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    if (k >= a.K) break;
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      const int c = c0 + (wc * CT + ct) * 16 + (lane & 15);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int n = n0 + wn * 16 + 4 * (lane >> 4) + e;
        if (n < a.N && c < a.C) pdst[(int64_t(n) * a.K + k) * a.C + c] = acc[k][ct][e];
      }
    }
  }
  if (want_bias && tid < NB && n0 + tid < a.N) bpart[int64_t(split) * a.N + n0 + tid] = bsum;
}

// bf16 weight gradient.  One workgroup owns (n-tile BN, c-tile 32, all K taps) and
// a contiguous range of 64-row m-tiles that never cross a sample boundary (so
// the causal halo can be zero/replicate-filled while staging and no per-element
// masks are needed).  Both MFMA operands reduce over m, i.e. over the ROW index
// of the row-major LDS tiles: they are read with ds_read_b64_tr_b16 (gfx950
// transposing LDS read, 4 rows x 16 columns per 16-lane group).  The MFMA k-index
// kk = 8g + e maps to tile row 4g + e (e < 4) / 16 + 4g + e - 4 (e >= 4) so that
// each 32-lane half reads 8 consecutive rows: with a row pitch of 8u dwords
// (u odd) those reads are bank-conflict free.
typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef short v8i16 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ v4i16 tr_read(const __bf16* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4i16*)(p));
}
__device__ __forceinline__ bf16x8 tr_frag(const __bf16* p, int pitch) {
  const v4i16 lo = tr_read(p);
  const v4i16 hi = tr_read(p + 16 * pitch);
  const v8i16 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, v);
}

// ---------------------------------------------------------------------------
// Residual unit at 32 channels: backward AND both weight gradients in one
// launch (the encoder's units, whose weights train; residual_unit.py:43-46,
// conv_layer.py:139-142).  k_ru32_bwd's two phases (gh, then gx), plus:
//  * ELU(bf16 h) of the tile rows -> LDS, from the h rows the gh phase already
//    holds for ELU'(h); ELU(x) of the tile + its causal halo -> LDS, staged with
//    g (the operands conv1 and the 1x1 consumed in the forward, same elu8);
//  * after gx, the 7 conv1 taps and the 1x1 as eight 32x32 MFMA accumulators,
//    two per wave (waves 0-2: taps 2w, 2w+1 sharing the gh operand; wave 3:
//    tap 6 and the 1x1), reduced over the tile rows with transposing LDS reads
//    (ds_read_b64_tr_b16: the k_wgrad3_bf16 operand scheme) and carried across
//    all of the block's tiles;
//  * one fp32 partial per block of each weight (+ the bias column sums of gh
//    and g, waves 0 and 3), in the packed [N][K][C] layout that
//    sel_wgrad_finish_many reduces in block order (deterministic).
// HBM per row: reads g, h, x and writes gx; the unfused path also wrote gh and
// re-read g, h, gh, x for the two weight-gradient launches (9 tensors).
// The gh and gx phases are k_ru32_bwd's arithmetic exactly (same bits).
// ---------------------------------------------------------------------------
template <int R>
struct Ru32W {
  static constexpr int P = F4_P;   // g / gh rows (80 B: conflict-free ds_read_b128 of the gx phase)
  static constexpr int PW = 32;    // ELU(x) / ELU(h) rows (64 B: conflict-free transposing reads)
  static constexpr int SPAN = R + F4_HALOMAX;
  static constexpr int NW1 = RU_C * RU_K * RU_C, NW2 = RU_C * RU_C;  // packed weight elements
  // g, gh and h planes (pitch P) + ELU(x) span and ELU(h) tile planes (pitch PW)
  static constexpr size_t LDS = size_t(3) * SPAN * P * 2 + size_t(SPAN + R) * PW * 2;
  static_assert(R % 128 == 0, "ru32 tile rows");
};

template <int R>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(SEL_W_RU32W))) void k_ru32_bwdw(Args a, const __bf16* __restrict__ g,
                                                   const __bf16* __restrict__ h, const __bf16* __restrict__ x,
                                                   const __bf16* __restrict__ wd1, const __bf16* __restrict__ wd2,
                                                   __bf16* __restrict__ gx, float* __restrict__ part1,
                                                   float* __restrict__ part2, int tiles_per_block) {
  using G = Ru32W<R>;
  constexpr int P = G::P, PW = G::PW;
  extern __shared__ __align__(16) unsigned char smem[];
  __bf16* const gs = reinterpret_cast<__bf16*>(smem);  // [SPAN][P]: g rows t0 ..
  __bf16* const ghs = gs + G::SPAN * P;                // [SPAN][P]: gh rows t0 ..
  __bf16* const xs = ghs + G::SPAN * P;                // [SPAN][PW]: ELU(x) rows t0 - halo ..
  __bf16* const es = xs + G::SPAN * PW;                // [R][PW]: ELU(h) rows t0 ..
  __bf16* const hs = es + R * PW;                      // [SPAN][P]: h rows t0 .. (the ELU'(h) factor)
  const int lane = threadIdx.x & 63, hl = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int halo = (RU_K - 1) * a.dil;
  const int span = R + halo;
  const int nsub = (span + 31) / 32;
  const int tps = (a.T + R - 1) / R;

  // weight-gradient jobs of this wave: job 0 = conv1 tap k0 (A = gh), job 1 =
  // conv1 tap k0 + 1 (waves 0-2, same A) or the 1x1 (wave 3: A = g, B = ELU(h))
  const int k0 = wave < 3 ? 2 * wave : 6;
  floatx16 wacc[2];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int e = 0; e < 16; ++e) wacc[j][e] = 0.f;
  float bsum = 0.f;  // wave 0: column sums of gh (conv1 bias), wave 3: of g (1x1 bias)
  // transposing-read lane geometry (k_wgrad3_bf16): rows 4 hl + q and 8 + 4 hl + q, 4 columns at col
  const int tq = (lane & 15) >> 2;
  const int tcol = ((lane >> 4) & 1) * 16 + 4 * (lane & 3);
  auto trfrag = [&](const __bf16* base, int pitch, int r0) {
    const v4i16 lo = tr_read(base + (r0 + 4 * hl + tq) * pitch + tcol);
    const v4i16 hi = tr_read(base + (r0 + 8 + 4 * hl + tq) * pitch + tcol);
    return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
  };

  int64_t tile0, tile_end;
  if (ru_tiles((a.rows / a.T) * tps, tiles_per_block, tile0, tile_end)) {
    bf16x8 wf[RU_K][2], w2f[1][2];
    ru_wfrags<RU_K>(wd1, wf);
    ru_wfrags<1>(wd2, w2f);
    ws_wait_vm<0>();  // weights landed: the tile loop's waits then count only its own loads

    // g, x and h rows staged one tile ahead (branch-free buffer loads): the gh
    // phase then reads h from LDS instead of waiting on a request made at the
    // top of the tile
    Ru32Stage<R> st, sx, sh;
    st.load(a, g, tile0 / tps, int(tile0 % tps) * R, 0, span);
    sx.load(a, x, tile0 / tps, int(tile0 % tps) * R, -halo, span);
    sh.load(a, h, tile0 / tps, int(tile0 % tps) * R, 0, span);
    ru_dummy_stores<2 * Ru32<R>::TM>(gx);  // the loop's gx stores after each prefetch
    for (int64_t tile = tile0; tile < tile_end; ++tile) {
      const int64_t b = tile / tps;
      const int t0 = int(tile % tps) * R;
      const int mrows = a.T - t0 < R ? a.T - t0 : R;
      __syncthreads();  // every wave is done with the previous tile's rows
      st.store(gs, span, false);
      sx.store(xs, span, true, nullptr, 0, PW);
      sh.store(hs, span, false);
      __syncthreads();
      constexpr int NSUB_W = (G::SPAN / 32 + 3) / 4;
      uint2 xpre[Ru32<R>::TM][4];
#pragma unroll
      for (int i = 0; i < Ru32<R>::TM; ++i) {
        const int lr = wave * (R / 4) + i * 32 + (lane & 31);
        const bool in = lr < mrows;
        const int64_t orow = (b * a.T + t0 + (in ? lr : 0)) * RU_C;
#pragma unroll
        for (int q = 0; q < 4; ++q)
          xpre[i][q] = in ? *reinterpret_cast<const uint2*>(x + orow + 8 * q + 4 * hl) : make_uint2(0, 0);
      }
      // gh for rows t0 .. t0 + span (k_ru32_bwd); ELU(h) of the tile rows -> es
#pragma unroll
      for (int j = 0; j < NSUB_W; ++j) {
        const int sb = wave + 4 * j;
        if (sb >= nsub) break;
        const int lr = sb * 32 + (lane & 31);
        floatx16 acc;
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[e] = 0.f;
        const __bf16* gw = gs + lr * P + 8 * hl;
#pragma unroll
        for (int c = 0; c < 2; ++c)
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w2f[0][c], *reinterpret_cast<const bf16x8*>(gw + 16 * c), acc, 0,
                                                        0, 0);
        uint2 hq[4];  // h rows (zero past T), as staged
#pragma unroll
        for (int q = 0; q < 4; ++q) hq[q] = *reinterpret_cast<const uint2*>(hs + lr * P + 8 * q + 4 * hl);
        float v[16];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const __bf16* hv = reinterpret_cast<const __bf16*>(&hq[q]);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[4 * q + e] = acc[4 * q + e] * elu_grad_fast(float(hv[e]));
        }
        bf16x8 ghf[2];
        ru_acc_to_frags(v, ghf);
        if (lr < span) {
          *reinterpret_cast<bf16x8*>(ghs + lr * P + 8 * hl) = ghf[0];
          *reinterpret_cast<bf16x8*>(ghs + lr * P + 16 + 8 * hl) = ghf[1];
        }
        if (sb < R / 32) {  // wave-uniform: a tile sub-tile (rows past T hold h = 0 -> ELU = 0)
#pragma unroll
          for (int qq = 0; qq < 2; ++qq) {
            const uint4 e8 = elu8(make_uint4(hq[2 * qq].x, hq[2 * qq].y, hq[2 * qq + 1].x, hq[2 * qq + 1].y));
            *reinterpret_cast<uint2*>(es + lr * PW + 16 * qq + 4 * hl) = make_uint2(e8.x, e8.y);
            *reinterpret_cast<uint2*>(es + lr * PW + 16 * qq + 8 + 4 * hl) = make_uint2(e8.z, e8.w);
          }
        }
      }
      __syncthreads();
      // the next tile's g and x rows, requested after the gh phase (k_ru64_bwd)
      {  // unconditional (a dead request loads nothing): exact counts
        const bool live = tile + 1 < tile_end;
        const int64_t nt = live ? tile + 1 : tile;
        st.load(a, g, nt / tps, int(nt % tps) * R, 0, span, live);
        sx.load(a, x, nt / tps, int(nt % tps) * R, -halo, span, live);
        sh.load(a, h, nt / tps, int(nt % tps) * R, 0, span, live);
      }
      // gx = conv1^T(gh) * ELU'(x) + g (k_ru32_bwd); every sub-tile stores
      // (rows past T to RU_OOB): a fixed count of stores per tile keeps the
      // next tile's staging waits exact (ru_bstore)
      const __amdgpu_buffer_rsrc_t rgx = ru_rsrc(gx + b * a.T * RU_C, int64_t(a.T) * RU_C);
#pragma unroll
      for (int i = 0; i < Ru32<R>::TM; ++i) {
        const int lr = wave * (R / 4) + i * 32 + (lane & 31);
        floatx16 acc;
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[e] = 0.f;
        const __bf16* hw = ghs + lr * P + 8 * hl;
#pragma unroll
        for (int k = 0; k < RU_K; ++k)
#pragma unroll
          for (int c = 0; c < 2; ++c)
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[k][c],
                                                          *reinterpret_cast<const bf16x8*>(hw + k * a.dil * P + 16 * c),
                                                          acc, 0, 0, 0);
        const bool valid = lr < mrows;
        float v[16];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint2 graw = *reinterpret_cast<const uint2*>(gs + lr * P + 8 * q + 4 * hl);
          const __bf16* xv = reinterpret_cast<const __bf16*>(&xpre[i][q]);
          const __bf16* gv = reinterpret_cast<const __bf16*>(&graw);
#pragma unroll
          for (int e = 0; e < 4; ++e)
            v[4 * q + e] = __fadd_rn(__fmul_rn(acc[4 * q + e], elu_grad_fast(float(xv[e]))), float(gv[e]));
        }
        bf16x8 of[2];
        ru_acc_to_frags(v, of);
        const int off = ((t0 + lr) * RU_C + 8 * hl) * 2;
        ru_bstore(rgx, valid ? off : RU_OOB, of[0]);
        ru_bstore(rgx, valid ? off + 32 : RU_OOB, of[1]);
      }
      // weight gradients over the tile rows (rows past T: g = 0 -> gh = 0)
      const __bf16* b0p = xs + k0 * a.dil * PW;
      const __bf16* b1p = wave < 3 ? b0p + a.dil * PW : es;
#pragma unroll
      for (int kh = 0; kh < R / 16; ++kh) {
        const bf16x8 A0 = trfrag(ghs, P, kh * 16);
        const bf16x8 B0 = trfrag(b0p, PW, kh * 16);
        const bf16x8 B1 = trfrag(b1p, PW, kh * 16);
        wacc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A0, B0, wacc[0], 0, 0, 0);
        if (wave < 3) {
          wacc[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A0, B1, wacc[1], 0, 0, 0);
          if (wave == 0) {
#pragma unroll
            for (int e = 0; e < 8; ++e) bsum += float(A0[e]);
          }
        } else {
          const bf16x8 A1 = trfrag(gs, P, kh * 16);
          wacc[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A1, B1, wacc[1], 0, 0, 0);
#pragma unroll
          for (int e = 0; e < 8; ++e) bsum += float(A1[e]);
        }
      }
    }
  }
  // this block's partials (zeros from a block without tiles): accumulator
  // element r of lane l -> n = (r & 3) + 8 (r >> 2) + 4 hl, c = l & 31
  const int nb = gridDim.x;
  float* const p1 = part1 + int64_t(blockIdx.x) * G::NW1;
  float* const p2 = part2 + int64_t(blockIdx.x) * G::NW2;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int n = (r & 3) + 8 * (r >> 2) + 4 * hl, c = lane & 31;
    p1[(n * RU_K + k0) * RU_C + c] = wacc[0][r];
    if (wave < 3) p1[(n * RU_K + k0 + 1) * RU_C + c] = wacc[1][r];
    else p2[n * RU_C + c] = wacc[1][r];
  }
  bsum += __shfl_xor(bsum, 32, 64);
  if (wave == 0 && lane < 32) part1[int64_t(nb) * G::NW1 + int64_t(blockIdx.x) * RU_C + lane] = bsum;
  if (wave == 3 && lane < 32) part2[int64_t(nb) * G::NW2 + int64_t(blockIdx.x) * RU_C + lane] = bsum;
}

// ---------------------------------------------------------------------------
// Residual unit at 64 channels: backward AND both weight gradients in one
// launch (round 4; the encoder's units, residual_unit.py:43-46 and the wgrad of
// conv_layer.py:139-142).  The weight-gradient accumulators (28 conv1 tiles +
// 4 1x1 tiles of 32x32 fp32 = 128 registers per lane over four waves) do not
// fit beside k_ru64_bwd's register-resident k7 adjoint (112 VGPRs), so the
// workgroup has eight waves in two roles that share every LDS plane:
//  * all eight stage the next tile's g, h and x span rows (registers, one
//    tile ahead, branch-free buffer loads) and compute gh = (W2^T g) * ELU'(h)
//    over the tile + its anti-causal halo (k_ru64_bwd's gh units) into LDS,
//    plus ELU(bf16 h) of the tile rows;
//  * waves 0-3 compute gx = conv1^T(gh) * ELU'(x) + g exactly as k_ru64_bwd
//    (same MFMA order, rounding points and epilogue: same bits);
//  * waves 4-7 accumulate the weight gradients over the tile rows with
//    transposing LDS reads (the k_ru32_bwdw / k_wgrad3_bf16 operand scheme):
//    wave 4 + v owns h-channel slice v & 1 and, for v < 2, conv1 taps 0-3, for
//    v >= 2 taps 4-6 and the 1x1 (A = g, B = ELU(h)), both input-channel
//    slices, plus the bias column sums of gh (v < 2) or g (v >= 2).
// A workgroup's waves are dealt to the SIMDs cyclically, so each SIMD runs one
// gx wave beside one weight-gradient wave.  The roles' tile loops are separate
// code (so neither role's registers are live in the other) with the same
// barrier sequence.  One workgroup per CU (the planes take 159 KB of LDS);
// one fp32 partial per workgroup of every weight, in the packed layouts that
// sel_wgrad_finish_many reduces in block order (deterministic).
// HBM per row: reads g, h, x and writes gx; k_ru64_bwd with gh plus the two
// k_wgrad3 launches moved 9 tensors.
// ---------------------------------------------------------------------------
template <int R>
struct Ru64W {
  static constexpr int C = 64, K = 7, P = F4_P, PW = 32;
  static constexpr int SPAN = R + F4_HALOMAX;
  static constexpr int CV = C / 8;
  static constexpr int XV = (SPAN * CV + 511) / 512;  // staged 16-B pieces per thread and tensor
  static constexpr int UPW = (2 * (SPAN / 32) + 7) / 8;  // gh (sub-tile, slice) units per wave
  static constexpr int NW1 = C * K * C, NW2 = C * C;
  static constexpr int W2P = C + 8;
  // planes (bf16 elements): g, gh, h [2][SPAN][P]; ELU(x) span [2][SPAN][PW];
  // raw x tile [2][R][P] (ELU'(x)); ELU(h) tile [2][R][PW]; the 1x1 adjoint [C][W2P]
  static constexpr size_t OFF_GH = size_t(2) * SPAN * P;
  static constexpr size_t OFF_H = 2 * OFF_GH;
  static constexpr size_t OFF_XS = 3 * OFF_GH;
  static constexpr size_t OFF_XR = OFF_XS + size_t(2) * SPAN * PW;
  static constexpr size_t OFF_ES = OFF_XR + size_t(2) * R * P;
  static constexpr size_t OFF_W2 = OFF_ES + size_t(2) * R * PW;
  static constexpr size_t LDS = (OFF_W2 + size_t(C) * W2P) * 2;
  static_assert(R % 64 == 0 && LDS <= 160 * 1024, "ru64w tile rows / LDS");
  static_assert(SPAN * CV % 512 == 0, "ru64w staging pieces");
};

template <int R>
struct Ru64WStage {
  uint4 g[Ru64W<R>::XV], h[Ru64W<R>::XV], x[Ru64W<R>::XV];
};

// one tile's g, h (rows t0 .. t0 + span) and x (rows t0 - halo .. t0 + R) into
// registers: branch-free buffer loads (rows outside [0, T), past the span or of
// a dead request read nothing and return zeros; Ru32Stage::load)
template <int R>
__device__ __forceinline__ void ru64w_load(Ru64WStage<R>& st, const Args& a, const __bf16* __restrict__ g,
                                           const __bf16* __restrict__ h, const __bf16* __restrict__ x, int64_t tile,
                                           int tps, int halo, bool live) {
  using G = Ru64W<R>;
  const int64_t b = tile / tps;
  const int t0 = int(tile % tps) * R;
  const int64_t base = b * a.T * G::C;
  const __amdgpu_buffer_rsrc_t rg = ru_rsrc(g + base, int64_t(a.T) * G::C);
  const __amdgpu_buffer_rsrc_t rh = ru_rsrc(h + base, int64_t(a.T) * G::C);
  const __amdgpu_buffer_rsrc_t rx = ru_rsrc(x + base, int64_t(a.T) * G::C);
  const int span = R + halo;
#pragma unroll
  for (int u = 0; u < G::XV; ++u) {
    const int v = threadIdx.x + u * 512;
    const int r = v / G::CV, c = (v % G::CV) * 8;
    const int tg = t0 + r, tx = t0 - halo + r;
    const bool gok = live && r < span && tg < a.T;
    const bool xok = live && r < span && tx >= 0 && tx < a.T;
    // program order pinned (sched_barrier): the loads leave in the same order
    // from the prologue and from the tile loop, so the waits of the staging
    // store count them exactly on both paths into it
    st.g[u] = ru_bload(rg, gok ? (tg * G::C + c) * 2 : RU_OOB);
    __builtin_amdgcn_sched_barrier(0);
    st.h[u] = ru_bload(rh, gok ? (tg * G::C + c) * 2 : RU_OOB);
    __builtin_amdgcn_sched_barrier(0);
    st.x[u] = ru_bload(rx, xok ? (tx * G::C + c) * 2 : RU_OOB);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// the staged tile -> LDS planes (out-of-range rows were loaded as zeros)
template <int R>
__device__ __forceinline__ void ru64w_store(const Ru64WStage<R>& st, __bf16* smem_bf, int span, int halo) {
  using G = Ru64W<R>;
  constexpr int P = G::P, PW = G::PW, SPAN = G::SPAN;
  __bf16* const gs = smem_bf;
  __bf16* const hs = smem_bf + G::OFF_H;
  __bf16* const xs = smem_bf + G::OFF_XS;
  __bf16* const xr = smem_bf + G::OFF_XR;
#pragma unroll
  for (int u = 0; u < G::XV; ++u) {
    const int v = threadIdx.x + u * 512;
    const int r = v / G::CV, c = (v % G::CV) * 8;
    if (r >= span) continue;
    const int pl = c >> 5, cc = c & 31;
    *reinterpret_cast<uint4*>(gs + (pl * SPAN + r) * P + cc) = st.g[u];
    *reinterpret_cast<uint4*>(hs + (pl * SPAN + r) * P + cc) = st.h[u];
    *reinterpret_cast<uint4*>(xs + (pl * SPAN + r) * PW + cc) = elu8(st.x[u]);
    if (r >= halo && r < halo + R) *reinterpret_cast<uint4*>(xr + (pl * R + r - halo) * P + cc) = st.x[u];
  }
}

// gh = (W2^T g) * ELU'(h) over rows t0 .. t0 + span (k_ru64_bwd's units, round
// robin over the eight waves) -> ghs; ELU(bf16 h) of the tile rows -> es
template <int R>
__device__ __forceinline__ void ru64w_gh(__bf16* smem_bf, int wave, int lane, int nsub, int span) {
  using G = Ru64W<R>;
  constexpr int P = G::P, PW = G::PW, SPAN = G::SPAN, C = G::C;
  const __bf16* const gs = smem_bf;
  __bf16* const ghs = smem_bf + G::OFF_GH;
  const __bf16* const hs = smem_bf + G::OFF_H;
  __bf16* const es = smem_bf + G::OFF_ES;
  const __bf16* const w2s = smem_bf + G::OFF_W2;
  const int hl = lane >> 5;
#pragma unroll
  for (int uu = 0; uu < G::UPW; ++uu) {
    const int unit = wave + 8 * uu;
    if (unit >= 2 * nsub) break;  // wave-uniform
    const int sb = unit >> 1, sl = unit & 1;
    const int lr = sb * 32 + (lane & 31);
    bf16x8 w2q[C / 16];
    {
      const __bf16* wr2 = w2s + (sl * 32 + (lane & 31)) * G::W2P + 8 * hl;
#pragma unroll
      for (int q = 0; q < C / 16; ++q) w2q[q] = *reinterpret_cast<const bf16x8*>(wr2 + 16 * q);
    }
    floatx16 acc;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = 0.f;
    const __bf16* gw = gs + lr * P + 8 * hl;
#pragma unroll
    for (int q = 0; q < C / 16; ++q)
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w2q[q], *reinterpret_cast<const bf16x8*>(gw + (q >> 1) * SPAN * P + 16 * (q & 1)),
                                                    acc, 0, 0, 0);
    uint2 hq[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) hq[q] = *reinterpret_cast<const uint2*>(hs + (sl * SPAN + lr) * P + 8 * q + 4 * hl);
    float v[16];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const __bf16* hv = reinterpret_cast<const __bf16*>(&hq[q]);
#pragma unroll
      for (int e = 0; e < 4; ++e) v[4 * q + e] = __fmul_rn(acc[4 * q + e], elu_grad_fast(float(hv[e])));
    }
    bf16x8 ghf[2];
    ru_acc_to_frags(v, ghf);
    if (lr < span) {
      *reinterpret_cast<bf16x8*>(ghs + (sl * SPAN + lr) * P + 8 * hl) = ghf[0];
      *reinterpret_cast<bf16x8*>(ghs + (sl * SPAN + lr) * P + 16 + 8 * hl) = ghf[1];
    }
    if (sb < R / 32) {  // wave-uniform: a tile sub-tile (rows past T hold h = 0 -> ELU = 0)
#pragma unroll
      for (int qq = 0; qq < 2; ++qq) {
        const uint4 e8 = elu8(make_uint4(hq[2 * qq].x, hq[2 * qq].y, hq[2 * qq + 1].x, hq[2 * qq + 1].y));
        *reinterpret_cast<uint2*>(es + (sl * R + lr) * PW + 16 * qq + 4 * hl) = make_uint2(e8.x, e8.y);
        *reinterpret_cast<uint2*>(es + (sl * R + lr) * PW + 16 * qq + 8 + 4 * hl) = make_uint2(e8.z, e8.w);
      }
    }
  }
}

// WG = false: the same kernel without the weight-gradient role (the decoder's
// units, whose weights are frozen): all eight waves compute gx, one 32-row
// sub-tile and 32-channel slice each (part1 / part2 unused).
template <int R, bool WG = true>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2))) void k_ru64_bwdw(
    Args a, const __bf16* __restrict__ g, const __bf16* __restrict__ h, const __bf16* __restrict__ x,
    const __bf16* __restrict__ wd1, const __bf16* __restrict__ wd2, __bf16* __restrict__ gx,
    float* __restrict__ part1, float* __restrict__ part2, int tiles_per_block) {
  using G = Ru64W<R>;
  constexpr int P = G::P, PW = G::PW, C = G::C, K = G::K, SPAN = G::SPAN;
  extern __shared__ __align__(16) unsigned char smem[];
  __bf16* const sb = reinterpret_cast<__bf16*>(smem);
  const __bf16* const gs = sb;
  const __bf16* const ghs = sb + G::OFF_GH;
  const __bf16* const xs = sb + G::OFF_XS;
  const __bf16* const xr = sb + G::OFF_XR;
  const __bf16* const es = sb + G::OFF_ES;
  const int tid = threadIdx.x, lane = tid & 63, hl = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int halo = (K - 1) * a.dil;
  const int span = R + halo;
  const int nsub = (span + 31) / 32;
  const int tps = (a.T + R - 1) / R;
  int64_t tile0 = 0, tile_end = 0;
  const bool any = ru_tiles((a.rows / a.T) * tps, tiles_per_block, tile0, tile_end);

  // the 1x1 adjoint's weights [C][C] -> LDS (rows padded to W2P; k_ru64_bwd)
  if (any) {
    __bf16* const w2s = sb + G::OFF_W2;
    for (int i = tid; i < C * C / 8; i += 512) {
      const int n = i / (C / 8), c8 = (i % (C / 8)) * 8;
      *reinterpret_cast<bf16x8*>(w2s + n * G::W2P + c8) = *reinterpret_cast<const bf16x8*>(wd2 + int64_t(n) * C + c8);
    }
  }

  if (!WG || wave < 4) {
    // ---- gx role: k_ru64_bwd's gx phase (row group rg, output slice ns) ----
    if (!any) return;  // workgroup-uniform: a block without tiles has no barriers
    const int ns = wave & 1, rg = wave >> 1;
    constexpr int WR = WG ? R / 2 : R / 4, TM = WR / 32;
    bf16x8 wf[K][C / 16];
    {
      const __bf16* wrow = wd1 + int64_t(ns * 32 + (lane & 31)) * K * C + 8 * hl;
#pragma unroll
      for (int k = 0; k < K; ++k)
#pragma unroll
        for (int q = 0; q < C / 16; ++q) wf[k][q] = *reinterpret_cast<const bf16x8*>(wrow + k * C + 16 * q);
    }
    ws_wait_vm<0>();  // weights landed: the tile loop's waits then count only its own loads
    Ru64WStage<R> st;
    ru64w_load<R>(st, a, g, h, x, tile0, tps, halo, true);
    ru_dummy_stores<2 * TM>(gx);  // the loop's gx stores after each prefetch
    for (int64_t tile = tile0; tile < tile_end; ++tile) {
      const int64_t b = tile / tps;
      const int t0 = int(tile % tps) * R;
      const int mrows = a.T - t0 < R ? a.T - t0 : R;
      __syncthreads();  // B1: every wave is done with the previous tile's planes
      ru64w_store<R>(st, sb, span, halo);
      __syncthreads();  // B2
      ru64w_load<R>(st, a, g, h, x, tile + 1 < tile_end ? tile + 1 : tile, tps, halo, tile + 1 < tile_end);
      ru64w_gh<R>(sb, wave, lane, nsub, span);
      __syncthreads();  // B3: gh planes complete
      floatx16 acc[TM];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][e] = 0.f;
      const __bf16* hw = ghs + (rg * WR + (lane & 31)) * P + 8 * hl;
#pragma unroll
      for (int k = 0; k < K; ++k)
#pragma unroll
        for (int q = 0; q < C / 16; ++q) {
          const __bf16* hb = hw + ((q >> 1) * SPAN + k * a.dil) * P + 16 * (q & 1);
#pragma unroll
          for (int i = 0; i < TM; ++i)
            acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[k][q], *reinterpret_cast<const bf16x8*>(hb + i * 32 * P),
                                                             acc[i], 0, 0, 0);
        }
      // every sub-tile is stored (rows past T to RU_OOB): a fixed count of
      // stores per tile keeps the next tile's staging wait exact (ru_bstore)
      const __amdgpu_buffer_rsrc_t rgx = ru_rsrc(gx + b * a.T * C, int64_t(a.T) * C);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int lr = rg * WR + i * 32 + (lane & 31);
        const bool valid = lr < mrows;
        float v[16];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint2 graw = *reinterpret_cast<const uint2*>(gs + (ns * SPAN + lr) * P + 8 * q + 4 * hl);
          const uint2 xraw = *reinterpret_cast<const uint2*>(xr + (ns * R + lr) * P + 8 * q + 4 * hl);
          const __bf16* xv = reinterpret_cast<const __bf16*>(&xraw);
          const __bf16* gv = reinterpret_cast<const __bf16*>(&graw);
#pragma unroll
          for (int e = 0; e < 4; ++e)
            v[4 * q + e] = __fadd_rn(__fmul_rn(acc[i][4 * q + e], elu_grad_fast(float(xv[e]))), float(gv[e]));
        }
        bf16x8 of[2];
        ru_acc_to_frags(v, of);
        const int off = ((t0 + lr) * C + ns * 32 + 8 * hl) * 2;
        ru_bstore(rgx, valid ? off : RU_OOB, of[0]);
        ru_bstore(rgx, valid ? off + 32 : RU_OOB, of[1]);
      }
    }
    return;
  }
  if constexpr (WG) {
  // ---- weight-gradient role ----
  const int v = wave - 4;
  const int wn = v & 1;     // h-channel (output) slice of the weight gradients
  const int upper = v >> 1;  // 0: conv1 taps 0-3; 1: taps 4-6 + the 1x1
  floatx16 wacc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int e = 0; e < 16; ++e) wacc[j][e] = 0.f;
  float bsum = 0.f;  // column sums of gh (upper = 0: conv1 bias) or g (upper = 1: the 1x1's)
  if (any) {
    const int tq = (lane & 15) >> 2;
    const int tcol = ((lane >> 4) & 1) * 16 + 4 * (lane & 3);
    auto trfrag = [&](const __bf16* base, int pitch, int r0) {
      const v4i16 lo = tr_read(base + (r0 + 4 * hl + tq) * pitch + tcol);
      const v4i16 hi = tr_read(base + (r0 + 8 + 4 * hl + tq) * pitch + tcol);
      return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
    };
    // wave-uniform operand bases: A0 = gh slice wn; jobs 0-5 = taps kb + j/2 over
    // ELU(x) input slice j & 1; jobs 6-7: A1 (gh again / g) against tap 3 of
    // ELU(x) (upper = 0) or ELU(h) (upper = 1), input slice j & 1
    const int kb = upper ? 4 : 0;
    const __bf16* const a0p = ghs + wn * SPAN * P;
    const __bf16* const a1p = upper ? gs + wn * SPAN * P : a0p;
    const __bf16* const b67 = upper ? es : xs + 3 * a.dil * PW;
    const int b67s = upper ? R * PW : SPAN * PW;
    Ru64WStage<R> st;
    ru64w_load<R>(st, a, g, h, x, tile0, tps, halo, true);
    for (int64_t tile = tile0; tile < tile_end; ++tile) {
      __syncthreads();  // B1
      ru64w_store<R>(st, sb, span, halo);
      __syncthreads();  // B2
      ru64w_load<R>(st, a, g, h, x, tile + 1 < tile_end ? tile + 1 : tile, tps, halo, tile + 1 < tile_end);
      ru64w_gh<R>(sb, wave, lane, nsub, span);
      __syncthreads();  // B3
      // rows past T hold g = 0 -> gh = 0: no masks
#pragma unroll 1
      for (int kh = 0; kh < R / 16; ++kh) {
        const bf16x8 A0 = trfrag(a0p, P, kh * 16);
        const bf16x8 A1 = trfrag(a1p, P, kh * 16);
#pragma unroll
        for (int j = 0; j < 6; ++j) {
          const bf16x8 B = trfrag(xs + ((j & 1) * SPAN + (kb + (j >> 1)) * a.dil) * PW, PW, kh * 16);
          wacc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A0, B, wacc[j], 0, 0, 0);
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const bf16x8 B = trfrag(b67 + j * b67s, PW, kh * 16);
          wacc[6 + j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A1, B, wacc[6 + j], 0, 0, 0);
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) bsum += float(A1[e]);
      }
    }
  }
  // this block's partials (zeros from a block without tiles): accumulator
  // element r of lane l -> n = wn*32 + (r & 3) + 8 (r >> 2) + 4 hl, c = slice*32 + (l & 31)
  const int nb = gridDim.x;
  float* const p1 = part1 + int64_t(blockIdx.x) * G::NW1;
  float* const p2 = part2 + int64_t(blockIdx.x) * G::NW2;
  const int kb = upper ? 4 : 0;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int n = wn * 32 + (r & 3) + 8 * (r >> 2) + 4 * hl, c = lane & 31;
#pragma unroll
    for (int j = 0; j < 6; ++j) p1[(n * K + kb + (j >> 1)) * C + (j & 1) * 32 + c] = wacc[j][r];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if (upper) p2[n * C + j * 32 + c] = wacc[6 + j][r];
      else p1[(n * K + 3) * C + j * 32 + c] = wacc[6 + j][r];
    }
  }
  bsum += __shfl_xor(bsum, 32, 64);
  if (lane < 32) {
    if (upper) part2[int64_t(nb) * G::NW2 + int64_t(blockIdx.x) * C + wn * 32 + lane] = bsum;
    else part1[int64_t(nb) * G::NW1 + int64_t(blockIdx.x) * C + wn * 32 + lane] = bsum;
  }
  }  // WG
}

constexpr int WB_BM = 64;
constexpr int WB_BC = 32;
constexpr int WB_MAXJ = 16;

template <int BN>
__global__ __launch_bounds__(256) void k_wgrad_bf16(Args a, const __bf16* __restrict__ gout,
                                                    const __bf16* __restrict__ in, int tiles_per_sample,
                                                    int64_t n_tiles, int tiles_per_split,
                                                    float* __restrict__ part, float* __restrict__ bpart) {
  constexpr int NT = BN / 16;
  constexpr int WPN = 4 / NT;        // waves sharing one n-subtile
  constexpr int PG = BN + 16;        // elements; (PG/2) dwords = 8 x odd
  constexpr int PX = WB_BC + 16;     // 48 elements = 24 dwords
  extern __shared__ __align__(16) unsigned char smem[];
  __bf16* gs = reinterpret_cast<__bf16*>(smem);
  __bf16* xs = gs + WB_BM * PG;
  const int halo = (a.K - 1) * a.dil;
  const int span = WB_BM + halo;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nt = wave % NT, wsub = wave / NT;
  const int n0 = blockIdx.x * BN, c0 = blockIdx.y * WB_BC;
  const int64_t tb = int64_t(blockIdx.z) * tiles_per_split;
  const int64_t te = tb + tiles_per_split < n_tiles ? tb + tiles_per_split : n_tiles;
  const int npairs = a.K * (WB_BC / 16);
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const bool vecG = (a.N % 8) == 0, vecX = (a.C % 8) == 0;

  floatx4 acc[WB_MAXJ];
#pragma unroll
  for (int j = 0; j < WB_MAXJ; ++j) acc[j] = floatx4{0.f, 0.f, 0.f, 0.f};
  float bsum = 0.f;

  for (int64_t tile = tb; tile < te; ++tile) {
    const int64_t b = tile / tiles_per_sample;
    const int t0 = int(tile % tiles_per_sample) * WB_BM;
    const int64_t rb = b * a.T;
    __syncthreads();
    for (int idx = tid; idx < WB_BM * (BN / 8); idx += 256) {
      const int r = idx / (BN / 8), v = (idx % (BN / 8)) * 8;
      const int t = t0 + r, n = n0 + v;
      __bf16 vals[8];
      if (t < a.T && vecG && n + 8 <= a.N) {
        *reinterpret_cast<uint4*>(vals) = *reinterpret_cast<const uint4*>(gout + (rb + t) * a.N + n);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e)
          vals[e] = (t < a.T && n + e < a.N) ? gout[(rb + t) * a.N + n + e] : __bf16(0.f);
      }
      *reinterpret_cast<uint4*>(gs + r * PG + v) = *reinterpret_cast<uint4*>(vals);
    }
    for (int idx = tid; idx < span * (WB_BC / 8); idx += 256) {
      const int r = idx / (WB_BC / 8), v = (idx % (WB_BC / 8)) * 8;
      int ti = t0 - a.pad + r;
      const int c = c0 + v;
      bool ok = ti >= 0 && ti < a.T;
      if (!ok && a.pad_mode == SEL_PAD_REPLICATE) {
        ti = ti < 0 ? 0 : a.T - 1;
        ok = true;
      }
      __bf16 vals[8];
      if (ok && vecX && c + 8 <= a.C) {
        *reinterpret_cast<uint4*>(vals) = *reinterpret_cast<const uint4*>(in + (rb + ti) * a.C + c);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) vals[e] = (ok && c + e < a.C) ? in[(rb + ti) * a.C + c + e] : __bf16(0.f);
      }
      if (a.in_elu) {
#pragma unroll
        for (int e = 0; e < 8; ++e) vals[e] = __bf16(elu_fast(float(vals[e])));
      }
      *reinterpret_cast<uint4*>(xs + r * PX + v) = *reinterpret_cast<uint4*>(vals);
    }
    __syncthreads();
    if (bpart && c0 == 0 && tid < BN) {
      for (int r = 0; r < WB_BM; ++r) bsum += float(gs[r * PG + tid]);
    }
#pragma unroll
    for (int grp = 0; grp < WB_BM / 32; ++grp) {
      const bf16x8 A = tr_frag(gs + (grp * 32 + 4 * g + q) * PG + nt * 16 + 4 * p, PG);
#pragma unroll
      for (int j = 0; j < WB_MAXJ; ++j) {
        const int pr = wsub + WPN * j;
        if (pr >= npairs) break;
        const int k = pr >> 1, ct = pr & 1;
        const bf16x8 Bf = tr_frag(xs + (grp * 32 + 4 * g + q + k * a.dil) * PX + ct * 16 + 4 * p, PX);
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A, Bf, acc[j], 0, 0, 0);
      }
    }
  }
  float* pdst = part + int64_t(blockIdx.z) * a.N * a.K * a.C;
#pragma unroll
  for (int j = 0; j < WB_MAXJ; ++j) {
    const int pr = wsub + WPN * j;
    if (pr >= npairs) break;
    const int k = pr >> 1, ct = pr & 1;
    const int c = c0 + ct * 16 + (lane & 15);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int n = n0 + nt * 16 + 4 * (lane >> 4) + e;
      if (n < a.N && c < a.C) pdst[(int64_t(n) * a.K + k) * a.C + c] = acc[j][e];
    }
  }
  if (bpart && c0 == 0 && tid < BN && n0 + tid < a.N) bpart[int64_t(blockIdx.z) * a.N + n0 + tid] = bsum;
}

// bf16 weight gradient, fast path (C % 32 == 0, N % 32 == 0, halo <= 64, K <= 8):
// block = (32 output channels n, 32 input channels c, m-split).  m-tiles are 128
// rows of one sample; each of the 4 waves owns 32 rows of the tile and
// accumulates ALL K taps as 32x32 tiles (v_mfma_f32_32x32x16_bf16), reading
// both operands with ds_read_b64_tr_b16 from 64-B LDS rows (rows 4h..4h+3 per
// 32-lane half: conflict free).  The next tile's rows are prefetched into
// registers during the MFMAs (branch-free clamped loads); the 4 waves' partial
// tiles are summed through LDS once per split.
constexpr int W2_BM = 128;
constexpr int W2_HALO = 64;

template <int TW>  // waves split taps into TW groups and rows into 4/TW groups
__global__ __launch_bounds__(256) void k_wgrad2_bf16(Args a, const __bf16* __restrict__ gout,
                                                     const __bf16* __restrict__ in, int tiles_per_sample,
                                                     int64_t n_tiles, int tiles_per_split,
                                                     float* __restrict__ part, float* __restrict__ bpart) {
  constexpr int GV = W2_BM * 32 / 8 / 256;                  // 2
  constexpr int XV = ((W2_BM + W2_HALO) * 4 + 255) / 256;   // 3
  constexpr int GS = W2_BM * 32, XS = (W2_BM + W2_HALO) * 32;  // elements per buffer
  constexpr int RG = 4 / TW;                                // row groups
  constexpr int RROWS = W2_BM / RG;                         // rows per wave per tile
  constexpr int KPW = TW == 1 ? 1 : 2;                      // taps per wave: K=1 | K<=4 (TW=2) | K<=8 (TW=4)
  extern __shared__ __align__(16) unsigned char smem[];
  __bf16* const base = reinterpret_cast<__bf16*>(smem);  // [buf]{G[128][32], X[192][32]}

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tg = wave % TW, rg = wave / TW;
  const int n0 = blockIdx.x * 32, c0 = blockIdx.y * 32;
  const int64_t tb = int64_t(blockIdx.z) * tiles_per_split;
  const int64_t te = tb + tiles_per_split < n_tiles ? tb + tiles_per_split : n_tiles;
  const int halo = (a.K - 1) * a.dil;
  const int span = W2_BM + halo;

  uint4 gr[GV], xr[XV];
  auto load = [&](int64_t tile) {
    const int64_t b = tile / tiles_per_sample;
    const int t0 = int(tile % tiles_per_sample) * W2_BM;
    const int64_t rb = b * a.T;
#pragma unroll
    for (int u = 0; u < GV; ++u) {
      const int v = tid + u * 256;
      const int t = t0 + (v >> 2);
      const bool ok = t < a.T;
      uint4 val = *reinterpret_cast<const uint4*>(gout + (rb + (ok ? t : 0)) * a.N + n0 + (v & 3) * 8);
      if (!ok) val = make_uint4(0, 0, 0, 0);
      gr[u] = val;
    }
#pragma unroll
    for (int u = 0; u < XV; ++u) {
      if (u * 64 >= span) {  // block-uniform: no halo rows to fetch (K = 1 / short halo)
        xr[u] = make_uint4(0, 0, 0, 0);
        continue;
      }
      const int v = tid + u * 256;
      const int r = v >> 2;
      int ti = t0 - a.pad + r;
      const bool inside = ti >= 0 && ti < a.T;
      const bool ok = r < span && (inside || a.pad_mode == SEL_PAD_REPLICATE);
      ti = ti < 0 ? 0 : (ti >= a.T ? a.T - 1 : ti);
      uint4 val = *reinterpret_cast<const uint4*>(in + (rb + ti) * a.C + c0 + (v & 3) * 8);
      if (!ok) val = make_uint4(0, 0, 0, 0);
      xr[u] = val;
    }
  };
  auto store = [&](int buf) {
    __bf16* g = base + buf * (GS + XS);
    __bf16* x = g + GS;
#pragma unroll
    for (int u = 0; u < GV; ++u) {
      const int v = tid + u * 256;
      *reinterpret_cast<uint4*>(g + (v >> 2) * 32 + (v & 3) * 8) = gr[u];
    }
#pragma unroll
    for (int u = 0; u < XV; ++u) {
      const int v = tid + u * 256;
      if ((v >> 2) >= W2_BM + W2_HALO) continue;
      uint4 val = xr[u];
      if (a.in_elu) {
        val = elu8(val);
      }
      *reinterpret_cast<uint4*>(x + (v >> 2) * 32 + (v & 3) * 8) = val;
    }
  };

  floatx16 acc[KPW];
#pragma unroll
  for (int j = 0; j < KPW; ++j)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[j][e] = 0.f;
  float bsum = 0.f;

  const int h = lane >> 5;
  const int col = ((lane >> 4) & 1) * 16 + 4 * (lane & 3);
  const int q = (lane & 15) >> 2;

  if (tb < te) load(tb);
  int buf = 0;
  for (int64_t tile = tb; tile < te; ++tile, buf ^= 1) {
    store(buf);
    __syncthreads();
    if (tile + 1 < te) load(tile + 1);
    const __bf16* g = base + buf * (GS + XS);
    const __bf16* x = g + GS;
#pragma unroll
    for (int kh = 0; kh < RROWS / 16; ++kh) {
      const int R = rg * RROWS + kh * 16;
      const v4i16 a0 = tr_read(g + (R + 4 * h + q) * 32 + col);
      const v4i16 a1 = tr_read(g + (R + 8 + 4 * h + q) * 32 + col);
      const bf16x8 A = __builtin_bit_cast(bf16x8, __builtin_shufflevector(a0, a1, 0, 1, 2, 3, 4, 5, 6, 7));
      if (bpart && tg == 0) {
#pragma unroll
        for (int e = 0; e < 8; ++e) bsum += float(A[e]);
      }
#pragma unroll
      for (int j = 0; j < KPW; ++j) {
        const int k = tg + j * TW;
        if (k >= a.K) break;
        const int Rx = R + k * a.dil;
        const v4i16 b0 = tr_read(x + (Rx + 4 * h + q) * 32 + col);
        const v4i16 b1 = tr_read(x + (Rx + 8 + 4 * h + q) * 32 + col);
        const bf16x8 Bf = __builtin_bit_cast(bf16x8, __builtin_shufflevector(b0, b1, 0, 1, 2, 3, 4, 5, 6, 7));
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A, Bf, acc[j], 0, 0, 0);
      }
    }
  }

  // sum the RG row-group partials of every tap, write the split partial
  __syncthreads();
  float* red = reinterpret_cast<float*>(smem);  // [wave][KPW][32*32]
#pragma unroll
  for (int j = 0; j < KPW; ++j) {
    if (tg + j * TW >= a.K) break;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      red[(wave * KPW + j) * 1024 + row * 32 + (lane & 31)] = acc[j][r];
    }
  }
  if (bpart) {
    bsum += __shfl_xor(bsum, 32, 64);
  }
  __syncthreads();
  float* pdst = part + int64_t(blockIdx.z) * a.N * a.K * a.C;
  for (int i = tid; i < a.K * 1024; i += 256) {
    const int k = i >> 10, e = i & 1023;
    const int t = k % TW, j = k / TW;
    float v = 0.f;
#pragma unroll
    for (int r = 0; r < RG; ++r) v += red[((r * TW + t) * KPW + j) * 1024 + e];
    const int n = n0 + (e >> 5), c = c0 + (e & 31);
    pdst[(int64_t(n) * a.K + k) * a.C + c] = v;
  }
  if (bpart && c0 == 0) {
    __syncthreads();
    if (tg == 0 && lane < 32) red[rg * 32 + lane] = bsum;
    __syncthreads();
    if (tid < 32) {
      float v = 0.f;
#pragma unroll
      for (int r = 0; r < RG; ++r) v += red[r * 32 + tid];
      bpart[int64_t(blockIdx.z) * a.N + n0 + tid] = v;
    }
  }
}

// rows of one k_wgrad3_bf16 X plane: the 128-row tile + this layer's halo,
// rounded up to 16 rows (at most W2_BM + W2_HALO)
__host__ __device__ constexpr int wgrad3_xrows(int K, int dil) { return W2_BM + (((K - 1) * dil + 15) & ~15); }

// bf16 weight gradient, general tr-read path (C % 32 == 0, N % 32 == 0,
// halo <= 64, K <= 8).  A block owns NB = 32*NT output channels x CB = 32*CT
// input channels x ALL K taps over a contiguous range of 128-row tiles, so a
// 64x64 layer streams gout and act(in) exactly once (the 32x32 kernel above
// re-read both per (n, c) block).  The TT = NT*CT*K 32x32 accumulator tiles are
// spread over the 4 waves (TPW each, contiguous so consecutive tiles share the
// gout fragment); with TT < 4 the waves split the tile rows instead (RG row
// groups) and meet in LDS.  Operands come from 64-B LDS rows through
// ds_read_b64_tr_b16 (conflict free); the next tile is prefetched into
// registers during the MFMAs.  Grid x = row split (fastest), so the blocks
// sharing a row range are 8-aligned apart... i.e. on the same XCD when the
// split count is a multiple of 8.
template <int NT, int CT, int MAXT, bool PIPE>
__global__ __launch_bounds__(256) void k_wgrad3_bf16(Args a, const __bf16* __restrict__ gout,
                                                     const __bf16* __restrict__ in, int tiles_per_sample,
                                                     int64_t n_tiles, int tiles_per_split,
                                                     float* __restrict__ part, float* __restrict__ bpart) {
  constexpr int NB = 32 * NT, CB = 32 * CT;
  constexpr int XROWS = W2_BM + W2_HALO;
  constexpr int GV = W2_BM * NB / 8 / 256;   // 2*NT
  constexpr int XV = XROWS * CB / 8 / 256;   // 3*CT
  constexpr int GS = NT * W2_BM * 32;
  constexpr int WPN = 4 / NT;                // waves per 32-wide n subtile
  extern __shared__ __align__(16) unsigned char smem[];
  __bf16* const base = reinterpret_cast<__bf16*>(smem);  // [buf]{G[NT][128][32], X[CT][192][32]}

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t split = blockIdx.x;
  const int n0 = blockIdx.y * NB, c0 = blockIdx.z * CB;
  const int64_t tb = split * tiles_per_split;
  const int64_t te = tb + tiles_per_split < n_tiles ? tb + tiles_per_split : n_tiles;
  const int halo = (a.K - 1) * a.dil;
  const int span = W2_BM + halo;
  // X planes sized for this layer's halo (wgrad3_xrows; the launch sizes the LDS
  // the same way): a k1 / k3 layer's blocks need less LDS, more fit on a CU
  const int xrows = wgrad3_xrows(a.K, a.dil);
  const int XS = CT * xrows * 32;
  // wave -> (n subtile, (ct, k) pairs); too few pairs -> the waves split the rows
  const int P = CT * a.K;
  const int RG = P >= WPN ? 1 : WPN / P;     // P in {1, 2} when RG > 1
  const int WPP = WPN / RG;                  // waves sharing the pair list
  const int nt = wave / WPN, wsub = wave % WPN;
  const int rg = wsub / WPP, pw = wsub % WPP;
  const int RROWS = W2_BM / RG;
  const bool do_bias = bpart && blockIdx.z == 0;

  uint4 gr[GV], xr[XV];
  bool gok[GV], xok[XV];
  // branch-free buffer loads over one sample (ru_bload: rows past T / the span,
  // padded rows and a dead request read nothing): the compiler then counts the
  // request exactly, and the MFMA phase no longer waits on it with vmcnt(0)
  auto load = [&](int64_t tile, bool live) {
    const int64_t b = tile / tiles_per_sample;
    const int t0 = int(tile % tiles_per_sample) * W2_BM;
    const int64_t rb = b * a.T;
    const __amdgpu_buffer_rsrc_t rg = ru_rsrc(gout + rb * a.N, int64_t(a.T) * a.N);
    const __amdgpu_buffer_rsrc_t rx = ru_rsrc(in + rb * a.C, int64_t(a.T) * a.C);
#pragma unroll
    for (int u = 0; u < GV; ++u) {
      const int v = tid + u * 256;
      const int t = t0 + v / (NB / 8);
      gok[u] = t < a.T;
      gr[u] = ru_bload(rg, live && gok[u] ? (t * a.N + n0 + (v % (NB / 8)) * 8) * 2 : RU_OOB);
    }
#pragma unroll
    for (int u = 0; u < XV; ++u) {
      const int v = tid + u * 256;
      const int r = v / (CB / 8);
      int ti = t0 - a.pad + r;
      const bool inside = ti >= 0 && ti < a.T;
      xok[u] = r < span && (inside || a.pad_mode == SEL_PAD_REPLICATE);
      ti = ti < 0 ? 0 : (ti >= a.T ? a.T - 1 : ti);
      xr[u] = ru_bload(rx, live && xok[u] ? (ti * a.C + c0 + (v % (CB / 8)) * 8) * 2 : RU_OOB);
    }
  };
  // zero-fill happens here, after the wait (see the v4 forward kernel's store())
  auto store = [&](int buf) {
    __bf16* g = base + buf * (GS + XS);
    __bf16* x = g + GS;
#pragma unroll
    for (int u = 0; u < GV; ++u) {
      const int v = tid + u * 256;
      const int r = v / (NB / 8), c8 = v % (NB / 8);
      *reinterpret_cast<uint4*>(g + (c8 >> 2) * (W2_BM * 32) + r * 32 + (c8 & 3) * 8) =
          gok[u] ? gr[u] : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < XV; ++u) {
      if (u * 256 / (CB / 8) >= span) continue;
      const int v = tid + u * 256;
      const int r = v / (CB / 8), c8 = v % (CB / 8);
      if (r >= span) continue;  // the X planes end at xrows (no tap reads past span - 1)
      uint4 val = xok[u] ? xr[u] : make_uint4(0, 0, 0, 0);
      if (a.in_elu) {
        val = elu8(val);
      }
      *reinterpret_cast<uint4*>(x + (c8 >> 2) * (xrows * 32) + r * 32 + (c8 & 3) * 8) = val;
    }
  };

  // pair j of this wave: p = pw + WPP*j -> (ct, k); slots past P compute into
  // accumulators that are never stored (branch-free MFMA stream)
  int xoff[MAXT];
#pragma unroll
  for (int j = 0; j < MAXT; ++j) {
    int p = pw + WPP * j;
    p = p < P ? p : P - 1;
    xoff[j] = (p / a.K) * (xrows * 32) + (p % a.K) * a.dil * 32;
  }

  floatx16 acc[MAXT];
#pragma unroll
  for (int j = 0; j < MAXT; ++j)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[j][e] = 0.f;
  float bsum = 0.f;
  const int bcol = tid % NB, brow = tid / NB;

  const int h = lane >> 5;
  const int col = ((lane >> 4) & 1) * 16 + 4 * (lane & 3);
  const int q = (lane & 15) >> 2;
  const int lrow = (4 * h + q) * 32 + col;

  if (tb < te) load(tb, true);
  int buf = 0;
  for (int64_t tile = tb; tile < te; ++tile, buf ^= 1) {
    store(buf);
    __syncthreads();
    load(tile + 1 < te ? tile + 1 : tile, tile + 1 < te);  // unconditional: exact counts
    const __bf16* g = base + buf * (GS + XS) + nt * (W2_BM * 32);
    const __bf16* x = base + buf * (GS + XS) + GS;
    if (do_bias) {
      // the column's rows in four independent chains (a single running sum
      // made every 2-byte LDS read wait for the previous one: the bias blocks
      // then trailed the others by ~3 k cycles per tile)
      constexpr int BSTEP = 256 / NB, BN_ = W2_BM / BSTEP;
      const __bf16* gb = base + buf * (GS + XS) + (bcol >> 5) * (W2_BM * 32) + (bcol & 31) + brow * 32;
      float b4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < BN_; ++i) b4[i & 3] += float(gb[i * BSTEP * 32]);
      bsum += (b4[0] + b4[1]) + (b4[2] + b4[3]);
    }
    // fragments of row step kh + 1 are read while step kh's MFMAs run (two
    // register sets, two steps per trip: RROWS / 16 is even)
    struct Frags {
      bf16x8 A, B[MAXT];
    };
    auto fetch = [&](int kh, Frags& f) {
      const int R = (rg * RROWS + kh * 16) * 32 + lrow;
      const v4i16 a0 = tr_read(g + R);
      const v4i16 a1 = tr_read(g + R + 8 * 32);
      f.A = __builtin_bit_cast(bf16x8, __builtin_shufflevector(a0, a1, 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
      for (int j = 0; j < MAXT; ++j) {
        const v4i16 b0 = tr_read(x + xoff[j] + R);
        const v4i16 b1 = tr_read(x + xoff[j] + R + 8 * 32);
        f.B[j] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(b0, b1, 0, 1, 2, 3, 4, 5, 6, 7));
      }
    };
    auto mma = [&](const Frags& f) {
#pragma unroll
      for (int j = 0; j < MAXT; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.A, f.B[j], acc[j], 0, 0, 0);
    };
    const int nk = RROWS / 16;
    if constexpr (PIPE) {
      Frags f0, f1;
      fetch(0, f0);
      for (int kh = 0; kh < nk; kh += 2) {
        fetch(kh + 1, f1);
        mma(f0);
        if (kh + 2 < nk) fetch(kh + 2, f0);
        mma(f1);
      }
    } else {
      // four pairs per wave (the k7 layers) and the short layers (T <= 400):
      // measured 2-6% slower pipelined (the second register set costs
      // occupancy), so one set, one step at a time
      for (int kh = 0; kh < nk; ++kh) {
        Frags f;
        fetch(kh, f);
        mma(f);
      }
    }
  }

  float* pdst = part + split * int64_t(a.N) * a.K * a.C;
  if (RG == 1) {
#pragma unroll
    for (int j = 0; j < MAXT; ++j) {
      const int p = pw + WPP * j;
      if (p >= P) break;
      const int ct = p / a.K, k = p % a.K;
      const int c = c0 + ct * 32 + (lane & 31);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int n = n0 + nt * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        pdst[(int64_t(n) * a.K + k) * a.C + c] = acc[j][r];
      }
    }
  } else {
    // RG > 1 only for P < WPN, i.e. MAXT slots hold at most one pair per wave
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
      const int ct = pi / a.K, k = pi % a.K;
      const int n = n0 + ni * 32 + (e >> 5), c = c0 + ct * 32 + (e & 31);
      pdst[(int64_t(n) * a.K + k) * a.C + c] = v;
    }
  }
  if (do_bias) {
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem);
    red[tid] = bsum;
    __syncthreads();
    if (tid < NB) {
      float v = 0.f;
      for (int r = 0; r < 256 / NB; ++r) v += red[r * NB + tid];
      bpart[split * a.N + n0 + tid] = v;
    }
  }
}

// Deterministic split reduction in two parallel passes:
//   pass 1: part2[g][i] = sum_{s in group g (32 splits)} part[s][i]   (grid: i-blocks x groups)
//   pass 2: out[j] = sum_g sum_{i % period == j} part2[g][i]
constexpr int SPLIT_GROUP = 32;

// sum of the partials p[0], p[n], ... p[(cnt - 1) n] of one split group (cnt <= 32)
template <int W>
__device__ __forceinline__ float split_tree(const float* __restrict__ p, int cnt, int64_t n) {
  // W loads in flight at once (slots past cnt hold exact zeros), then a fixed
  // pairwise tree: deterministic for a given cnt
  float v[W];
#pragma unroll
  for (int u = 0; u < W; ++u) v[u] = u < cnt ? p[int64_t(u) * n] : 0.f;
#pragma unroll
  for (int w = 1; w < W; w *= 2)
#pragma unroll
    for (int u = 0; u < W; u += 2 * w) v[u] += v[u + w];
  return v[0];
}
__device__ __forceinline__ float split_group_sum(const float* __restrict__ p, int cnt, int64_t n,
                                                 bool four_at_a_time = false) {
  // a full group: all 32 loads in flight at once (a serial chain of dependent
  // adds made the compiler issue them a few at a time: latency-bound)
  if (cnt == SPLIT_GROUP) return split_tree<SPLIT_GROUP>(p, cnt, n);
  // partial groups (round 6: the RU256 k7 layers' 16 splits, 29 MB each, went
  // four loads per round trip): the smallest power-of-two tree holding cnt;
  // tune key 68 = 1: the four-at-a-time loop
  if (!four_at_a_time) {
    if (cnt > 16) return split_tree<32>(p, cnt, n);
    if (cnt > 8) return split_tree<16>(p, cnt, n);
    if (cnt > 4) return split_tree<8>(p, cnt, n);
    return split_tree<4>(p, cnt, n);
  }
  float acc = 0.f;
  int u = 0;
  for (; u + 4 <= cnt; u += 4) {
    const float a0 = p[int64_t(u) * n], a1 = p[int64_t(u + 1) * n], a2 = p[int64_t(u + 2) * n],
                a3 = p[int64_t(u + 3) * n];
    acc += (a0 + a1) + (a2 + a3);
  }
  for (; u < cnt; ++u) acc += p[int64_t(u) * n];
  return acc;
}

__global__ __launch_bounds__(256) void k_split_sum1(const float* __restrict__ part, int nsplit, int64_t n,
                                                    float* __restrict__ part2) {
  const int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x;
  if (i >= n) return;
  const int s0 = blockIdx.y * SPLIT_GROUP;
  const int s1 = s0 + SPLIT_GROUP < nsplit ? s0 + SPLIT_GROUP : nsplit;
  part2[int64_t(blockIdx.y) * n + i] = split_group_sum(part + int64_t(s0) * n + i, s1 - s0, n);
}

__global__ __launch_bounds__(256) void k_split_sum2(const float* __restrict__ part2, int ngroups, int64_t n,
                                                    int period, float* __restrict__ out) {
  const int64_t j = int64_t(blockIdx.x) * 256 + threadIdx.x;
  if (j >= period) return;
  float acc = 0.f;
  for (int g = 0; g < ngroups; ++g)
    for (int64_t i = j; i < n; i += period) acc += part2[int64_t(g) * n + i];
  out[j] = acc;
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

// Multi-tensor pack: every job's fwd pack Wp and (optionally) its dgrad form Wd
// in ONE launch (the per-layer launches of sel_pack_weight + sel_pack_dgrad were
// ~120 x 4 us per training step).  Grid-stride over TWO ranges of the
// concatenated packed elements: [0, total) writes Wp in its own order, [total,
// 2 total) writes Wd in ITS own order (gathering the source element), so both
// write streams are coalesced (writing Wd as the transpose of the Wp walk made
// every 2-B store its own partial line: 45 us per C3 step).  A thread
// binary-searches its job in the device job table.
template <typename TO>
__global__ void k_pack_many(const sel_pack_job* __restrict__ jobs, int njobs, int64_t total) {
  for (int64_t i2 = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i2 < 2 * total;
       i2 += int64_t(gridDim.x) * blockDim.x) {
    const bool dg = i2 >= total;  // dgrad-form range
    const int64_t i = dg ? i2 - total : i2;
    int lo = 0, hi = njobs - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (jobs[mid].offset <= i) lo = mid;
      else hi = mid - 1;
    }
    const sel_pack_job& J = jobs[lo];
    if (dg && !J.wdgrad) continue;
    // a layer's packed index fits 32 bits (host-checked): unsigned 32-bit
    // division instead of the 64-bit sequences (the per-step pack of the C3
    // weights took 105 us with them)
    const unsigned li = unsigned(i - J.offset);
    const unsigned s = unsigned(J.stride), cin = unsigned(J.cin), cout = unsigned(J.cout), K = unsigned(J.k);
    // packed geometry: Wp[n][kp][cp] (N rows, KP taps, CP channels per tap)
    unsigned N, KP, CP;
    if (J.kind == SEL_PACK_FWD) N = cout, KP = K, CP = cin;
    else if (J.kind == SEL_PACK_FWD_STRIDED) N = cout, KP = 3, CP = s * cin;
    else N = s * cout, KP = 2, CP = cin;
    unsigned n, kp, cp;
    if (!dg) {  // li = (n * KP + kp) * CP + cp
      const unsigned q = li / CP;
      cp = li - q * CP;
      n = q / KP;
      kp = q - n * KP;
    } else {  // Wd[c][j][n] = Wp[n][KP-1-j][c]: li = (cp * KP + j) * N + n
      const unsigned r = li / N;
      n = li - r * N;
      cp = r / KP;
      kp = KP - 1 - (r - cp * KP);
    }
    float v = 0.f;
    if (J.kind == SEL_PACK_FWD) {
      v = J.w[(n * cin + cp) * K + kp];
    } else if (J.kind == SEL_PACK_FWD_STRIDED) {
      const unsigned ph = cp / cin, ci = cp - ph * cin;
      const int k = strided_k(int(kp), int(ph), int(s));
      v = k >= 0 ? J.w[(n * cin + ci) * (2 * s) + unsigned(k)] : 0.f;
    } else {
      const unsigned ph = n / cout, co = n - ph * cout;
      const unsigned k = kp == 0 ? ph + s : ph;
      v = J.w[(cp * cout + co) * (2 * s) + k];
    }
    static_cast<TO*>(dg ? J.wdgrad : J.wpack)[li] = from_f<TO>(v);
  }
}

// The same with the job table in the kernel arguments (sel_pack_many_host): no
// device copy of the table, hence no pinned staging and no host-to-device copy
// in the step (the pinned allocation + copy per weight update of the device-table
// form left the GPU idle ~0.3 ms per C3 step while the host waited on them).
// A launch packs the element range [lo, hi) of `total` that its jobs cover.
constexpr int PM_MAXJ = 48;
struct PackJobs {
  sel_pack_job j[PM_MAXJ];
  int n;
};
template <typename TO>
__global__ void k_pack_many_arg(PackJobs pj, int64_t lo, int64_t hi, int64_t total) {
  const int64_t len = hi - lo;
  for (int64_t i2 = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i2 < 2 * len;
       i2 += int64_t(gridDim.x) * blockDim.x) {
    const bool dg = i2 >= len;
    const int64_t i = lo + (dg ? i2 - len : i2);
    int a = 0, b = pj.n - 1;
    while (a < b) {
      const int mid = (a + b + 1) >> 1;
      if (pj.j[mid].offset <= i) a = mid;
      else b = mid - 1;
    }
    const sel_pack_job& J = pj.j[a];
    if (dg && !J.wdgrad) continue;
    const unsigned li = unsigned(i - J.offset);
    const unsigned s = unsigned(J.stride), cin = unsigned(J.cin), cout = unsigned(J.cout), K = unsigned(J.k);
    unsigned N, KP, CP;
    if (J.kind == SEL_PACK_FWD) N = cout, KP = K, CP = cin;
    else if (J.kind == SEL_PACK_FWD_STRIDED) N = cout, KP = 3, CP = s * cin;
    else N = s * cout, KP = 2, CP = cin;
    unsigned n, kp, cp;
    if (!dg) {
      const unsigned q = li / CP;
      cp = li - q * CP;
      n = q / KP;
      kp = q - n * KP;
    } else {
      const unsigned r = li / N;
      n = li - r * N;
      cp = r / KP;
      kp = KP - 1 - (r - cp * KP);
    }
    float v = 0.f;
    if (J.kind == SEL_PACK_FWD) {
      v = J.w[(n * cin + cp) * K + kp];
    } else if (J.kind == SEL_PACK_FWD_STRIDED) {
      const unsigned ph = cp / cin, ci = cp - ph * cin;
      const int k = strided_k(int(kp), int(ph), int(s));
      v = k >= 0 ? J.w[(n * cin + ci) * (2 * s) + unsigned(k)] : 0.f;
    } else {
      const unsigned ph = n / cout, co = n - ph * cout;
      const unsigned k = kp == 0 ? ph + s : ph;
      v = J.w[(cp * cout + co) * (2 * s) + k];
    }
    static_cast<TO*>(dg ? J.wdgrad : J.wpack)[li] = from_f<TO>(v);
  }
  (void)total;
}

// Tiled form of k_pack_many_arg (the product's per-step repack): a workgroup
// owns a 32 (n) x 32 (cp) x KP tile of one job's packed geometry, gathers it
// from the torch-layout weight with (cp, kp)-contiguous reads into an fp32 LDS
// tile, then writes the tile's forward form Wp[n][kp][cp] (32 consecutive cp per
// run) and its dgrad form Wd[cp][KP-1-kp][n] (32 consecutive n per run): both
// forms leave as coalesced runs.  The per-element form gathered the dgrad
// form's source across whole weight rows (one cache line per lane): 72 us per
// C3 step for 31 MB of traffic (rocprof, profiles/r6f_kernel_stats.md).  Same
// values (a copy with the same rounding).
constexpr int PT_T = 32, PT_KMAX = 8, PT_P = PT_T + 1;
struct PackTiles {
  sel_pack_job j[PM_MAXJ];
  int tstart[PM_MAXJ + 1];  // first tile of each job; tstart[n] = tile count
  int n;
};
__device__ __forceinline__ void pack_geom(const sel_pack_job& J, unsigned& N, unsigned& KP, unsigned& CP) {
  const unsigned s = unsigned(J.stride), cin = unsigned(J.cin), cout = unsigned(J.cout), K = unsigned(J.k);
  if (J.kind == SEL_PACK_FWD) N = cout, KP = K, CP = cin;
  else if (J.kind == SEL_PACK_FWD_STRIDED) N = cout, KP = 3, CP = s * cin;
  else N = s * cout, KP = 2, CP = cin;
}
// 1024 threads: one (n, cp) pair of the 32 x 32 tile per thread, with all its
// KP taps, so no index needs a division by the job's tap count, and the KP
// loads of a pair are all issued before its LDS stores.  (At 256 threads, four
// elements a thread one after another, the small launches of a C3 step -- 32-64
// tiles, one workgroup each -- took 17-18 us; now 6-7 us, and the 640-tile
// launch 11.4 -> 9.8 us.)
template <typename TO, unsigned PT_THREADS>
__global__ __launch_bounds__(PT_THREADS) void k_pack_tiles(PackTiles pt) {
  __shared__ float tile[PT_T * PT_KMAX * PT_P];
  int a = 0, b = pt.n - 1;
  const int t = int(blockIdx.x);
  while (a < b) {  // block-uniform
    const int mid = (a + b + 1) >> 1;
    if (pt.tstart[mid] <= t) a = mid;
    else b = mid - 1;
  }
  const sel_pack_job& J = pt.j[a];
  unsigned N, KP, CP;
  pack_geom(J, N, KP, CP);
  const unsigned s = unsigned(J.stride), cin = unsigned(J.cin), cout = unsigned(J.cout), K = unsigned(J.k);
  const unsigned ntc = (CP + PT_T - 1) / PT_T;
  const unsigned lt = unsigned(t - pt.tstart[a]);
  const unsigned n0 = (lt / ntc) * PT_T, c0 = (lt % ntc) * PT_T;
  // gather: pair (nl, cl), cl fastest; its KP taps are contiguous in the FWD
  // source; out-of-range taps load w[0] and are replaced by zeros
  for (unsigned r = threadIdx.x; r < PT_T * PT_T; r += PT_THREADS) {
    const unsigned cl = r % PT_T, nl = r / PT_T;
    const unsigned n = n0 + nl, cp = c0 + cl;
    const bool in = n < N && cp < CP;
    unsigned base = 0, ph = 0;
    if (J.kind == SEL_PACK_FWD) {
      base = (n * cin + cp) * K;
    } else if (J.kind == SEL_PACK_FWD_STRIDED) {
      ph = cp / cin;
      base = (n * cin + (cp - ph * cin)) * (2 * s);
    } else {
      ph = n / cout;
      base = (cp * cout + (n - ph * cout)) * (2 * s);
    }
    float v[PT_KMAX];
    bool ok[PT_KMAX];
#pragma unroll
    for (unsigned kp = 0; kp < PT_KMAX; ++kp) {
      if (kp >= KP) break;  // block-uniform
      int k = int(kp);
      if (J.kind == SEL_PACK_FWD_STRIDED) k = strided_k(int(kp), int(ph), int(s));
      else if (J.kind == SEL_PACK_CONVT) k = int(kp == 0 ? ph + s : ph);
      ok[kp] = in && k >= 0;
      v[kp] = J.w[ok[kp] ? base + unsigned(k) : 0];
    }
#pragma unroll
    for (unsigned kp = 0; kp < PT_KMAX; ++kp) {
      if (kp >= KP) break;
      tile[(nl * KP + kp) * PT_P + cl] = ok[kp] ? v[kp] : 0.f;
    }
  }
  __syncthreads();
  TO* const wp = static_cast<TO*>(J.wpack);
  for (unsigned r = threadIdx.x; r < PT_T * PT_T; r += PT_THREADS) {  // Wp[n][kp][cp]: cp fastest
    const unsigned cl = r % PT_T, nl = r / PT_T;
    const unsigned n = n0 + nl, cp = c0 + cl;
    if (n < N && cp < CP)
      for (unsigned kp = 0; kp < KP; ++kp) wp[(n * KP + kp) * CP + cp] = from_f<TO>(tile[(nl * KP + kp) * PT_P + cl]);
  }
  if (J.wdgrad) {
    TO* const wd = static_cast<TO*>(J.wdgrad);
    for (unsigned r = threadIdx.x; r < PT_T * PT_T; r += PT_THREADS) {  // Wd[cp][j][n]: n fastest
      const unsigned nl = r % PT_T, cl = r / PT_T;
      const unsigned n = n0 + nl, cp = c0 + cl;
      if (n < N && cp < CP)
        for (unsigned j = 0; j < KP; ++j)
          wd[(cp * KP + j) * N + n] = from_f<TO>(tile[(nl * KP + (KP - 1 - j)) * PT_P + cl]);
    }
  }
}

// Packed index of torch-layout weight element i (the gather map of k_unpack).
__device__ __forceinline__ int64_t unpack_src(int kind, int64_t i, int cout, int cin, int K, int s) {
  if (kind == SEL_PACK_FWD) {
    const int k = int(i % K);
    const int ci = int((i / K) % cin);
    const int co = int(i / (int64_t(K) * cin));
    return (int64_t(co) * K + k) * cin + ci;
  }
  const int KK = 2 * s;
  const int k = int(i % KK);
  if (kind == SEL_PACK_FWD_STRIDED) {
    const int ci = int((i / KK) % cin);
    const int co = int(i / (int64_t(KK) * cin));
    int tap, ph;
    if (k <= s - 2) { tap = 0; ph = k + 1; }
    else if (k <= 2 * s - 2) { tap = 1; ph = k - s + 1; }
    else { tap = 2; ph = 0; }
    return (int64_t(co) * 3 + tap) * (int64_t(s) * cin) + ph * cin + ci;
  }
  const int co = int((i / KK) % cout);
  const int ci = int(i / (int64_t(KK) * cout));
  const int ph = k < s ? k : k - s;
  const int tap = k < s ? 1 : 0;
  return (int64_t(ph * cout + co) * 2 + tap) * cin + ci;
}

// Second reduction pass fused with the unpack: gw (torch layout) = sum over the
// split groups of the packed partials (one launch instead of two per layer).
__global__ __launch_bounds__(256) void k_split_sum2_unpack(const float* __restrict__ part2, int ngroups, int64_t n,
                                                           int64_t n_torch, int kind, int cout, int cin, int K,
                                                           int s, float* __restrict__ gw) {
  const int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x;
  if (i >= n_torch) return;
  const int64_t j = unpack_src(kind, i, cout, cin, K, s);
  const float* p = part2 + j;
  float acc = 0.f;
  int g = 0;
  for (; g + 4 <= ngroups; g += 4) {  // 4 loads in flight, fixed order
    const float a0 = p[int64_t(g) * n], a1 = p[int64_t(g + 1) * n], a2 = p[int64_t(g + 2) * n],
                a3 = p[int64_t(g + 3) * n];
    acc += (a0 + a1) + (a2 + a3);
  }
  for (; g < ngroups; ++g) acc += p[int64_t(g) * n];
  gw[i] = acc;
}

// One split group (nsplit <= 32): both reduction passes, the unpack and the bias
// fold in one launch, with the arithmetic of k_split_sum1 + k_split_sum2(_unpack)
// (the second pass adds one group sum to 0, exactly): threads [0, nt) write the
// weight gradient (torch layout when kind >= 0, else the packed one), threads
// [nt, nt + period) the bias.
__global__ __launch_bounds__(256) void k_split_finish1(const float* __restrict__ part, int nsplit, int64_t nw,
                                                       int64_t nt, int kind, int cout, int cin, int K, int s,
                                                       float* __restrict__ gw, const float* __restrict__ bpart,
                                                       int64_t nb, int period, float* __restrict__ gb) {
  const int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x;
  if (i < nt) {
    const int64_t j = kind >= 0 ? unpack_src(kind, i, cout, cin, K, s) : i;
    gw[i] = 0.f + split_group_sum(part + j, nsplit, nw);
  } else if (gb && i < nt + period) {
    const int64_t jb = i - nt;
    float acc = 0.f;
    for (int64_t q = jb; q < nb; q += period) acc += split_group_sum(bpart + q, nsplit, nb);
    gb[jb] = acc;
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

// adjoint of the replicate pad: gin[b*T, c] += sum_n gout[b*T, n] * Wp[n][0][c]
// block = (sample b, 64 channels); 16 waves split n, LDS reduce.
template <typename T>
__global__ __launch_bounds__(1024) void k_replicate_fix(Args a, const T* __restrict__ gout, const T* __restrict__ wp,
                                                        T* __restrict__ gin) {
  __shared__ float red[16][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t row = int64_t(blockIdx.x) * a.T;
  const int c = blockIdx.y * 64 + lane;
  float s = 0.f;
  if (c < a.C) {
    // 8 (gout, weight) pairs in flight per step, summed in the same n order
    int n = wave;
    for (; n + 16 * 7 < a.N; n += 16 * 8) {
      float gv[8], wv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        gv[u] = to_f(gout[row * a.N + n + 16 * u]);
        wv[u] = to_f(wp[(int64_t(n + 16 * u) * a.K + 0) * a.C + c]);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) s += gv[u] * wv[u];
    }
    for (; n < a.N; n += 16) s += to_f(gout[row * a.N + n]) * to_f(wp[(int64_t(n) * a.K + 0) * a.C + c]);
  }
  red[wave][lane] = s;
  __syncthreads();
  if (wave == 0 && c < a.C) {
    float t = 0.f;
    for (int w = 0; w < 16; ++w) t += red[w][lane];
    gin[row * a.C + c] = from_f<T>(to_f(gin[row * a.C + c]) + t);
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
  a.tin_valid = a.tin_pitch = a.tout_valid = d->T;
  a.ldx = d->C;
  a.ldo = d->N;
  a.epi = a.act = 0;
  a.slope = 0.f;
  a.seq_pitch = 0;
  return a;
}

template <typename TI, typename TO, int BM, int BN>
size_t fwd_lds(const Args& a) {
  const size_t stage = (size_t(BM + (a.K - 1) * a.dil) + size_t(a.K) * BN) * Pitch<TI>::v * sizeof(TI);
  const size_t epi = size_t(BM) * (BN + 4) * sizeof(float);
  return stage > epi ? stage : epi;
}

template <typename TI, typename TO, int BM, int BN>
int launch_fwd(const Args& a, const void* in, const void* wp, const float* bias, const void* aux,
               const void* res, void* out, hipStream_t s) {
  const size_t lds = fwd_lds<TI, TO, BM, BN>(a);
  SEL_REQUIRE(lds <= 160 * 1024, SEL_ERR_UNSUPPORTED, "conv tile needs %zu B of LDS", lds);
  dim3 grid(unsigned((a.rows + BM - 1) / BM), unsigned((a.N + BN - 1) / BN));
  if (grid.x == 0) return SEL_OK;
  auto kern = k_conv_fwd<TI, TO, BM, BN>;
  if (lds > 64 * 1024)
    SEL_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, int(lds)));
  hipLaunchKernelGGL(kern, grid, dim3(256), lds, s, a, static_cast<const TI*>(in),
                     static_cast<const TI*>(wp), bias, static_cast<const TO*>(aux),
                     static_cast<const TO*>(res), static_cast<TO*>(out));
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

template <int BM, int BN>
int launch_fwd_f32(const Args& a, const void* in, const void* wp, const float* bias, const void* aux,
                   const void* res, void* out, hipStream_t s) {
  const size_t stage = (size_t(BM + FF_HALO) + size_t(a.K) * BN) * FF_P * sizeof(float);
  const size_t epi = size_t(BM) * (BN + 4) * sizeof(float);
  const size_t lds = stage > epi ? stage : epi;
  const int64_t tiles = (a.rows / a.T) * ((a.T + BM - 1) / BM);  // sample-aligned tiles
  if (tiles == 0) return SEL_OK;
  dim3 grid(unsigned(tiles), unsigned(a.N / BN));
  const void* kern = a.K == 1 ? (const void*)k_conv_fwd_f32<1, BM, BN>
                     : a.K <= 3 ? (const void*)k_conv_fwd_f32<3, BM, BN> : (const void*)k_conv_fwd_f32<8, BM, BN>;
  if (lds > 64 * 1024) SEL_HIP(hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, int(lds)));
  const float* x = static_cast<const float*>(in);
  const float* w = static_cast<const float*>(wp);
  const float* ax = static_cast<const float*>(aux);
  const float* rs = static_cast<const float*>(res);
  float* o = static_cast<float*>(out);
  if (a.K == 1)
    hipLaunchKernelGGL((k_conv_fwd_f32<1, BM, BN>), grid, dim3(256), lds, s, a, x, w, bias, ax, rs, o);
  else if (a.K <= 3)
    hipLaunchKernelGGL((k_conv_fwd_f32<3, BM, BN>), grid, dim3(256), lds, s, a, x, w, bias, ax, rs, o);
  else
    hipLaunchKernelGGL((k_conv_fwd_f32<8, BM, BN>), grid, dim3(256), lds, s, a, x, w, bias, ax, rs, o);
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

template <int BM, int BN, int WAVES_M, int KMAX, typename TO>
int launch_fwd4(const Args& a, const void* in, const void* wp, const float* bias, const void* aux,
                const void* res, void* out, hipStream_t s) {
  const int span = BM + (a.K - 1) * a.dil;
  const size_t lds = (size_t(span) + size_t(a.K) * BN) * F4_P * 2;
  const int64_t tiles = (a.rows / a.T) * ((a.T + BM - 1) / BM);  // sample-aligned tiles
  const int ncol = (a.N + BN - 1) / BN;
  if (tiles == 0) return SEL_OK;
  // tune key 8 = 1: plain 2-D grid instead of the XCD-aware 1-D order
  const bool xcd = ncol > 1 && tune(8) == 0 && tiles * ncol < (int64_t(1) << 31);
  const dim3 grid = xcd ? dim3(unsigned(tiles * ncol)) : dim3(unsigned(tiles), unsigned(ncol));
  auto kern = k_conv_fwd_bf16<BM, BN, WAVES_M, KMAX, TO>;
  if (lds > 64 * 1024)
    SEL_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, int(lds)));
  hipLaunchKernelGGL(kern, grid, dim3(256), lds, s, a, static_cast<const __bf16*>(in),
                     static_cast<const __bf16*>(wp), bias, static_cast<const TO*>(aux), static_cast<const TO*>(res),
                     static_cast<TO*>(out), xcd ? ncol : 0);
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

// (measured and dropped in round 2: four consumer waves of 128 x 64, two
// chunks per barrier for the two-tap layers)
template <int KT, typename TO>
int launch_ws(const Args& a, const void* in, const void* wp, const float* bias, const void* aux, const void* res,
              void* out, hipStream_t s) {
  const size_t lds = ws_lds_bytes(KT, 1);
  const int64_t tiles = (a.rows / a.T) * ((a.T + WS_BM - 1) / WS_BM);
  const int ncol = a.N / WS_BN;
  if (tiles == 0) return SEL_OK;
  const bool xcd = ncol > 1 && tune(8) == 0 && tiles * ncol < (int64_t(1) << 31);
  const dim3 grid = xcd ? dim3(unsigned(tiles * ncol)) : dim3(unsigned(tiles), unsigned(ncol));
  auto kern = k_conv_ws_bf16<KT, TO, 8, 1>;
  SEL_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, int(lds)));
  hipLaunchKernelGGL(kern, grid, dim3(768), lds, s, a, static_cast<const __bf16*>(in),
                     static_cast<const __bf16*>(wp), bias, static_cast<const TO*>(aux), static_cast<const TO*>(res),
                     static_cast<TO*>(out), xcd ? ncol : 0, tune(13));
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

template <int KT, typename TO, int BM, int BN, int HALO, int TM = 4>
int launch_ws8(const Args& a, const void* in, const void* wp, const float* bias, const void* aux, const void* res,
               void* out, hipStream_t s) {
  using G = Ws8<KT, BM, BN, HALO, TM>;
  SEL_REQUIRE(a.K == KT && a.N % BN == 0 && a.C % WS_CK == 0 && a.C <= WS_CMAX && (KT - 1) * a.dil <= HALO &&
                  a.T > 0 && a.rows % a.T == 0,
              SEL_ERR_ARG, "k_conv_ws8<%d, %d, %d>: bad shape C=%d N=%d K=%d dil=%d", KT, BM, BN, a.C, a.N, a.K,
              a.dil);
  const int64_t tiles = (a.rows / a.T) * ((a.T + BM - 1) / BM);
  const int ncol = a.N / BN;
  if (tiles == 0) return SEL_OK;
  const bool xcd = ncol > 1 && tune(8) == 0 && tiles * ncol < (int64_t(1) << 31);
  const dim3 grid = xcd ? dim3(unsigned(tiles * ncol)) : dim3(unsigned(tiles), unsigned(ncol));
  auto kern = k_conv_ws8<KT, TO, BM, BN, HALO, TM>;
  SEL_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, int(G::LDS)));
  hipLaunchKernelGGL(kern, grid, dim3(512), G::LDS, s, a, static_cast<const __bf16*>(in),
                     static_cast<const __bf16*>(wp), bias, static_cast<const TO*>(aux), static_cast<const TO*>(res),
                     static_cast<TO*>(out), xcd ? ncol : 0, tune(13));
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

// the eight-wave kernel's 512 x 128 tiles for the 128-wide k7 layers (legal
// shapes; forced with tune key 0 = 28)
bool ws8_gen_ok(const Args& a) {
  return a.K == 7 && a.N == 128 && a.C % WS_CK == 0 && a.C <= WS_CMAX && (a.K - 1) * a.dil <= 64 && a.T >= 1024;
}
// ... and where the heuristic takes them: the k7 dgrads at >= 64 k rows (the C3
// RU128 dgrads at T = 2000: 4 tiles per sample, 256 per launch); tune key 37:
// 1 = off (the 12-wave kernel), 2 = the ELU-prologue forwards too
bool ws8_gen_pick(const Args& a) {
  return tune(37) != 1 && ws8_gen_ok(a) && a.rows >= 65536 && ((a.pad == 0 && !a.in_elu) || tune(37) == 2);
}
// eight waves of 64 x 64 on the 12-wave kernel's 256 x 128 tile (variant 29):
// the 256-wide K = 3 / 7 layers at T = 400; tune key 38 = 1: on
bool ws8w_ok(const Args& a) {
  return (a.K == 7 || a.K == 3) && a.N % 128 == 0 && a.C % WS_CK == 0 && a.C <= WS_CMAX &&
         (a.K - 1) * a.dil <= 64;
}

// the warp-specialised kernel's legal shapes: K in {3, 7}, 128-multiple N,
// 16-multiple C within the zero source, halo within the staged span, the
// 4-slot ring within 160 KB
bool ws_ok(const Args& a) {
  // (K = 2: the phase-view transposed convs and their adjoints, round 4;
  // tune key 46 = 1: those on the tiled kernel again)
  return ((a.K == 2 && tune(46) != 1) || a.K == 3 || a.K == 7) && a.N % WS_BN == 0 && a.C % WS_CK == 0 && a.C <= WS_CMAX &&
         (a.K - 1) * a.dil <= F4_HALOMAX && ws_lds_bytes(a.K) <= 160 * 1024;
}

template <typename TO>
int launch_ws_k(const Args& a, const void* in, const void* wp, const float* bias, const void* aux, const void* res,
                void* out, hipStream_t s) {
  return a.K == 7 ? launch_ws<7, TO>(a, in, wp, bias, aux, res, out, s)
         : a.K == 3 ? launch_ws<3, TO>(a, in, wp, bias, aux, res, out, s)
                    : launch_ws<2, TO>(a, in, wp, bias, aux, res, out, s);
}


// Variant the dispatcher picks for a bf16 forward launch (see fwd4_variant);
// -1 when the generic (non-pipelined) kernel is used.
// the sample-tile kernel (conv_wss.hip, variant 30) for the 256-wide layers at
// T = 400: tune key 47 = 1 on, 2 off, 0 = kWssDefault
constexpr bool kWssDefault = true;
bool wss_pick(const Args& a) {
  const int k = tune(47);
  int S = 0, tm = 0;
  // (at T = 2000 not the replicate-pad transposed conv 128 -> 256 phases:
  // tools/conv_bench.py 49.6 us on k_conv_ws_bf16 against 53.0)
  return (k == 1 || (k == 0 && kWssDefault)) && a.N >= 256 && a.rows >= 16384 && wss_ok(a) &&
         wss_geometry(a, S, tm) && (S == 25 || a.pad_mode == SEL_PAD_ZERO);
}
// ... and its 512-row tiles (S = 32) for the 128-wide layers at T = 2000 without an
// input ELU or replicate pad (the k7 / k3 / k2 adjoints and the s4 down conv:
// tools/conv_bench.py RU128 k7d9 dgrad 47.3 -> 40.9 us, down1 45.3 -> 43.2; the
// ELU'd forwards gain nothing, the replicate-pad up conv loses); tune key 50:
// 1 = on, 2 = off, 0 = kWssTallDefault
constexpr bool kWssTallDefault = true;
bool wss_pick_tall(const Args& a) {
  const int k = tune(50);
  int S = 0, tm = 0;
  return (k == 1 || (k == 0 && kWssTallDefault)) && a.N == 128 && a.rows >= 65536 && !a.in_elu &&
         a.pad_mode == SEL_PAD_ZERO && wss_ok(a) && wss_geometry(a, S, tm) && S == 32;
}
// the (16, 128) tiles for the ELU'd 128-wide forwards at T = 2000 (tune key 52:
// 1 = on, 2 = off, 0 = kWssEluDefault): tools/conv_bench.py RU128 k7d9 fwd
// 49.4 (k_conv_fwd_bf16<256, 64>) -> 43.9 us; neutral in the step (the
// launches overlap the side-stream weight gradients)
constexpr bool kWssEluDefault = true;
bool wss_pick_elu(const Args& a) {
  const int k = tune(52);
  int S = 0, tm = 0;
  return (k == 1 || (k == 0 && kWssEluDefault)) && a.N == 128 && a.rows >= 65536 && a.in_elu &&
         a.pad_mode == SEL_PAD_ZERO && wss_ok(a) && wss_geometry(a, S, tm) && S == 16;
}

// out_f32: an fp32-output launch (the sample-tile kernel takes those at T <= 400
// only, wss_ok_out; fwd4_variant's dispatch applies the same condition)
// the sample-tile kernel on five-sample tiles for the T = 80 layers (the C3
// down / up convs at the 512-wide stage and their adjoints run on 128 x 32 tiles
// at 80 of 128 rows per tile).  Measured in round 6: 55.7 -> 52.7, 50.6 -> 45.4,
// 46.2 -> 44.8 us for the wide layers, but 14.9 -> 23.3 and 22.2 -> 39.2 us at
// N = 64 (13 tiles per 64-wide column are too few workgroups), and the step
// unchanged or slower in same-call A/Bs either way (5.42-5.46 off, 5.47-5.48
// for N >= 512, 5.50-5.51 everywhere).  So off by default; tune key 67: 1 = on
// wherever it applies, 3 = for N >= 512 only
bool wss_pick_short(const Args& a) {
  const int k = tune(67);
  return (k == 1 || (k == 3 && a.N >= 512)) && wss_spt(a) > 1 && a.N % 64 == 0 && wss_ok(a);
}

int fwd4_choice(const Args& a, bool out_f32) {
  const int v = tune(0);
  if (!((a.C % CK) == 0 && (a.K - 1) * a.dil <= F4_HALOMAX && a.K <= 8 && (v == 0 || v > 20))) return -1;
  if (v > 20 && (v != 27 || ws_ok(a)) && (v != 28 || ws8_gen_ok(a)) && (v != 29 || ws8w_ok(a)) &&
      (v != 30 || wss_ok_out(a, out_f32)))
    return v;
  // (the T = 80 layers: 128 x 64 / 128 x 128 / 64 x 128 tiles measured 13-50 us
  // slower per graph-replayed C3 step, round 6)
  if (wss_pick_short(a) && wss_ok_out(a, out_f32)) return 30;
  if (a.N <= 32 || (a.N % 64) != 0 || a.rows < 8192) return 22;
  if (a.N >= 256 && a.K == 1) return 26;
  if (a.N >= 256 && a.rows >= 16384)
    return wss_pick(a) && wss_ok_out(a, out_f32) ? 30 : tune(38) == 1 && ws8w_ok(a) ? 29 : ws_ok(a) ? 27 : 24;
  if (a.N <= 64 || a.rows < 65536) return 23;
  if ((wss_pick_tall(a) || wss_pick_elu(a)) && wss_ok_out(a, out_f32)) return 30;
  if (ws8_gen_pick(a)) return 28;
  if (a.N == 128 && ws_ok(a) && (a.K <= 3 || (a.K == 7 && a.pad == 0 && !a.in_elu))) return 27;
  if (a.N == 128 && a.K > 1 && a.pad == 0 && !a.in_elu) return 22;
  return 24;
}

template <int KMAX, typename TO>
int fwd4_variant(int v, const Args& a, const void* in, const void* wp, const float* bias, const void* aux,
                 const void* res, void* out, hipStream_t s) {
  switch (v) {
    case 21: return launch_fwd4<256, 32, 4, KMAX, TO>(a, in, wp, bias, aux, res, out, s);
    case 22: return launch_fwd4<128, 32, 4, KMAX, TO>(a, in, wp, bias, aux, res, out, s);
    case 23: return launch_fwd4<128, 64, 2, KMAX, TO>(a, in, wp, bias, aux, res, out, s);
    case 24: return launch_fwd4<256, 64, 4, KMAX, TO>(a, in, wp, bias, aux, res, out, s);
    case 25: return launch_fwd4<128, 128, 2, KMAX, TO>(a, in, wp, bias, aux, res, out, s);
    case 26: return launch_fwd4<64, 128, 1, KMAX, TO>(a, in, wp, bias, aux, res, out, s);
    case 27:
      if (!ws_ok(a)) break;
      return launch_ws_k<TO>(a, in, wp, bias, aux, res, out, s);
    case 28:
      if (!ws8_gen_ok(a)) break;
      return launch_ws8<7, TO, 512, 128, 64>(a, in, wp, bias, aux, res, out, s);
    case 29:
      if (!ws8w_ok(a)) break;
      if (a.K == 7) return launch_ws8<7, TO, 256, 128, 64, 2>(a, in, wp, bias, aux, res, out, s);
      return launch_ws8<3, TO, 256, 128, 64, 2>(a, in, wp, bias, aux, res, out, s);
    case 30:
      if (!wss_ok_out(a, sizeof(TO) == 4)) break;
      return launch_wss<TO>(a, in, wp, bias, aux, res, out, s);
    default: break;
  }
  // heuristic from tools/conv_bench.py on the C3 layer shapes (profiles/r1_conv_bench.md):
  // narrow / non-64-multiple outputs and short row counts favour 128x32 tiles
  // (more workgroups in flight); wide layers 128x64 or 256x64.
  if (wss_pick_short(a) && wss_ok_out(a, sizeof(TO) == 4)) return launch_wss<TO>(a, in, wp, bias, aux, res, out, s);
  if (a.N <= 32 || (a.N % 64) != 0 || a.rows < 8192)
    return launch_fwd4<128, 32, 4, KMAX, TO>(a, in, wp, bias, aux, res, out, s);
  // 256-wide 1x1 (RU256 1x1 fwd 27.5 -> 20.9 us, dgrad 22.5 -> 19.2): 64x128 tiles
  if (a.N >= 256 && a.K == 1) return launch_fwd4<64, 128, 1, KMAX, TO>(a, in, wp, bias, aux, res, out, s);
  // 256-wide layers at 400 samples x 64 clips (25.6k rows): the warp-specialised
  // 256x128 kernel where legal (rocprofv3 kernel trace, profiles/r2_ws_conv.md:
  // RU256 k7 fwd+dgrad 43.5 -> 38.4 us, down2 46.6 -> 41.8), else 256x64 tiles
  // (RU256 k7 fwd 50.7 -> 36.2 us, dgrad 54.2 -> 43.0, down2 51.2 -> 43.1)
  if (a.N >= 256 && a.rows >= 16384) {
    if (wss_pick(a) && wss_ok_out(a, sizeof(TO) == 4)) return launch_wss<TO>(a, in, wp, bias, aux, res, out, s);
    if (tune(38) == 1 && ws8w_ok(a)) return fwd4_variant<KMAX, TO>(29, a, in, wp, bias, aux, res, out, s);
    if (ws_ok(a)) return launch_ws_k<TO>(a, in, wp, bias, aux, res, out, s);
    return launch_fwd4<256, 64, 4, KMAX, TO>(a, in, wp, bias, aux, res, out, s);
  }
  if (a.N <= 64 || a.rows < 65536) return launch_fwd4<128, 64, 2, KMAX, TO>(a, in, wp, bias, aux, res, out, s);
  // 128-wide layers at >= 64 k rows on the warp-specialised kernel (one
  // 128-column tile: no input re-read across column tiles) for the k7 dgrads
  // (RU128 d9: 63.6 -> 53.2 us) and the k3 convs (down1: 49.3 -> 44.1 us), not
  // the k7 forwards with their ELU'd 54-row halo (48.6 -> 52.9 us);
  // tools/conv_bench.py.
  if ((wss_pick_tall(a) || wss_pick_elu(a)) && wss_ok_out(a, sizeof(TO) == 4))
    return launch_wss<TO>(a, in, wp, bias, aux, res, out, s);
  if (ws8_gen_pick(a)) return launch_ws8<7, TO, 512, 128, 64>(a, in, wp, bias, aux, res, out, s);
  if (a.N == 128 && ws_ok(a) && (a.K <= 3 || (a.K == 7 && a.pad == 0 && !a.in_elu)))
    return launch_ws_k<TO>(a, in, wp, bias, aux, res, out, s);
  // 128-wide k7 dgrad at 2000 samples (pad 0, no input ELU): 128x32 tiles (76.5 -> 62.6 us)
  if (a.N == 128 && a.K > 1 && a.pad == 0 && !a.in_elu)
    return launch_fwd4<128, 32, 4, KMAX, TO>(a, in, wp, bias, aux, res, out, s);
  return launch_fwd4<256, 64, 4, KMAX, TO>(a, in, wp, bias, aux, res, out, s);
}

// Weight-stationary thin kernel (tune key 4: 0 = use where legal, 1 = off;
// key 5: target workgroup count, 0 = 1024).  Returns kNotThin when the shape
// has no instance.
constexpr int kNotThin = 1;

template <int C, int N, int K, int R, bool E>
int launch_thin(const Args& a, const void* in, const void* wp, const float* bias, const void* aux,
                const void* res, void* out, hipStream_t s) {
  using G = Thin<C, N, K, R, E>;
  const int64_t ntiles = (a.rows / a.T) * ((a.T + R - 1) / R);
  if (ntiles == 0) return SEL_OK;
  // one round of resident workgroups (each pays the weight-fragment prologue
  // once; a grid just past the resident capacity would add a whole round for
  // its tail); tune key 5 > 0 overrides the workgroup target
  static const int64_t slots = [] {
    int dev = 0, cus = 0, per_cu = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_conv_thin_bf16<C, N, K, R, E>, 256, G::LDS_TOTAL) !=
            hipSuccess)
      return int64_t(0);
    return int64_t(cus) * per_cu / 8 * 8;
  }();
  const int64_t target = tune(5) > 0 ? tune(5) : (slots > 0 ? slots : 1024);
  const int64_t tpb = std::max<int64_t>(1, (ntiles + target - 1) / target);
  const unsigned nb = unsigned(((ntiles + tpb - 1) / tpb + 7) / 8 * 8);  // multiple of 8 (XCD map)
  hipLaunchKernelGGL((k_conv_thin_bf16<C, N, K, R, E>), dim3(nb), dim3(256), G::LDS_TOTAL, s, a,
                     static_cast<const __bf16*>(in), static_cast<const __bf16*>(wp), bias,
                     static_cast<const __bf16*>(aux), static_cast<const __bf16*>(res), static_cast<__bf16*>(out),
                     int(tpb), 3 & ~tune(11));
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

// the (i, C, N, K) instances with their default / alternative tile rows:
// residual-unit k7 / 1x1 at 32 and 64 channels, the first strided conv
// (96 -> 64, 3 taps), the last transposed conv's dgrad (96 -> 64, 2 taps),
// the 128-channel residual-unit 1x1 (one 32-channel output slice per wave;
// k_pw_bf16 by default), and the last transposed conv's forward (64 -> 96,
// 2 taps, replicate pad) and the first strided conv's dgrad (64 -> 96, 3
// taps): three output slices, the fourth wave stages and stores only.
// A/B knobs: tune key 7 bit i = instance i off (tiled kernel instead),
// key 6 bit i = instance i on its alternative tile rows
#define SEL_THIN_SHAPES(X) X(0, 32, 32, 7, 256, 128) X(1, 32, 32, 1, 256, 128) X(2, 64, 64, 7, 128, 64) \
  X(3, 64, 64, 1, 128, 64) X(4, 96, 64, 3, 128, 64) X(5, 96, 64, 2, 128, 64) X(6, 128, 128, 1, 64, 32) \
  X(7, 64, 96, 2, 128, 64) X(8, 64, 96, 3, 128, 64)

int thin_index(const Args& a) {
  // (one sample's rows must fit a 2^31-byte buffer resource: ru_rsrc)
  if (tune(4) == 1 || (a.K - 1) * a.dil > F4_HALOMAX || !ru_region_ok(int64_t(a.T) * a.C * 2)) return -1;
#define SEL_THIN_IDX(I_, C_, N_, K_, R_, R2_) \
  if (a.C == C_ && a.N == N_ && a.K == K_) return (tune(7) >> I_) & 1 ? -1 : I_;
  SEL_THIN_SHAPES(SEL_THIN_IDX)
#undef SEL_THIN_IDX
  return -1;
}

bool thin_ok(const Args& a) { return thin_index(a) >= 0; }

int thin_rows(const Args& a) {
  const int i = thin_index(a);
#define SEL_THIN_R(I_, C_, N_, K_, R_, R2_) if (i == I_) return (tune(6) >> I_) & 1 ? R2_ : R_;
  SEL_THIN_SHAPES(SEL_THIN_R)
#undef SEL_THIN_R
  return 0;
}

// measured per layer (tools/conv_bench.py 30 34 35 36 37, profiles/r1_conv_bench_epf.md):
// the prefetch pays on the k7 dgrads (ELU'(aux) operand) at 32 channels /
// 256 rows (113 -> 88 us) and 64 channels / 64 rows (77 -> 72 us); on the
// 1x1 and strided instances the VGPRs it takes cost more occupancy than it hides
constexpr int kThinEpfDefault = 0b101;  // instances 0 and 2
constexpr int kThinEpfAlt = 0b100;      // instance 2 on its 64-row tiles

// epilogue prefetch + split loop: only for launches with epilogue operands
// (aux and/or res), per instance by kThinEpfDefault (key 12 bit i flips
// instance i, key 11 bit 0 forces it off); kThinEpfAlt instances run it on
// their alternative tile rows.  Returns the E flag, sets the tile rows.
bool thin_variant(const Args& a, bool has_epilogue, int& rows) {
  const int i = thin_index(a);
  const bool epf = has_epilogue && ((kThinEpfDefault ^ tune(12)) >> i & 1) && !(tune(11) & 1);
  const bool alt = (((tune(6) >> i) & 1) != 0) != (epf && ((kThinEpfAlt >> i) & 1));
  rows = 0;
#define SEL_THIN_RV(I_, C_, N_, K_, R_, R2_) if (i == I_) rows = alt ? R2_ : R_;
  SEL_THIN_SHAPES(SEL_THIN_RV)
#undef SEL_THIN_RV
  return epf;
}

int dispatch_thin(const Args& a, const void* in, const void* wp, const float* bias, const void* aux,
                  const void* res, void* out, hipStream_t s) {
  const int i = thin_index(a);
  if (i < 0) return kNotThin;
  int rows_unused;
  const bool epf = thin_variant(a, aux || res, rows_unused);
  const bool alt = (((tune(6) >> i) & 1) != 0) != (epf && ((kThinEpfAlt >> i) & 1));
#define SEL_THIN_LAUNCH(I_, C_, N_, K_, R_, R2_)                                             \
  if (i == I_)                                                                               \
    return epf ? (alt ? launch_thin<C_, N_, K_, R2_, true>(a, in, wp, bias, aux, res, out, s)   \
                      : launch_thin<C_, N_, K_, R_, true>(a, in, wp, bias, aux, res, out, s))   \
               : (alt ? launch_thin<C_, N_, K_, R2_, false>(a, in, wp, bias, aux, res, out, s)  \
                      : launch_thin<C_, N_, K_, R_, false>(a, in, wp, bias, aux, res, out, s));
  SEL_THIN_SHAPES(SEL_THIN_LAUNCH)
#undef SEL_THIN_LAUNCH
  return kNotThin;
}

// Fused residual-unit forward instances: (C, K, R) = (32, 7, 128), (64, 7, 64).
template <int C, int K, int R>
int launch_ru_thin(const Args& a, const void* in, const void* w1p, const float* b1, const void* w2p,
                   const float* b2, void* h, void* out, hipStream_t s) {
  using RU = RuThin<C, K, R>;
  const int64_t ntiles = (a.rows / a.T) * ((a.T + R - 1) / R);
  if (ntiles == 0) return SEL_OK;
  const int64_t target = 1024;
  const int64_t tpb = std::max<int64_t>(1, (ntiles + target - 1) / target);
  const unsigned nb = unsigned(((ntiles + tpb - 1) / tpb + 7) / 8 * 8);  // multiple of 8 (XCD map)
  hipLaunchKernelGGL((k_ru_thin_bf16<C, K, R>), dim3(nb), dim3(256), RU::LDS, s, a,
                     static_cast<const __bf16*>(in), static_cast<const __bf16*>(w1p), b1,
                     static_cast<const __bf16*>(w2p), b2, static_cast<__bf16*>(h), static_cast<__bf16*>(out),
                     int(tpb));
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

// fused 32-channel residual unit: one round of resident workgroups, each
// walking an XCD-contiguous range of sample-aligned tiles
template <int R, bool BWD>
int64_t ru32_tiles_per_block(int64_t ntiles) {
  static const int64_t slots = [] {
    int dev = 0, cus = 0, per_cu = 0;
    const size_t lds = BWD ? Ru32<R>::LDS_BWD : Ru32<R>::LDS_FWD;
    const void* kern = BWD ? (const void*)k_ru32_bwd<R> : (const void*)k_ru32_fwd<R>;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 256, lds) != hipSuccess)
      return int64_t(0);
    return int64_t(cus) * per_cu / 8 * 8;
  }();
  const int64_t target = slots > 0 ? slots : 1024;
  return std::max<int64_t>(1, (ntiles + target - 1) / target);
}

template <int R>
int launch_ru32_fwd(const Args& a, const void* x, const void* w1p, const float* b1, const void* w2p,
                    const float* b2, void* h, void* out, hipStream_t s) {
  const int64_t ntiles = (a.rows / a.T) * ((a.T + R - 1) / R);
  if (ntiles == 0) return SEL_OK;
  const int64_t tpb = ru32_tiles_per_block<R, false>(ntiles);
  const unsigned nb = unsigned(((ntiles + tpb - 1) / tpb + 7) / 8 * 8);
  hipLaunchKernelGGL(k_ru32_fwd<R>, dim3(nb), dim3(256), Ru32<R>::LDS_FWD, s, a, static_cast<const __bf16*>(x),
                     static_cast<const __bf16*>(w1p), b1, static_cast<const __bf16*>(w2p), b2,
                     static_cast<__bf16*>(h), static_cast<__bf16*>(out), int(tpb), tune(15));
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

int launch_ru32_fwd4(const Args& a, const void* x, const void* w1p, const float* b1, const void* w2p,
                     const float* b2, void* h, void* out, hipStream_t s) {
  constexpr int R = 256;
  const int64_t ntiles = (a.rows / a.T) * ((a.T + R - 1) / R);
  if (ntiles == 0) return SEL_OK;
  static const int64_t slots = [] {
    int dev = 0, cus = 0, per_cu = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_ru32_fwd4<R>, 256, Ru32F4<R>::LDS) != hipSuccess)
      return int64_t(0);
    return int64_t(cus) * per_cu / 8 * 8;
  }();
  const int64_t target = slots > 0 ? slots : 1024;
  const int64_t tpb = std::max<int64_t>(1, (ntiles + target - 1) / target);
  const unsigned nb = unsigned(((ntiles + tpb - 1) / tpb + 7) / 8 * 8);
  hipLaunchKernelGGL(k_ru32_fwd4<R>, dim3(nb), dim3(256), Ru32F4<R>::LDS, s, a, static_cast<const __bf16*>(x),
                     static_cast<const __bf16*>(w1p), b1, static_cast<const __bf16*>(w2p), b2,
                     static_cast<__bf16*>(h), static_cast<__bf16*>(out), int(tpb));
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

template <int R>
int launch_ru64_fwd(const Args& a, const void* x, const void* w1p, const float* b1, const void* w2p,
                    const float* b2, void* h, void* out, hipStream_t s) {
  const int64_t ntiles = (a.rows / a.T) * ((a.T + R - 1) / R);
  if (ntiles == 0) return SEL_OK;
  static const int64_t slots = [] {
    int dev = 0, cus = 0, per_cu = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_ru64_fwd<R>, 256, Ru64<R>::LDS) != hipSuccess)
      return int64_t(0);
    return int64_t(cus) * per_cu / 8 * 8;
  }();
  const int64_t target = tune(24) > 0 ? tune(24) : (slots > 0 ? slots : 1024);
  const int64_t tpb = std::max<int64_t>(1, (ntiles + target - 1) / target);
  const unsigned nb = unsigned(((ntiles + tpb - 1) / tpb + 7) / 8 * 8);
  hipLaunchKernelGGL(k_ru64_fwd<R>, dim3(nb), dim3(256), Ru64<R>::LDS, s, a, static_cast<const __bf16*>(x),
                     static_cast<const __bf16*>(w1p), b1, static_cast<const __bf16*>(w2p), b2,
                     static_cast<__bf16*>(h), static_cast<__bf16*>(out), int(tpb));
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

template <int R>
int launch_ru64_bwd(const Args& a, const void* g, const void* h, const void* x, const void* wd1, const void* wd2,
                    void* gh, void* gx, hipStream_t s) {
  const int64_t ntiles = (a.rows / a.T) * ((a.T + R - 1) / R);
  if (ntiles == 0) return SEL_OK;
  static const int64_t slots = [] {
    int dev = 0, cus = 0, per_cu = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_ru64_bwd<R>, 256, Ru64B<R>::LDS) != hipSuccess)
      return int64_t(0);
    return int64_t(cus) * per_cu / 8 * 8;
  }();
  const int64_t target = slots > 0 ? slots : 1024;
  const int64_t tpb = std::max<int64_t>(1, (ntiles + target - 1) / target);
  const unsigned nb = unsigned(((ntiles + tpb - 1) / tpb + 7) / 8 * 8);
  hipLaunchKernelGGL(k_ru64_bwd<R>, dim3(nb), dim3(256), Ru64B<R>::LDS, s, a, static_cast<const __bf16*>(g),
                     static_cast<const __bf16*>(h), static_cast<const __bf16*>(x), static_cast<const __bf16*>(wd1),
                     static_cast<const __bf16*>(wd2), static_cast<__bf16*>(gh), static_cast<__bf16*>(gx), int(tpb));
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

template <int R>
int launch_ru32_bwd(const Args& a, const void* g, const void* h, const void* x, const void* wd1, const void* wd2,
                    void* gh, void* gx, hipStream_t s) {
  const int64_t ntiles = (a.rows / a.T) * ((a.T + R - 1) / R);
  if (ntiles == 0) return SEL_OK;
  const int64_t tpb = ru32_tiles_per_block<R, true>(ntiles);
  const unsigned nb = unsigned(((ntiles + tpb - 1) / tpb + 7) / 8 * 8);
  hipLaunchKernelGGL(k_ru32_bwd<R>, dim3(nb), dim3(256), Ru32<R>::LDS_BWD, s, a, static_cast<const __bf16*>(g),
                     static_cast<const __bf16*>(h), static_cast<const __bf16*>(x), static_cast<const __bf16*>(wd1),
                     static_cast<const __bf16*>(wd2), static_cast<__bf16*>(gh), static_cast<__bf16*>(gx), int(tpb));
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

// fused 32-channel backward with the weight gradients: one block per partial
template <int R>
int ru32w_blocks(int64_t ntiles, int64_t& tpb) {
  static const int64_t slots = [] {
    int dev = 0, cus = 0, per_cu = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_ru32_bwdw<R>, 256, Ru32W<R>::LDS) != hipSuccess)
      return int64_t(0);
    return int64_t(cus) * per_cu / 8 * 8;
  }();
  const int64_t target = tune(35) > 0 ? tune(35) : (slots > 0 ? slots : 512);
  tpb = std::max<int64_t>(1, (ntiles + target - 1) / target);
  return int(((ntiles + tpb - 1) / tpb + 7) / 8 * 8);
}

template <int R>
int launch_ru32_bwdw(const Args& a, const void* g, const void* h, const void* x, const void* wd1, const void* wd2,
                     void* gx, float* part1, float* part2, int nsplit, hipStream_t s) {
  const int64_t ntiles = (a.rows / a.T) * ((a.T + R - 1) / R);
  int64_t tpb = 1;
  const int nb = ru32w_blocks<R>(ntiles, tpb);
  SEL_REQUIRE(nb == nsplit, SEL_ERR_ARG, "sel_resunit_bwd_wgrad: nsplit %d, this shape needs %d", nsplit, nb);
  hipLaunchKernelGGL(k_ru32_bwdw<R>, dim3(unsigned(nb)), dim3(256), Ru32W<R>::LDS, s, a, static_cast<const __bf16*>(g),
                     static_cast<const __bf16*>(h), static_cast<const __bf16*>(x), static_cast<const __bf16*>(wd1),
                     static_cast<const __bf16*>(wd2), static_cast<__bf16*>(gx), part1, part2, int(tpb));
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

// fused 64-channel backward with the weight gradients: one 512-thread block per
// CU (its LDS planes), one partial per block
template <int R, bool WG = true>
int ru64w_blocks(int64_t ntiles, int64_t& tpb) {
  static const int64_t slots = [] {
    int dev = 0, cus = 0, per_cu = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipFuncSetAttribute((const void*)k_ru64_bwdw<R, WG>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            int(Ru64W<R>::LDS)) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_ru64_bwdw<R, WG>, 512, Ru64W<R>::LDS) != hipSuccess)
      return int64_t(0);
    return int64_t(cus) * per_cu / 8 * 8;
  }();
  const int64_t target = tune(40) > 0 ? tune(40) : (slots > 0 ? slots : 256);
  tpb = std::max<int64_t>(1, (ntiles + target - 1) / target);
  return int(((ntiles + tpb - 1) / tpb + 7) / 8 * 8);
}

template <int R, bool WG = true>
int launch_ru64_bwdw(const Args& a, const void* g, const void* h, const void* x, const void* wd1, const void* wd2,
                     void* gx, float* part1, float* part2, int nsplit, hipStream_t s) {
  const int64_t ntiles = (a.rows / a.T) * ((a.T + R - 1) / R);
  if (ntiles == 0 && !WG) return SEL_OK;
  int64_t tpb = 1;
  const int nb = ru64w_blocks<R, WG>(ntiles, tpb);
  SEL_REQUIRE(!WG || nb == nsplit, SEL_ERR_ARG, "sel_resunit_bwd_wgrad: nsplit %d, this shape needs %d", nsplit, nb);
  SEL_HIP(hipFuncSetAttribute((const void*)k_ru64_bwdw<R, WG>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              int(Ru64W<R>::LDS)));
  hipLaunchKernelGGL((k_ru64_bwdw<R, WG>), dim3(unsigned(nb)), dim3(512), Ru64W<R>::LDS, s, a,
                     static_cast<const __bf16*>(g), static_cast<const __bf16*>(h), static_cast<const __bf16*>(x),
                     static_cast<const __bf16*>(wd1), static_cast<const __bf16*>(wd2), static_cast<__bf16*>(gx), part1,
                     part2, int(tpb));
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}


// Pointwise kernel (k_pw_bf16) where it applies: 1x1, C = N in {128, 256}
// (the RU128 / RU256 1x1 forwards and dgrads; rocprof on the C3 shapes:
// 21.0 -> 19.6 us at 128 (thin kernel before), 19.1 -> 14.3 us at 256);
// tune key 42: 1 = off; key 43 > 0: workgroup count
bool pw_ok(const Args& a) {
  // (a forced tiled variant, tune key 0, takes precedence)
  if (a.K != 1 || a.C != a.N || a.pad != 0 || tune(42) == 1 || tune(0) != 0) return false;
  if (!(a.N == 256 || a.N == 128)) return false;
  // every block's row range is one buffer resource
  return ru_region_ok(a.rows * int64_t(a.N) * 2);
}

template <int C, int N, bool ELU, bool AUX, bool RES>
int launch_pw_t(const Args& a, const void* in, const void* wp, const float* bias, const void* aux, const void* res,
                void* out, hipStream_t s) {
  using G = Pw<C, N>;
  if (a.rows == 0) return SEL_OK;
  // one round of resident workgroups, each over an equal contiguous row range
  static const int64_t slots = [] {
    int dev = 0, cus = 0, per_cu = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_pw_bf16<C, N, ELU, AUX, RES>, G::THREADS, G::LDS) !=
            hipSuccess)
      return int64_t(256);
    return std::max<int64_t>(1, int64_t(cus) * std::max(per_cu, 1));
  }();
  const int64_t target = tune(43) > 0 ? tune(43) : slots;
  int64_t nb = std::min<int64_t>(target, (a.rows + G::R - 1) / G::R);
  // (a pass covers RB rows: a range of more rows takes several passes)
  const int64_t rpb = (a.rows + nb - 1) / nb;
  nb = (a.rows + rpb - 1) / rpb;
  hipLaunchKernelGGL((k_pw_bf16<C, N, ELU, AUX, RES>), dim3(unsigned(nb)), dim3(G::THREADS), G::LDS, s, a,
                     static_cast<const __bf16*>(in), static_cast<const __bf16*>(wp), bias,
                     static_cast<const __bf16*>(aux), static_cast<const __bf16*>(res), static_cast<__bf16*>(out),
                     int(rpb));
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

template <int C, int N, bool ELU>
int launch_pw_e(const Args& a, const void* in, const void* wp, const float* bias, const void* aux, const void* res,
                void* out, hipStream_t s) {
  if (aux && res) return launch_pw_t<C, N, ELU, true, true>(a, in, wp, bias, aux, res, out, s);
  if (aux) return launch_pw_t<C, N, ELU, true, false>(a, in, wp, bias, aux, res, out, s);
  if (res) return launch_pw_t<C, N, ELU, false, true>(a, in, wp, bias, aux, res, out, s);
  return launch_pw_t<C, N, ELU, false, false>(a, in, wp, bias, aux, res, out, s);
}

template <int C, int N>
int launch_pw(const Args& a, const void* in, const void* wp, const float* bias, const void* aux, const void* res,
              void* out, hipStream_t s) {
  return a.in_elu ? launch_pw_e<C, N, true>(a, in, wp, bias, aux, res, out, s)
                  : launch_pw_e<C, N, false>(a, in, wp, bias, aux, res, out, s);
}

bool ru_fused_ok(const Args& a) {
  return (a.C == 32 || a.C == 64) && a.N == a.C && a.K == 7 && a.pad == (a.K - 1) * a.dil &&
         a.pad_mode == SEL_PAD_ZERO && a.in_elu == 1 && (a.K - 1) * a.dil <= F4_HALOMAX &&
         (a.bias_period == 0 || a.bias_period == a.N) && ru_region_ok(int64_t(a.T) * a.C * 2);
}

// single-input-channel forward (k_conv_c1_bf16): one resident round of
// workgroups walking TR-row tiles (they prefetch their next tile); tune key
// 44 = 1: the round-3 256-row tiles
template <typename TI, typename TO, int TR>
int launch_c1(const Args& a, const void* in, const void* wp, const float* bias, const void* aux, const void* res,
              void* out, hipStream_t s) {
  static const int64_t slots = [] {
    int dev = 0, cus = 0, per_cu = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_conv_c1<TI, TO, TR>, 256, 0) != hipSuccess)
      return int64_t(4096);
    return std::max<int64_t>(256, int64_t(cus) * per_cu);
  }();
  const int64_t blocks = std::min<int64_t>((a.rows / a.T) * ((a.T + TR - 1) / TR), tune(23) > 0 ? tune(23) : slots);
  if (blocks <= 0) return SEL_OK;
  hipLaunchKernelGGL((k_conv_c1<TI, TO, TR>), dim3(unsigned(blocks)), dim3(256), 0, s, a,
                     static_cast<const TI*>(in), static_cast<const TI*>(wp), bias,
                     static_cast<const TO*>(aux), static_cast<const TO*>(res), static_cast<TO*>(out));
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

template <typename TI, typename TO>
int dispatch_fwd(const Args& a, const void* in, const void* wp, const float* bias, const void* aux,
                 const void* res, void* out, hipStream_t s) {
  if constexpr (sizeof(TI) == 2 && sizeof(TO) == 2) {
    if (pw_ok(a))
      return a.N == 256 ? launch_pw<256, 256>(a, in, wp, bias, aux, res, out, s)
                        : launch_pw<128, 128>(a, in, wp, bias, aux, res, out, s);
    const int rc = dispatch_thin(a, in, wp, bias, aux, res, out, s);
    if (rc != kNotThin) return rc;
  }
  if constexpr (sizeof(TI) == 2) {
    if (a.C == 1 && a.N % 8 == 0 && a.N <= C1_NMAX && a.K <= C1_KMAX && (a.K - 1) * a.dil <= C1_HALO &&
        tune(3) == 0)
      return tune(44) == 1   ? launch_c1<TI, TO, 256>(a, in, wp, bias, aux, res, out, s)
             : tune(44) == 2 ? launch_c1<TI, TO, 1024>(a, in, wp, bias, aux, res, out, s)
                             : launch_c1<TI, TO, C1F_TR>(a, in, wp, bias, aux, res, out, s);
    const int v = tune(0);
    const bool fast = (a.C % CK) == 0 && (a.K - 1) * a.dil <= F4_HALOMAX && a.K <= 8 && (v == 0 || v > 20);
    if (fast) {
      if (a.K == 1) return fwd4_variant<1, TO>(v, a, in, wp, bias, aux, res, out, s);
      if (a.K <= 3) return fwd4_variant<3, TO>(v, a, in, wp, bias, aux, res, out, s);
      return fwd4_variant<8, TO>(v, a, in, wp, bias, aux, res, out, s);
    }
    switch (v) {
      case 1: return launch_fwd<TI, TO, 128, 32>(a, in, wp, bias, aux, res, out, s);
      case 2: return launch_fwd<TI, TO, 128, 64>(a, in, wp, bias, aux, res, out, s);
      case 3: return launch_fwd<TI, TO, 128, 128>(a, in, wp, bias, aux, res, out, s);
      case 4: return launch_fwd<TI, TO, 64, 64>(a, in, wp, bias, aux, res, out, s);
      case 5: return launch_fwd<TI, TO, 256, 32>(a, in, wp, bias, aux, res, out, s);
      case 6: return launch_fwd<TI, TO, 256, 64>(a, in, wp, bias, aux, res, out, s);
      default: break;
    }
  }
  if (sizeof(TI) == 4) {
    if constexpr (sizeof(TO) == 4) {
      // single input channel: the streaming kernel with exact fp32 ELU (tune key 55 = 1: generic)
      if (a.C == 1 && a.N % 4 == 0 && a.N <= C1_NMAX && a.K <= C1_KMAX && (a.K - 1) * a.dil <= C1_HALO &&
          tune(55) != 1)
        return launch_c1<TI, TO, C1F_TR>(a, in, wp, bias, aux, res, out, s);
      // sample-aligned fp32 tiles (tune key 55 = 1: the generic kernel)
      if (a.C % FF_CK == 0 && a.N % 32 == 0 && a.K <= 8 && (a.K - 1) * a.dil <= FF_HALO && tune(55) != 1) {
        if (a.N % 64 == 0) return launch_fwd_f32<64, 64>(a, in, wp, bias, aux, res, out, s);
        return launch_fwd_f32<128, 32>(a, in, wp, bias, aux, res, out, s);
      }
    }
    if (a.N <= 32) return launch_fwd<TI, TO, 128, 32>(a, in, wp, bias, aux, res, out, s);
    return launch_fwd<TI, TO, 64, 64>(a, in, wp, bias, aux, res, out, s);
  }
  if (a.N <= 32) return launch_fwd<TI, TO, 128, 32>(a, in, wp, bias, aux, res, out, s);
  if (a.N <= 64 || a.K >= 5) return launch_fwd<TI, TO, 128, 64>(a, in, wp, bias, aux, res, out, s);
  if (a.rows >= 4096) return launch_fwd<TI, TO, 128, 128>(a, in, wp, bias, aux, res, out, s);
  return launch_fwd<TI, TO, 64, 64>(a, in, wp, bias, aux, res, out, s);
}

constexpr int kWgBN = 64;

int wgrad_bn(int N) { return N <= 16 ? 16 : (N <= 32 ? 32 : 64); }

// Split plan shared by both dtypes: 64-row m-tiles that never cross a sample,
// enough splits for ~2 workgroups per CU, partial buffer capped at 64 MB.
struct WgPlan {
  int64_t tiles_per_sample, n_tiles;
  int nsplit, tiles_per_split, bn;
  int mode;  // 0 generic (k_wgrad_bf16 / fp32), 2 k_wgrad2_bf16 (32x32), 3 k_wgrad3_bf16
  int nt, ct, maxt;
};

bool wgrad_tr_ok(const sel_conv_desc* d) {
  // (one sample's gout / input rows must fit a 2^31-byte buffer resource: ru_rsrc)
  return d->C % 32 == 0 && d->N % 32 == 0 && (d->K - 1) * d->dil <= W2_HALO && d->K <= 8 &&
         ru_region_ok(int64_t(d->T) * std::max(d->C, d->N) * 2);
}

// tune key 1: 0 = k_wgrad3 where legal, 1 = generic, 2 = k_wgrad2 (32x32 blocks)
bool wgrad_c1_ok(const sel_conv_desc* d) {
  return d->C == 1 && d->N % 8 == 0 && d->N <= C1_NMAX && d->K <= C1_KMAX && (d->K - 1) * d->dil <= C1_HALO;
}

int wgrad_mode(const sel_conv_desc* d, int dtype) {
  // fp32: the single-channel kernel where it applies (tune key 54 = 1: generic)
  if (dtype != SEL_BF16) return wgrad_c1_ok(d) && tune(54) != 1 ? 4 : 0;
  const int t = tune(1);
  if (wgrad_c1_ok(d) && t != 1) return 4;
  if (t == 1 || !wgrad_tr_ok(d)) return 0;
  return t == 2 ? 2 : 3;
}

WgPlan wgrad_plan(const sel_conv_desc* d, int mode) {
  WgPlan p;
  p.mode = mode;
  p.nt = p.ct = p.maxt = 1;
  if (mode == 4) {  // k_wgrad_c1_bf16: contiguous ranges of sample-aligned 256-row tiles
    p.bn = d->N;
    p.tiles_per_sample = (d->T + C1_TR - 1) / C1_TR;
    p.n_tiles = (d->rows / d->T) * p.tiles_per_sample;
    p.tiles_per_split = int(std::max<int64_t>(1, (p.n_tiles + 511) / 512));
    p.nsplit = int((p.n_tiles + p.tiles_per_split - 1) / p.tiles_per_split);
    return p;
  }
  const bool tr = mode >= 2;
  const int bm = tr ? W2_BM : WB_BM;
  int bn, bc;
  if (mode == 3) {
    // widest block whose per-wave tile count stays <= 4 (8 accumulators = 1 wave/SIMD,
    // measured slower than re-reading a 32-wide operand from L2)
    auto tiles_per_wave = [&](int nt, int ct) {
      const int wpn = 4 / nt, pairs = ct * d->K;
      const int wpp = pairs >= wpn ? wpn : pairs;  // waves sharing one pair list (kernel: WPN / RG)
      return (pairs + wpp - 1) / wpp;
    };
    p.nt = d->N % 64 == 0 ? 2 : 1;
    p.ct = d->C % 64 == 0 ? 2 : 1;
    if (tiles_per_wave(p.nt, p.ct) > 4 && p.ct == 2) p.ct = 1;
    if (tiles_per_wave(p.nt, p.ct) > 4 && p.nt == 2) p.nt = 1;
    const int tpw = tiles_per_wave(p.nt, p.ct);
    // exact per-wave tile count (the strided k3 layers at 64 input channels per
    // block: 3 pairs per wave, which the 4-slot form ran with a never-stored slot)
    p.maxt = tpw <= 4 ? tpw : 8;
    bn = 32 * p.nt;
    bc = 32 * p.ct;
  } else {
    bn = tr ? 32 : wgrad_bn(d->N);
    bc = tr ? 32 : WB_BC;
  }
  p.bn = bn;
  p.tiles_per_sample = (d->T + bm - 1) / bm;
  p.n_tiles = (d->rows / d->T) * p.tiles_per_sample;
  const int64_t blocks = int64_t((d->N + bn - 1) / bn) * ((d->C + bc - 1) / bc);
  // tune key 10 > 0: workgroup-count target override (A/B sweeps)
  const int64_t target = tune(10) > 0 ? tune(10) : (mode == 3 ? 512 : 768);
  int64_t want = std::max<int64_t>(1, (target + blocks - 1) / blocks);
  if (mode == 3) want = (want + 7) / 8 * 8;  // splits on x: blocks of one row range share an XCD
  const int64_t per_split = (int64_t(d->N) * d->K * d->C + d->N) * 4;
  // split partials per layer capped at 32 MB (mode 3; tune key 62 > 0: another cap in MB)
  const int64_t cap_mb = mode == 3 ? (tune(62) > 0 ? tune(62) : 32) : 64;
  want = std::min<int64_t>(want, std::max<int64_t>(1, (cap_mb << 20) / per_split));
  want = std::min<int64_t>(want, std::max<int64_t>(1, p.n_tiles));
  p.tiles_per_split = int((p.n_tiles + want - 1) / want);
  if (p.tiles_per_split < 1) p.tiles_per_split = 1;
  p.nsplit = int((p.n_tiles + p.tiles_per_split - 1) / p.tiles_per_split);
  if (p.nsplit < 1) p.nsplit = 1;
  return p;
}

template <int NT, int CT>
hipError_t launch_wgrad3(const WgPlan& p, const Args& a, const __bf16* gout, const __bf16* in, float* part,
                         float* bpart, hipStream_t s) {
  constexpr size_t lds_max = size_t(2) * (NT * W2_BM * 32 + CT * (W2_BM + W2_HALO) * 32) * sizeof(__bf16);
  const size_t lds = size_t(2) * (NT * W2_BM * 32 + CT * wgrad3_xrows(a.K, a.dil) * 32) * sizeof(__bf16);
  dim3 grid(unsigned(p.nsplit), unsigned(a.N / (32 * NT)), unsigned(a.C / (32 * CT)));
  // the two-set fragment pipeline (tune key 57 = 1) for the k2 / k3 layers
  // with >= 64 k rows: faster in tools/ab_wgrad.sh (256 -> 128 down conv
  // 69 -> 58 us, inputs re-read from the cache), not inside the profiled C3
  // step (<2, 1, 2> 55.8 -> 59 us, <2, 2, 3> 53.5 -> 52.3 us), so off
  const bool pipe = p.maxt <= 3 && a.rows >= 65536 && tune(57) == 1;
#define SEL_WG3(MT)                                                                                            \
  {                                                                                                            \
    auto kern = pipe ? k_wgrad3_bf16<NT, CT, MT, (MT <= 3)> : k_wgrad3_bf16<NT, CT, MT, false>;                \
    if (lds_max > 64 * 1024) {                                                                                 \
      hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, int(lds_max)); \
      if (e != hipSuccess) return e;                                                                           \
    }                                                                                                          \
    hipLaunchKernelGGL(kern, grid, dim3(256), lds, s, a, gout, in, int(p.tiles_per_sample), p.n_tiles,          \
                       p.tiles_per_split, part, bpart);                                                        \
  }
  if (p.maxt == 1) SEL_WG3(1)
  else if (p.maxt == 2) SEL_WG3(2)
  else if (p.maxt == 3) SEL_WG3(3)
  else if (p.maxt == 4) SEL_WG3(4)
  else SEL_WG3(8)
#undef SEL_WG3
  return hipGetLastError();
}

}  // namespace

// Discriminator layers (dconv.hip, sel_dconv_desc) on the warp-specialised
// 256 x 128 kernel: one group, a contiguous reduction row (S == 1 or Cs == Cg:
// the phase view of a strided layer is S * Cg contiguous channels), contiguous
// output columns, K in {2, 3, 5, 7}.  The MPD's (5,1) convs are K = 5 (stride 1)
// or K = 2 taps over 3 * Cin channels (stride 3, phase view); their adjoints the
// same K over gout with So = 3 output phases.  Returns SEL_ERR_UNSUPPORTED for
// any other shape (the caller keeps its own kernels).
namespace sel {
namespace conv {
int dconv_ws_mode(const sel_dconv_desc* d) {
  const int width = d->So * d->Ng, nred = d->S * d->Cg;
  const bool ok = d->G == 1 && (d->S == 1 || d->Cs == d->Cg) && (d->So == 1 || d->Ns == d->Ng) &&
                  (d->K == 2 || d->K == 3 || d->K == 5 || d->K == 7) && width % WS_BN == 0 &&
                  nred % WS_CK == 0 && nred <= WS_CMAX && d->ldx % 8 == 0 && d->ldo % 8 == 0 &&
                  d->ldx >= nred && d->ldo >= width && d->Tvo > 0 && d->B > 0 && d->Tv <= d->Tvs &&
                  d->K - 1 <= F4_HALOMAX && -d->q0 <= F4_HALOMAX && ws_lds_bytes(d->K) <= 160 * 1024;
  if (!ok) return -1;
  // flat tiling (tune key 22: 1 = off) where the layout leaves zero gaps
  // between sequences (sel.dconvops allocates the MPD chain so; its deep layers
  // have 54-300 rows per period column, a 256-row sample-aligned tile wastes up
  // to 80% there): every row a tap may read across a sequence boundary lies in a gap
  // (input row >= Tv) or feeds an output row that is written as zero (>= Tvalid)
  const int P = d->Tvo;
  const bool flat = tune(22) != 1 && d->Tvs == P && P - d->Tv >= -d->q0 && P - d->Tvalid >= d->q0 + d->K - 1 &&
                    int64_t(d->B) * P < (int64_t(1) << 31);
  return flat ? 1 : 0;
}

// the eight-wave kernel's 256 x 256 tiles for the MPD's 128 -> 512 stride-3
// layer (K = 2 taps over 384 phase channels: 141 -> 126 us at period 2, D
// step, tools/ws8_probe.py); the deeper K = 2 / 5 layers stay on the 12-wave
// kernel (512 -> 1024 s3: 218 vs 248 us, 1024 -> 1024 k5: 279 vs 339 us: with
// 64-96 chunks per tile the DMA issue the eight waves take on costs more than
// the fragment reads they save); tune key 37 = 1: off
bool dconv_ws8_ok(const sel_dconv_desc* d) {
  return tune(37) != 1 && d->K == 2 && d->S * d->Cg <= 512 && (d->So * d->Ng) % 256 == 0 && dconv_ws_mode(d) >= 0;
}

int dconv_ws_fwd(const sel_dconv_desc* d, const void* x, const void* wp, const float* bias, const void* aux,
                 const void* res, void* out, hipStream_t s) {
  const int mode = dconv_ws_mode(d);
  if (mode < 0) return SEL_ERR_UNSUPPORTED;
  const bool flat = mode == 1;
  const int width = d->So * d->Ng, nred = d->S * d->Cg;
  const int P = d->Tvo;
  Args a;
  a.rows = int64_t(d->B) * d->Tvo;
  a.T = flat ? int(a.rows) : d->Tvo;
  a.seq_pitch = flat ? P : 0;
  a.C = nred;
  a.N = width;
  a.K = d->K;
  a.dil = 1;
  a.pad = -d->q0;
  a.pad_mode = SEL_PAD_ZERO;
  a.in_elu = 0;
  a.bias_period = 0;
  a.tin_valid = d->Tv;
  a.tin_pitch = d->Tvs;
  a.ldx = d->ldx;
  a.ldo = d->ldo;
  a.tout_valid = d->Tvalid;
  a.epi = 1;
  a.act = d->act;
  a.slope = d->slope;
  if (dconv_ws8_ok(d)) {
    if (d->K == 2) return launch_ws8<2, __bf16, 256, 256, 32>(a, x, wp, bias, aux, res, out, s);
    return launch_ws8<5, __bf16, 256, 256, 32>(a, x, wp, bias, aux, res, out, s);
  }
  switch (d->K) {
    case 2: return launch_ws<2, __bf16>(a, x, wp, bias, aux, res, out, s);
    case 3: return launch_ws<3, __bf16>(a, x, wp, bias, aux, res, out, s);
    case 5: return launch_ws<5, __bf16>(a, x, wp, bias, aux, res, out, s);
    default: return launch_ws<7, __bf16>(a, x, wp, bias, aux, res, out, s);
  }
}
}  // namespace conv
}  // namespace sel

extern "C" {

int sel_conv_fwd_kernel_id(const sel_conv_desc* d, int in_dtype, int out_dtype, int has_epilogue) {
  if (!d || in_dtype != SEL_BF16 || check_desc(d) != SEL_OK) return -1;
  const Args a = to_args(d);
  if (out_dtype == SEL_BF16 && pw_ok(a)) return 930000000 + a.N;  // pointwise: 9.3e8 + N
  if (out_dtype == SEL_BF16 && thin_ok(a)) {  // thin: 1e9 + E*5e8 + ((R/32*1000 + C)*1000 + N)*10 + K
    int r = 0;
    const bool e = thin_variant(a, has_epilogue != 0, r);
    return 1000000000 + (e ? 500000000 : 0) + ((r / 32 * 1000 + a.C) * 1000 + a.N) * 10 + a.K;
  }
  const int v = fwd4_choice(a, out_dtype == SEL_F32);
  if (v < 0) return -1;
  // warp-specialised kernels: 9e8 + K (12 waves), 9.1e8 + K (eight waves, 512 x 128)
  if (v == 27) return 900000000 + a.K;
  if (v == 28) return 910000000 + a.K;
  if (v == 29) return 920000000 + a.K;
  if (v == 30) {  // sample-tile kernel: 9.4e8 + 1e6 (SPT - 1) + 1e4 BN + 10 S + K
    int S = 0, tm = 0, BN = 0;
    wss_geometry(a, S, tm, BN);
    return 940000000 + 1000000 * (wss_spt(a) - 1) + 10000 * BN + 10 * S + a.K;
  }
  const int kmax = a.K == 1 ? 1 : (a.K <= 3 ? 3 : 8);
  static const int bm[] = {256, 128, 128, 256, 128, 64}, bn[] = {32, 32, 64, 64, 128, 128}, wm[] = {4, 4, 2, 4, 2, 1};
  const int i = v - 21;
  return ((bm[i] * 1000 + bn[i]) * 10 + wm[i]) * 10 + kmax;  // BM,BN,WAVES_M,KMAX packed
}

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

/* Fused residual unit forward (residual_unit.py:43-46): h = conv1(ELU(x)) and
 * out = x + conv1x1(ELU(h)) in one pass (bf16, C = N in {32, 64}, or 128 where
 * the (16, 128) k_conv_wss tile applies, K = 7, causal
 * zero pad, ELU prologue; d1 describes conv1, its bias_period 0 or N).  Returns
 * SEL_ERR_UNSUPPORTED for other shapes (callers then use two sel_conv_fwd calls). */
int sel_resunit_fwd(const sel_conv_desc* d1, int dtype, const void* x, const void* w1pack, const float* b1,
                    const void* w2pack, const float* b2, void* h, void* out, sel_stream_t stream) {
  if (int rc = check_desc(d1)) return rc;
  const Args a = to_args(d1);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  // 128 channels (round 6): the (16, 128) k_conv_wss tile with the 1x1 in its
  // epilogue, where conv1 alone runs on that tile (T = 2000, >= 65536 rows:
  // the C3 RU128 units); tune key 69 = 1: off
  if (dtype == SEL_BF16 && a.C == 128 && fwd4_choice(a, false) == 30 && wss_pw_ok(a))
    return launch_wss_pw(a, x, w1pack, b1, w2pack, b2, h, out, s);
  SEL_REQUIRE(dtype == SEL_BF16 && ru_fused_ok(a), SEL_ERR_UNSUPPORTED,
              "sel_resunit_fwd: fused path needs bf16, C = N in {32, 64} (128 on the (16, 128) k_conv_wss tile), "
              "K = 7, causal zero pad, ELU prologue");
  // tune key 56 = 1: 128-row tiles (4 resident workgroups per CU instead of 3):
  // 66-67 -> 58.6-59 us per unit in tools/ru_bench.py, which re-reads the same
  // input, but 69.5 -> 72.6 us inside the profiled C3 step, so off
  // tune key 70 = 1: k_ru32_fwd4 (W1 in LDS, four blocks per CU; bit-identical)
  if (a.C == 32 && tune(70) == 1 && tune(56) != 1) return launch_ru32_fwd4(a, x, w1pack, b1, w2pack, b2, h, out, s);
  if (a.C == 32)
    return tune(56) == 1 ? launch_ru32_fwd<128>(a, x, w1pack, b1, w2pack, b2, h, out, s)
                         : launch_ru32_fwd<256>(a, x, w1pack, b1, w2pack, b2, h, out, s);
  // tune key 24 < 0: the LDS-staged k_ru_thin_bf16 (round 2) instead of k_ru64_fwd
  if (tune(24) < 0) return launch_ru_thin<64, 7, 64>(a, x, w1pack, b1, w2pack, b2, h, out, s);
  return launch_ru64_fwd<128>(a, x, w1pack, b1, w2pack, b2, h, out, s);
}

/* Fused residual unit backward at 32 channels (residual_unit.py:43-46 adjoint):
 * gh = (W2^T g) * ELU'(h), gx = conv1^T(gh) * ELU'(x) + g in one launch.  d1 is
 * the forward conv1 descriptor; wd1 / wd2 the dgrad-packed weights; gh may be
 * null (only the weight gradient of conv1 needs it). */
int sel_resunit_bwd(const sel_conv_desc* d1, int dtype, const void* g, const void* h, const void* x,
                    const void* wd1pack, const void* wd2pack, void* gh, void* gx, sel_stream_t stream) {
  if (int rc = check_desc(d1)) return rc;
  const Args a = to_args(d1);
  SEL_REQUIRE(dtype == SEL_BF16 && ru_fused_ok(a), SEL_ERR_UNSUPPORTED,
              "sel_resunit_bwd: fused path needs bf16, C = N in {32, 64}, K = 7, causal zero pad, ELU prologue");
  SEL_REQUIRE(g && h && x && wd1pack && wd2pack && gx, SEL_ERR_ARG, "null pointer");
  // tune key 41 = 1 (without gh): the eight-wave LDS-staged form, k_ru64_bwdw's
  // gx role on all waves (one workgroup per CU: measured slower than two
  // four-wave k_ru64_bwd workgroups, 82-83 vs 72 us per unit at C3)
  if (a.C == 64 && gh == nullptr && tune(41) == 1)
    return launch_ru64_bwdw<128, false>(a, g, h, x, wd1pack, wd2pack, gx, nullptr, nullptr, 0,
                                        reinterpret_cast<hipStream_t>(stream));
  if (a.C == 64)
    return launch_ru64_bwd<128>(a, g, h, x, wd1pack, wd2pack, gh, gx, reinterpret_cast<hipStream_t>(stream));
  return launch_ru32_bwd<128>(a, g, h, x, wd1pack, wd2pack, gh, gx, reinterpret_cast<hipStream_t>(stream));
}

int sel_resunit_wgrad_splits(const sel_conv_desc* d1, int dtype) {
  if (int rc = check_desc(d1)) return rc;
  const Args a = to_args(d1);
  SEL_REQUIRE(dtype == SEL_BF16 && ru_fused_ok(a) && a.rows > 0, SEL_ERR_UNSUPPORTED,
              "sel_resunit_bwd_wgrad: needs bf16, C = N in {32, 64}, K = 7, causal zero pad, ELU prologue");
  int64_t tpb = 1;
  const int64_t ntiles = (a.rows / a.T) * ((a.T + 127) / 128);
  return a.C == 64 ? ru64w_blocks<128>(ntiles, tpb) : ru32w_blocks<128>(ntiles, tpb);
}

int sel_resunit_bwd_wgrad(const sel_conv_desc* d1, int dtype, const void* g, const void* h, const void* x,
                          const void* wd1pack, const void* wd2pack, void* gx, float* part1, float* part2, int nsplit,
                          sel_stream_t stream) {
  if (int rc = check_desc(d1)) return rc;
  const Args a = to_args(d1);
  SEL_REQUIRE(dtype == SEL_BF16 && ru_fused_ok(a) && a.rows > 0, SEL_ERR_UNSUPPORTED,
              "sel_resunit_bwd_wgrad: needs bf16, C = N in {32, 64}, K = 7, causal zero pad, ELU prologue");
  SEL_REQUIRE(g && h && x && wd1pack && wd2pack && gx && part1 && part2, SEL_ERR_ARG, "null pointer");
  if (a.C == 64)
    return launch_ru64_bwdw<128>(a, g, h, x, wd1pack, wd2pack, gx, part1, part2, nsplit,
                                 reinterpret_cast<hipStream_t>(stream));
  return launch_ru32_bwdw<128>(a, g, h, x, wd1pack, wd2pack, gx, part1, part2, nsplit,
                               reinterpret_cast<hipStream_t>(stream));
}

size_t sel_conv_wgrad_workspace(const sel_conv_desc* d) {
  // (an invalid descriptor sizes nothing: sel_conv_wgrad* rejects it itself)
  if (!d || d->rows <= 0 || check_desc(d) != SEL_OK) return 16;
  int ns = wgrad_plan(d, 0).nsplit;
  if (wgrad_tr_ok(d)) ns = std::max(ns, std::max(wgrad_plan(d, 2).nsplit, wgrad_plan(d, 3).nsplit));
  if (wgrad_c1_ok(d)) ns = std::max(ns, wgrad_plan(d, 4).nsplit);
  const int ng = (ns + SPLIT_GROUP - 1) / SPLIT_GROUP;
  return size_t(ns + ng) * (size_t(d->N) * d->K * d->C + d->N) * sizeof(float);
}

namespace sel {
namespace conv {
struct UnpackSpec {
  int kind, cout, cin, k, stride;
};
int wgrad_impl(const sel_conv_desc* d, int dtype, const void* gout, const void* in, float* gwout,
               const UnpackSpec* up, float* gbias, void* ws, size_t ws_bytes, sel_stream_t stream,
               int* partials_only = nullptr);
}  // namespace conv
}  // namespace sel

int sel_conv_wgrad(const sel_conv_desc* d, int dtype, const void* gout, const void* in, float* gwpack,
                   float* gbias, void* ws, size_t ws_bytes, sel_stream_t stream) {
  return sel::conv::wgrad_impl(d, dtype, gout, in, gwpack, nullptr, gbias, ws, ws_bytes, stream);
}

int sel_conv_wgrad_unpacked(const sel_conv_desc* d, int dtype, const void* gout, const void* in, int kind, int cout,
                            int cin, int k, int stride, float* gw, float* gbias, void* ws, size_t ws_bytes,
                            sel_stream_t stream) {
  SEL_REQUIRE(kind >= SEL_PACK_FWD && kind <= SEL_PACK_CONVT, SEL_ERR_ARG, "bad pack kind");
  const int64_t packed = kind == SEL_PACK_FWD ? int64_t(cout) * k * cin
                         : kind == SEL_PACK_FWD_STRIDED ? int64_t(cout) * 3 * stride * cin
                                                        : int64_t(stride) * cout * 2 * cin;
  SEL_REQUIRE(d && packed == int64_t(d->N) * d->K * d->C, SEL_ERR_ARG, "weight shape does not match the descriptor");
  const sel::conv::UnpackSpec up{kind, cout, cin, k, stride};
  return sel::conv::wgrad_impl(d, dtype, gout, in, gw, &up, gbias, ws, ws_bytes, stream);
}

}  // extern "C"

namespace sel {
namespace conv {
int wgrad_impl(const sel_conv_desc* d, int dtype, const void* gout, const void* in, float* gwpack,
               const UnpackSpec* up, float* gbias, void* ws, size_t ws_bytes, sel_stream_t stream,
               int* partials_only) {
  if (int rc = check_desc(d)) return rc;
  SEL_REQUIRE(d->K * 2 <= WB_MAXJ * 1 || dtype == SEL_F32, SEL_ERR_UNSUPPORTED, "wgrad: K=%d too large", d->K);
  SEL_REQUIRE(dtype == SEL_BF16 || d->K * (kWgBN / 16) * 2 <= 4 * WG_MAXT, SEL_ERR_UNSUPPORTED,
              "wgrad: K=%d too large", d->K);
  SEL_REQUIRE(ws_bytes >= sel_conv_wgrad_workspace(d), SEL_ERR_WORKSPACE, "workspace too small");
  const Args a = to_args(d);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const WgPlan p = wgrad_plan(d, wgrad_mode(d, dtype));
  float* part = static_cast<float*>(ws);
  float* bpart = gbias ? part + size_t(p.nsplit) * d->N * d->K * d->C : nullptr;
  if (d->rows > 0 && p.mode == 4) {
    if (dtype == SEL_F32) {
      auto kc1 = d->N == 8 ? k_wgrad_c1<float, 1> : d->N == 16 ? k_wgrad_c1<float, 2>
                 : d->N == 32 ? k_wgrad_c1<float, 4> : k_wgrad_c1<float, 8>;
      hipLaunchKernelGGL(kc1, dim3(unsigned(p.nsplit)), dim3(256), 0, s, a, static_cast<const float*>(gout),
                         static_cast<const float*>(in), int64_t(p.tiles_per_split), part, bpart);
    } else {
      auto kc1 = d->N == 8 ? k_wgrad_c1<__bf16, 1> : d->N == 16 ? k_wgrad_c1<__bf16, 2>
                 : d->N == 32 ? k_wgrad_c1<__bf16, 4> : k_wgrad_c1<__bf16, 8>;
      hipLaunchKernelGGL(kc1, dim3(unsigned(p.nsplit)), dim3(256), 0, s, a, static_cast<const __bf16*>(gout),
                         static_cast<const __bf16*>(in), int64_t(p.tiles_per_split), part, bpart);
    }
    SEL_LAUNCH_CHECK();
  } else if (d->rows > 0 && p.mode == 3) {
    const __bf16* g16 = static_cast<const __bf16*>(gout);
    const __bf16* x16 = static_cast<const __bf16*>(in);
    if (p.nt == 1 && p.ct == 1) SEL_HIP((launch_wgrad3<1, 1>(p, a, g16, x16, part, bpart, s)));
    else if (p.nt == 2 && p.ct == 1) SEL_HIP((launch_wgrad3<2, 1>(p, a, g16, x16, part, bpart, s)));
    else if (p.nt == 1 && p.ct == 2) SEL_HIP((launch_wgrad3<1, 2>(p, a, g16, x16, part, bpart, s)));
    else SEL_HIP((launch_wgrad3<2, 2>(p, a, g16, x16, part, bpart, s)));
  } else if (d->rows > 0 && p.mode == 2) {
    // staging double buffer (40 KB) also hosts the [wave][taps][32x32] fp32 reduction
    const size_t lds = std::max<size_t>(size_t(2) * (W2_BM * 32 + (W2_BM + W2_HALO) * 32) * sizeof(__bf16),
                                        size_t(4) * 8 * 1024 * sizeof(float) / 4 * 1);
    dim3 grid(unsigned(d->N / 32), unsigned(d->C / 32), unsigned(p.nsplit));
#define SEL_WG2_LAUNCH(KM)                                                                                    \
  hipLaunchKernelGGL(k_wgrad2_bf16<KM>, grid, dim3(256), lds, s, a, static_cast<const __bf16*>(gout),          \
                     static_cast<const __bf16*>(in), int(p.tiles_per_sample), p.n_tiles, p.tiles_per_split, part, \
                     bpart)
    if (d->K == 1) SEL_WG2_LAUNCH(1);
    else if (d->K <= 4) SEL_WG2_LAUNCH(2);
    else SEL_WG2_LAUNCH(4);
#undef SEL_WG2_LAUNCH
    SEL_LAUNCH_CHECK();
  } else if (d->rows > 0 && dtype == SEL_BF16) {
    const int span = WB_BM + (d->K - 1) * d->dil;
    const size_t lds = (size_t(WB_BM) * (p.bn + 16) + size_t(span) * (WB_BC + 16)) * sizeof(__bf16);
    SEL_REQUIRE(lds <= 160 * 1024, SEL_ERR_UNSUPPORTED, "wgrad tile needs %zu B of LDS", lds);
    dim3 grid(unsigned((d->N + p.bn - 1) / p.bn), unsigned((d->C + WB_BC - 1) / WB_BC), unsigned(p.nsplit));
#define SEL_WG_LAUNCH(BNV)                                                                                     \
  {                                                                                                            \
    auto kern = k_wgrad_bf16<BNV>;                                                                             \
    if (lds > 64 * 1024)                                                                                       \
      SEL_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, int(lds)));   \
    hipLaunchKernelGGL(kern, grid, dim3(256), lds, s, a, static_cast<const __bf16*>(gout),                     \
                       static_cast<const __bf16*>(in), int(p.tiles_per_sample), p.n_tiles, p.tiles_per_split,  \
                       part, bpart);                                                                           \
  }
    if (p.bn == 16) SEL_WG_LAUNCH(16)
    else if (p.bn == 32) SEL_WG_LAUNCH(32)
    else SEL_WG_LAUNCH(64)
#undef SEL_WG_LAUNCH
    SEL_LAUNCH_CHECK();
  } else if (d->rows > 0 && dtype == SEL_F32 && d->C % 4 == 0 && d->N % 4 == 0 && d->K <= 8 &&
             (d->K - 1) * d->dil <= WF_XR - WF_BM && d->pad <= (d->K - 1) * d->dil && tune(54) != 1) {
    // fp32 on sample-aligned tiles (tune key 54 = 1: the generic kernel below);
    // every split of the plan owns at least one tile
    // block shape: 64 x 32 channels, or 32 x 64 / 32 x 32 for the 32-wide layers
    const int nb = d->N <= 32 ? 32 : 64, cb = nb == 64 ? 32 : (d->C % 64 == 0 ? 64 : 32);
    dim3 grid(unsigned((d->N + nb - 1) / nb), unsigned((d->C + cb - 1) / cb), unsigned(p.nsplit));
#define SEL_WGF(NB, CB)                                                                                       \
  {                                                                                                           \
    auto kern = d->K == 1 ? k_wgrad_f32<1, NB, CB> : d->K <= 3 ? k_wgrad_f32<3, NB, CB> : k_wgrad_f32<8, NB, CB>; \
    hipLaunchKernelGGL(kern, grid, dim3(256), 0, s, a, static_cast<const float*>(gout),                       \
                       static_cast<const float*>(in), int(p.tiles_per_sample), p.n_tiles, p.tiles_per_split, \
                       part, bpart);                                                                          \
  }
    if (nb == 64) SEL_WGF(64, 32)
    else if (cb == 64) SEL_WGF(32, 64)
    else SEL_WGF(32, 32)
#undef SEL_WGF
    SEL_LAUNCH_CHECK();
  } else if (d->rows > 0 && dtype == SEL_F32) {
    // fp32 parity path: flat row ranges, same number of splits as the plan
    const int64_t rps = ((d->rows + p.nsplit - 1) / p.nsplit + WG_BM - 1) / WG_BM * WG_BM;
    const int nsplit = int((d->rows + rps - 1) / rps);
    SEL_REQUIRE(nsplit <= p.nsplit, SEL_ERR_STATE, "internal split plan mismatch");
    const int span = WG_BM + (d->K - 1) * d->dil;
    const size_t lds = (size_t(WG_BM) * (kWgBN + WG_GP) + size_t(span) * (CK + WG_GP)) * sizeof(float);
    SEL_REQUIRE(lds <= 160 * 1024, SEL_ERR_UNSUPPORTED, "wgrad tile needs %zu B of LDS", lds);
    // unused tail splits must contribute zeros
    if (nsplit < p.nsplit)
      SEL_HIP(hipMemsetAsync(part + size_t(nsplit) * d->N * d->K * d->C, 0,
                             size_t(p.nsplit - nsplit) * d->N * d->K * d->C * sizeof(float), s));
    if (bpart && nsplit < p.nsplit)
      SEL_HIP(hipMemsetAsync(bpart + size_t(nsplit) * d->N, 0, size_t(p.nsplit - nsplit) * d->N * sizeof(float), s));
    dim3 grid(unsigned((d->N + kWgBN - 1) / kWgBN), unsigned((d->C + CK - 1) / CK), unsigned(nsplit));
    auto kern = k_conv_wgrad<float, kWgBN>;
    if (lds > 64 * 1024)
      SEL_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, int(lds)));
    hipLaunchKernelGGL(kern, grid, dim3(256), lds, s, a, static_cast<const float*>(gout),
                       static_cast<const float*>(in), rps, part, bpart);
    SEL_LAUNCH_CHECK();
  } else if (d->rows > 0) {
    set_error("bad dtype %d", dtype);
    return SEL_ERR_ARG;
  }
  if (partials_only) {  // sel_conv_wgrad_partials: the reduction is batched later
    *partials_only = p.nsplit;
    return SEL_OK;
  }
  // two-pass split reduction; the second-level partials live after the first-level ones
  const int64_t nw = int64_t(d->N) * d->K * d->C;
  const int ng = (p.nsplit + SPLIT_GROUP - 1) / SPLIT_GROUP;
  if (ng == 1 && tune(20) != 1) {  // one launch for both passes, the unpack and the bias (tune key 20: 1 = off)
    const int64_t nt = up ? (up->kind == SEL_PACK_CONVT ? int64_t(up->cin) * up->cout * 2 * up->stride
                             : int64_t(up->cout) * up->cin * (up->kind == SEL_PACK_FWD ? up->k : 2 * up->stride))
                          : nw;
    const int64_t nthreads = nt + (gbias ? d->bias_period : 0);
    hipLaunchKernelGGL(k_split_finish1, dim3(unsigned((nthreads + 255) / 256)), dim3(256), 0, s, part, p.nsplit, nw, nt,
                       up ? up->kind : -1, up ? up->cout : 0, up ? up->cin : 0, up ? up->k : 0, up ? up->stride : 0,
                       gwpack, bpart, int64_t(d->N), gbias ? d->bias_period : 0, gbias);
    SEL_LAUNCH_CHECK();
    return SEL_OK;
  }
  float* part2 = part + size_t(p.nsplit) * (size_t(d->N) * d->K * d->C + d->N);
  hipLaunchKernelGGL(k_split_sum1, dim3(unsigned((nw + 255) / 256), unsigned(ng)), dim3(256), 0, s, part, p.nsplit,
                     nw, part2);
  SEL_LAUNCH_CHECK();
  if (up) {
    const int64_t nt = up->kind == SEL_PACK_CONVT ? int64_t(up->cin) * up->cout * 2 * up->stride
                       : int64_t(up->cout) * up->cin * (up->kind == SEL_PACK_FWD ? up->k : 2 * up->stride);
    hipLaunchKernelGGL(k_split_sum2_unpack, dim3(unsigned((nt + 255) / 256)), dim3(256), 0, s, part2, ng, nw, nt,
                       up->kind, up->cout, up->cin, up->k, up->stride, gwpack);
  } else {
    hipLaunchKernelGGL(k_split_sum2, dim3(unsigned((nw + 255) / 256)), dim3(256), 0, s, part2, ng, nw, int(nw),
                       gwpack);
  }
  SEL_LAUNCH_CHECK();
  if (gbias) {
    float* bpart2 = part2 + size_t(ng) * nw;
    hipLaunchKernelGGL(k_split_sum1, dim3(unsigned((d->N + 255) / 256), unsigned(ng)), dim3(256), 0, s, bpart,
                       p.nsplit, int64_t(d->N), bpart2);
    SEL_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_split_sum2, dim3(unsigned((d->bias_period + 255) / 256)), dim3(256), 0, s, bpart2, ng,
                       int64_t(d->N), d->bias_period, gbias);
    SEL_LAUNCH_CHECK();
  }
  return SEL_OK;
}
}  // namespace conv
}  // namespace sel

namespace sel {
namespace conv {
// Batched split reduction (sel_wgrad_finish_many), with exactly the arithmetic
// of k_split_sum1 + k_split_sum2_unpack / k_split_sum2 (and of k_split_finish1,
// the one-group case of the same formula): group sums of 32 splits
// (split_group_sum), then the groups in order, four at a time.  A weight block
// owns 256 consecutive PACKED elements of one job (coalesced partial reads),
// one per thread: the thread adds its element's group sums in order and
// scatters to the torch layout.  A bias block owns one bias
// element: its threads compute the (group, column) sums, thread 0 adds them in
// order.  Block ranges per job come in the kernel argument.
constexpr int FM_MAXJ = 24;
constexpr int FM_MAXG = 32;  // split groups per job (nsplit <= 1024)
struct FinishJobs {
  sel_wgrad_job j[FM_MAXJ];
  int wblocks[FM_MAXJ];  // weight blocks of job j; its bias blocks follow
  int bstart[FM_MAXJ + 1];
  int njobs;
  int four;  // tune key 68 = 1: partial split groups four loads at a time (A/B)
};

// packed weight index -> torch-layout index (-1: a structural zero of the strided form)
__device__ __forceinline__ int64_t pack_dst(int kind, int64_t j, int cout, int cin, int K, int s) {
  if (kind < 0) return j;
  const int ci = int(j % cin);
  if (kind == SEL_PACK_FWD) {
    const int k = int((j / cin) % K);
    const int64_t co = j / (int64_t(cin) * K);
    return (co * cin + ci) * K + k;
  }
  if (kind == SEL_PACK_FWD_STRIDED) {
    const int ph = int((j / cin) % s);
    const int tap = int((j / (int64_t(s) * cin)) % 3);
    const int64_t co = j / (int64_t(3) * s * cin);
    const int k = tap == 0 ? (ph >= 1 ? ph - 1 : -1) : (tap == 1 ? ph + s - 1 : (ph == 0 ? 2 * s - 1 : -1));
    return k < 0 ? -1 : (co * cin + ci) * (2 * s) + k;
  }
  const int tap = int((j / cin) % 2);
  const int64_t r = j / (int64_t(2) * cin);
  const int ph = int(r / cout), co = int(r % cout);
  const int k = tap ? ph : ph + s;
  return (int64_t(ci) * cout + co) * (2 * s) + k;
}

__global__ __launch_bounds__(256) void k_wgrad_finish_many(FinishJobs fj) {
  __shared__ float gs[FM_MAXG][65];
  int jb = 0;
  while (jb + 1 < fj.njobs && int(blockIdx.x) >= fj.bstart[jb + 1]) ++jb;  // block-uniform
  const sel_wgrad_job& J = fj.j[jb];
  const int lb = int(blockIdx.x) - fj.bstart[jb];
  const int ng = (J.nsplit + SPLIT_GROUP - 1) / SPLIT_GROUP;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  auto group = [&](const float* p, int g, int64_t n) {
    const int s0 = g * SPLIT_GROUP, cnt = J.nsplit - s0 < SPLIT_GROUP ? J.nsplit - s0 : SPLIT_GROUP;
    return split_group_sum(p + int64_t(s0) * n, cnt, n, fj.four != 0);
  };
  if (lb < fj.wblocks[jb]) {
    // one packed element per thread, its group sums in order (the reduction
    // needs no LDS: all 256 threads stream partials, where the 64-element
    // blocks left three of four waves idle for the common one-group jobs)
    (void)lane;
    (void)wave;
    const int64_t j = int64_t(lb) * 256 + tid;
    if (j < J.nw) {
      float acc = 0.f;
      int g = 0;
      for (; g + 4 <= ng; g += 4) {
        const float g0 = group(J.part + j, g, J.nw), g1 = group(J.part + j, g + 1, J.nw);
        const float g2 = group(J.part + j, g + 2, J.nw), g3 = group(J.part + j, g + 3, J.nw);
        acc += (g0 + g1) + (g2 + g3);
      }
      for (; g < ng; ++g) acc += group(J.part + j, g, J.nw);
      const int64_t i = pack_dst(J.kind, j, J.cout, J.cin, J.k, J.stride);
      if (i >= 0) J.gw[i] = acc;
    }
  } else {
    const int jb2 = lb - fj.wblocks[jb];  // bias element
    const int M = J.N / J.bias_period;     // columns folded into it
    const float* bp = J.part + int64_t(J.nsplit) * J.nw;
    float* const ts = &gs[0][0];           // [g][m]
    for (int t = tid; t < ng * M; t += 256) ts[t] = group(bp + jb2 + int64_t(t % M) * J.bias_period, t / M, J.N);
    __syncthreads();
    if (tid == 0) {
      float acc = 0.f;
      for (int t = 0; t < ng * M; ++t) acc += ts[t];
      J.gb[jb2] = acc;
    }
  }
}
}  // namespace conv
}  // namespace sel

extern "C" {

int sel_conv_wgrad_partials(const sel_conv_desc* d, int dtype, const void* gout, const void* in, int want_bias,
                            void* ws, size_t ws_bytes, int* nsplit, sel_stream_t stream) {
  SEL_REQUIRE(nsplit, SEL_ERR_ARG, "null nsplit");
  int ns = 0;
  // a non-null bias pointer only selects the bias partials (it is never written here)
  float dummy = 0.f;
  const int rc = sel::conv::wgrad_impl(d, dtype, gout, in, nullptr, nullptr, want_bias ? &dummy : nullptr, ws,
                                       ws_bytes, stream, &ns);
  *nsplit = ns;
  return rc;
}

int sel_wgrad_finish_many(const sel_wgrad_job* jobs, int njobs, sel_stream_t stream) {
  using namespace sel::conv;
  SEL_REQUIRE(njobs >= 0 && (njobs == 0 || jobs), SEL_ERR_ARG, "bad job list");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  for (int j0 = 0; j0 < njobs; j0 += FM_MAXJ) {
    FinishJobs fj{};
    fj.njobs = std::min(FM_MAXJ, njobs - j0);
    fj.four = tune(68) == 1;
    int64_t blocks = 0;
    for (int j = 0; j < fj.njobs; ++j) {
      const sel_wgrad_job& J = jobs[j0 + j];
      SEL_REQUIRE(J.part && J.gw && J.nsplit > 0 && J.nsplit <= FM_MAXG * SPLIT_GROUP && J.nw > 0 && J.N > 0 &&
                      (J.gb == nullptr || (J.bias_period > 0 && J.N % J.bias_period == 0 &&
                                           (J.N / J.bias_period) * ((J.nsplit + SPLIT_GROUP - 1) / SPLIT_GROUP) <=
                                               FM_MAXG * 65)),
                  SEL_ERR_ARG, "bad wgrad job %d", j0 + j);
      fj.j[j] = J;
      fj.wblocks[j] = int((J.nw + 255) / 256);
      fj.bstart[j] = int(blocks);
      blocks += fj.wblocks[j] + (J.gb ? J.bias_period : 0);
    }
    fj.bstart[fj.njobs] = int(blocks);
    SEL_REQUIRE(blocks < (int64_t(1) << 31), SEL_ERR_ARG, "wgrad jobs too large");
    if (blocks > 0) {
      hipLaunchKernelGGL(k_wgrad_finish_many, dim3(unsigned(blocks)), dim3(256), 0, s, fj);
      SEL_LAUNCH_CHECK();
    }
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

int sel_pack_many(const sel_pack_job* jobs, int njobs, int64_t total, int dtype, sel_stream_t stream) {
  SEL_REQUIRE(jobs && njobs > 0 && total > 0, SEL_ERR_ARG, "empty pack job table");
  // (the job table is device memory: each job's element count is checked < 2^31
  // by the host binding, sel/convops.py PackCache._refresh)
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  dim3 grid(unsigned(std::min<int64_t>(8192, (2 * total + 255) / 256)));
  if (dtype == SEL_F32)
    hipLaunchKernelGGL(k_pack_many<float>, grid, dim3(256), 0, s, jobs, njobs, total);
  else
    hipLaunchKernelGGL(k_pack_many<__bf16>, grid, dim3(256), 0, s, jobs, njobs, total);
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

int sel_pack_many_host(const sel_pack_job* jobs, int njobs, int64_t total, int dtype, sel_stream_t stream) {
  using namespace sel::conv;
  SEL_REQUIRE(jobs && njobs > 0 && total > 0, SEL_ERR_ARG, "empty pack job table");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  for (int j0 = 0; j0 < njobs; j0 += PM_MAXJ) {
    PackJobs pj{};
    pj.n = std::min(PM_MAXJ, njobs - j0);
    for (int j = 0; j < pj.n; ++j) {
      pj.j[j] = jobs[j0 + j];
      SEL_REQUIRE(pj.j[j].offset >= 0 && pj.j[j].offset < total && (j == 0 || pj.j[j].offset > pj.j[j - 1].offset),
                  SEL_ERR_ARG, "pack jobs must have increasing offsets within total");
    }
    // tiled kernel (k_pack_tiles) unless a job's taps exceed its tile (K > 8)
    // or tune key 60 = 1 asks for the per-element form
    PackTiles pt{};
    bool tiled = tune(60) != 1;
    int64_t tiles = 0;
    pt.n = pj.n;
    for (int j = 0; j < pj.n && tiled; ++j) {
      const sel_pack_job& J = pj.j[j];
      const int64_t N = J.kind == SEL_PACK_CONVT ? int64_t(J.stride) * J.cout : J.cout;
      const int64_t KP = J.kind == SEL_PACK_FWD ? J.k : J.kind == SEL_PACK_FWD_STRIDED ? 3 : 2;
      const int64_t CP = J.kind == SEL_PACK_FWD_STRIDED ? int64_t(J.stride) * J.cin : J.cin;
      if (KP > PT_KMAX) tiled = false;
      pt.j[j] = J;
      pt.tstart[j] = int(tiles);
      tiles += ((N + PT_T - 1) / PT_T) * ((CP + PT_T - 1) / PT_T);
    }
    pt.tstart[pt.n] = int(tiles);
    if (tiled && tiles > 0 && tiles < (int64_t(1) << 31)) {
      if (dtype == SEL_F32)
        hipLaunchKernelGGL((k_pack_tiles<float, 1024>), dim3(unsigned(tiles)), dim3(1024), 0, s, pt);
      else
        hipLaunchKernelGGL((k_pack_tiles<__bf16, 1024>), dim3(unsigned(tiles)), dim3(1024), 0, s, pt);
      SEL_LAUNCH_CHECK();
      continue;
    }
    const int64_t lo = pj.j[0].offset;
    const int64_t hi = j0 + pj.n < njobs ? jobs[j0 + pj.n].offset : total;
    dim3 grid(unsigned(std::min<int64_t>(8192, (2 * (hi - lo) + 255) / 256)));
    if (dtype == SEL_F32)
      hipLaunchKernelGGL(k_pack_many_arg<float>, grid, dim3(256), 0, s, pj, lo, hi, total);
    else
      hipLaunchKernelGGL(k_pack_many_arg<__bf16>, grid, dim3(256), 0, s, pj, lo, hi, total);
    SEL_LAUNCH_CHECK();
  }
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
  const dim3 grid(nb, unsigned((d->C + 63) / 64));
  if (dtype == SEL_F32)
    hipLaunchKernelGGL(k_replicate_fix<float>, grid, dim3(1024), 0, s, a, static_cast<const float*>(gout),
                       static_cast<const float*>(wpack), static_cast<float*>(gin));
  else
    hipLaunchKernelGGL(k_replicate_fix<__bf16>, grid, dim3(1024), 0, s, a, static_cast<const __bf16*>(gout),
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
