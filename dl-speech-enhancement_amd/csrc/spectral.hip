// Spectral hot path of the denoise trainer on gfx950:
//   STFT magnitude (losses/stft_loss.py:19-35), fused STFT loss (stft_loss.py:100-117),
//   log-mel (losses/mel_loss.py:74-94) and their backward passes.
//
// Design (one frame = one n_fft window of one signal):
//   * a frame is owned by TPF = n_fft/8 lanes; a 256-lane workgroup holds
//     FPB = 256/TPF frames (n_fft 2048: 1, 1024: 2, 512: 4, 256: 8);
//   * load: reflect-padded, window-multiplied samples are packed two per complex
//     point (even + i*odd) straight from HBM into LDS — coalesced 8-B pairs;
//   * FFT: half-size (n_fft/2) complex Stockham autosort in LDS, radix-4 passes
//     (+ one radix-2 pass when log2(n_fft/2) is odd), twiddles from a
//     device-resident table computed in double on the host;
//   * real split -> X_k, k = 0..n_fft/2, kept in registers (4 bins per lane,
//     bin n_fft/2 on lane 0);
//   * epilogues: |X| store, fused loss partial sums, sparse mel projection + log;
//   * backward: dL/dX from the epilogue's adjoint, c2r through the same forward
//     FFT on conjugated data, window multiply, per-frame slab -> overlap-add +
//     reflect-pad fold in a separate gather kernel (deterministic, no atomics).
#include <cmath>

#include "sel_common.h"
#include "spectral_tables.h"

namespace sel {
namespace spec {

__device__ float2 g_tw[kTwTotal];

hipError_t upload_twiddles(const float2* host, size_t count) {
  return hipMemcpyToSymbol(HIP_SYMBOL(g_tw), host, count * sizeof(float2));
}

__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
// multiply by -i
__device__ __forceinline__ float2 cmni(float2 a) { return make_float2(a.y, -a.x); }
__device__ __forceinline__ float2 conjf2(float2 a) { return make_float2(a.x, -a.y); }

template <int LOGN>
struct Geo {
  static constexpr int N = 1 << LOGN;
  static constexpr int M = N / 2;
  static constexpr int TPF = N / 8;                       // lanes per frame
  static constexpr int FPB = TPF >= 256 ? 1 : 256 / TPF;  // frames per block
  static constexpr int BLOCK = TPF * FPB;
  static constexpr int BUF = M + 8;                       // complex slots per LDS buffer
};

struct FrameArgs {
  int64_t B, T;
  int F, hop, win, left, P;  // P = n_fft/2 reflect pad
};

__device__ __forceinline__ int64_t reflect_index(int64_t j, int64_t T) {
  j = j < 0 ? -j : j;
  j = j >= T ? 2 * (T - 1) - j : j;
  return j;
}

// Windowed, reflect-padded frame -> packed complex buffer (even + i*odd).
template <int LOGN>
__device__ __forceinline__ void load_frame(const float* __restrict__ x, const FrameArgs& a, int f,
                                           const float* __restrict__ window, float2* buf, int t,
                                           bool active) {
  using G = Geo<LOGN>;
  const int64_t base = int64_t(f) * a.hop - a.P;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int m = t + q * G::TPF;
    const int n0 = 2 * m, n1 = n0 + 1;
    float v0 = 0.f, v1 = 0.f;
    if (active) {
      const int w0 = n0 - a.left, w1 = n1 - a.left;
      if (w0 >= 0 && w0 < a.win) v0 = window[w0] * x[reflect_index(base + n0, a.T)];
      if (w1 >= 0 && w1 < a.win) v1 = window[w1] * x[reflect_index(base + n1, a.T)];
    }
    buf[m] = make_float2(v0, v1);
  }
}

// In-LDS forward complex FFT of M = N/2 points (Stockham autosort, natural order).
// All block lanes must call it (contains __syncthreads). Returns the result buffer.
template <int LOGN>
__device__ __forceinline__ float2* fft_half(float2* src, float2* dst, int t) {
  using G = Geo<LOGN>;
  constexpr int M = G::M;
  const float2* __restrict__ twM = g_tw + tw_off(LOGN);
  int Ns = 1;
#pragma unroll
  for (int pass = 0; pass < (LOGN - 1) / 2; ++pass) {
    const int j = t;
    const int k = j & (Ns - 1);
    float2 v0 = src[j], v1 = src[j + M / 4], v2 = src[j + M / 2], v3 = src[j + 3 * M / 4];
    if (pass > 0) {
      const int step = M / (4 * Ns);
      v1 = cmul(v1, twM[k * step]);
      v2 = cmul(v2, twM[2 * k * step]);
      v3 = cmul(v3, twM[3 * k * step]);
    }
    const float2 t0 = cadd(v0, v2), t1 = csub(v0, v2), t2 = cadd(v1, v3), t3 = cmni(csub(v1, v3));
    const int d = (j - k) * 4 + k;
    dst[d] = cadd(t0, t2);
    dst[d + Ns] = cadd(t1, t3);
    dst[d + 2 * Ns] = csub(t0, t2);
    dst[d + 3 * Ns] = csub(t1, t3);
    __syncthreads();
    float2* tmp = src;
    src = dst;
    dst = tmp;
    Ns *= 4;
  }
  if ((LOGN - 1) & 1) {  // final radix-2 pass, Ns = M/2
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int j = t + h * G::TPF;  // j < M/2 == Ns -> k == j
      const float2 v0 = src[j];
      const float2 v1 = cmul(src[j + M / 2], twM[j]);
      dst[j] = cadd(v0, v1);
      dst[j + M / 2] = csub(v0, v1);
    }
    __syncthreads();
    src = dst;
  }
  return src;
}

// Real split: X_k for this lane's bins k = t + q*TPF (q < 4) and X_M (lane 0).
template <int LOGN>
__device__ __forceinline__ void real_split(const float2* Z, int t, float2 (&X)[4], float2& XM) {
  using G = Geo<LOGN>;
  constexpr int M = G::M;
  const float2* __restrict__ twN = g_tw + tw_off(LOGN) + M;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int k = t + q * G::TPF;
    if (k == 0) {
      const float2 z0 = Z[0];
      X[q] = make_float2(z0.x + z0.y, 0.f);
      XM = make_float2(z0.x - z0.y, 0.f);
    } else {
      const float2 zk = Z[k], zm = Z[M - k];
      const float2 e = make_float2(0.5f * (zk.x + zm.x), 0.5f * (zk.y - zm.y));
      const float2 o = make_float2(0.5f * (zk.y + zm.y), -0.5f * (zk.x - zm.x));
      X[q] = cadd(e, cmul(twN[k], o));
    }
  }
}

// Inverse of real_split for a gradient: given G_k (k = 0..M) in `Gb`, build the
// half-size spectrum Z'_k, run the forward FFT on conj(Z') and return the
// buffer holding conj(z'); r[2m] = R[m].x, r[2m+1] = -R[m].y with
// r_n = Re sum_{k=0}^{M} G_k exp(+2 pi i k n / N).
template <int LOGN>
__device__ __forceinline__ float2* c2r_grad(float2* Gb, float2* other, int t) {
  using G = Geo<LOGN>;
  constexpr int M = G::M;
  const float2* __restrict__ twN = g_tw + tw_off(LOGN) + M;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int k = t + q * G::TPF;
    float2 zp;
    if (k == 0) {
      const float h0 = Gb[0].x, hm = Gb[M].x;
      zp = make_float2(h0 + hm, h0 - hm);
    } else {
      const float2 gk = Gb[k], gm = Gb[M - k];
      const float2 s = make_float2(gk.x + gm.x, gk.y - gm.y);  // gk + conj(gm)
      const float2 d = make_float2(gk.x - gm.x, gk.y + gm.y);  // gk - conj(gm)
      const float2 wd = cmul(conjf2(twN[k]), d);                // W^-k * d
      // 0.5 * (s + i * wd)
      zp = make_float2(0.5f * (s.x - wd.y), 0.5f * (s.y + wd.x));
    }
    other[k] = conjf2(zp);
  }
  __syncthreads();
  return fft_half<LOGN>(other, Gb, t);
}

// Windowed frame-gradient slab: ws[(frame)*win + (n - left)] = window * r_n.
template <int LOGN>
__device__ __forceinline__ void store_frame_grad(const float2* R, const FrameArgs& a,
                                                 const float* __restrict__ window,
                                                 float* __restrict__ slab, int t, bool active) {
  using G = Geo<LOGN>;
  if (!active) return;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int m = t + q * G::TPF;
    const float2 r = R[m];
    const int w0 = 2 * m - a.left, w1 = w0 + 1;
    if (w0 >= 0 && w0 < a.win) slab[w0] = window[w0] * r.x;
    if (w1 >= 0 && w1 < a.win) slab[w1] = window[w1] * (-r.y);
  }
}

__device__ __forceinline__ float clamp_sqrt(float p, float floor_) { return sqrtf(fmaxf(p, floor_)); }
__device__ __forceinline__ float pw(float2 z) { return z.x * z.x + z.y * z.y; }

// -------------------------------------------------------------------------
// Kernels
// -------------------------------------------------------------------------

#define FRAME_PROLOGUE(LOGN)                                               \
  using G = Geo<LOGN>;                                                     \
  __shared__ float2 lds[G::FPB][2][G::BUF];                                \
  const int g = threadIdx.x / G::TPF;                                      \
  const int t = threadIdx.x % G::TPF;                                      \
  const int64_t fr = int64_t(blockIdx.x) * G::FPB + g;                    \
  const bool active = fr < a.B * a.F;                                      \
  const int64_t b = active ? fr / a.F : 0;                                 \
  const int f = active ? int(fr % a.F) : 0;                                \
  float2* buf0 = lds[g][0];                                                \
  float2* buf1 = lds[g][1];

template <int LOGN>
__global__ __launch_bounds__(Geo<LOGN>::BLOCK) void k_stft_mag_fwd(
    const float* __restrict__ x, FrameArgs a, const float* __restrict__ window, float floor_,
    float* __restrict__ mag) {
  FRAME_PROLOGUE(LOGN)
  load_frame<LOGN>(x + b * a.T, a, f, window, buf0, t, active);
  __syncthreads();
  const float2* Z = fft_half<LOGN>(buf0, buf1, t);
  float2 X[4], XM;
  real_split<LOGN>(Z, t, X, XM);
  if (!active) return;
  constexpr int K = G::M + 1;
  float* out = mag + fr * K;
#pragma unroll
  for (int q = 0; q < 4; ++q) out[t + q * G::TPF] = clamp_sqrt(pw(X[q]), floor_);
  if (t == 0) out[G::M] = clamp_sqrt(pw(XM), floor_);
}

template <int LOGN>
__global__ __launch_bounds__(Geo<LOGN>::BLOCK) void k_stft_mag_bwd(
    const float* __restrict__ x, FrameArgs a, const float* __restrict__ window, float floor_,
    const float* __restrict__ gmag, float* __restrict__ slab) {
  FRAME_PROLOGUE(LOGN)
  load_frame<LOGN>(x + b * a.T, a, f, window, buf0, t, active);
  __syncthreads();
  float2* Z = fft_half<LOGN>(buf0, buf1, t);
  float2 X[4], XM;
  real_split<LOGN>(Z, t, X, XM);
  __syncthreads();  // everyone done reading Z before it is overwritten with G
  constexpr int K = G::M + 1;
  const float* gm = gmag + (active ? fr : 0) * K;
  float2* Gb = Z;
  float2* other = (Z == buf0) ? buf1 : buf0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int k = t + q * G::TPF;
    const float p = pw(X[q]);
    const float s = (active && p >= floor_) ? gm[k] / sqrtf(p) : 0.f;
    Gb[k] = make_float2(s * X[q].x, s * X[q].y);
  }
  if (t == 0) {
    const float p = pw(XM);
    const float s = (active && p >= floor_) ? gm[G::M] / sqrtf(p) : 0.f;
    Gb[G::M] = make_float2(s * XM.x, s * XM.y);
  }
  __syncthreads();
  const float2* R = c2r_grad<LOGN>(Gb, other, t);
  store_frame_grad<LOGN>(R, a, window, slab + (active ? fr : 0) * a.win, t, active);
}

// Fused STFT loss forward: both signals' spectra in LDS, block partial sums
// {sum (ym-xm)^2, sum ym^2, sum |ln ym - ln xm|} (stft_loss.py:56, :77).
template <int LOGN>
__global__ __launch_bounds__(Geo<LOGN>::BLOCK) void k_stft_loss_fwd(
    const float* __restrict__ x, const float* __restrict__ y, FrameArgs a,
    const float* __restrict__ window, float floor_, double* __restrict__ partials) {
  FRAME_PROLOGUE(LOGN)
  __shared__ double red[16];
  float ym[5];
  {
    load_frame<LOGN>(y + b * a.T, a, f, window, buf0, t, active);
    __syncthreads();
    const float2* Z = fft_half<LOGN>(buf0, buf1, t);
    float2 X[4], XM;
    real_split<LOGN>(Z, t, X, XM);
#pragma unroll
    for (int q = 0; q < 4; ++q) ym[q] = clamp_sqrt(pw(X[q]), floor_);
    ym[4] = clamp_sqrt(pw(XM), floor_);
    __syncthreads();
  }
  load_frame<LOGN>(x + b * a.T, a, f, window, buf0, t, active);
  __syncthreads();
  const float2* Z = fft_half<LOGN>(buf0, buf1, t);
  float2 X[4], XM;
  real_split<LOGN>(Z, t, X, XM);
  float s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (active) {
#pragma unroll
    for (int q = 0; q < 5; ++q) {
      if (q == 4 && t != 0) break;
      const float xm = clamp_sqrt(pw(q < 4 ? X[q] : XM), floor_);
      const float d = ym[q] - xm;
      s1 += d * d;
      s2 += ym[q] * ym[q];
      s3 += fabsf(logf(ym[q]) - logf(xm));
    }
  }
  const double r1 = block_sum<double>(s1, red);
  const double r2 = block_sum<double>(s2, red);
  const double r3 = block_sum<double>(s3, red);
  if (threadIdx.x == 0) {
    partials[3 * blockIdx.x + 0] = r1;
    partials[3 * blockIdx.x + 1] = r2;
    partials[3 * blockIdx.x + 2] = r3;
  }
}

template <int LOGN>
__global__ __launch_bounds__(Geo<LOGN>::BLOCK) void k_stft_loss_bwd(
    const float* __restrict__ x, const float* __restrict__ y, FrameArgs a,
    const float* __restrict__ window, float floor_, const float* __restrict__ coef,
    float* __restrict__ slab) {
  FRAME_PROLOGUE(LOGN)
  float ym[5];
  {
    load_frame<LOGN>(y + b * a.T, a, f, window, buf0, t, active);
    __syncthreads();
    const float2* Z = fft_half<LOGN>(buf0, buf1, t);
    float2 X[4], XM;
    real_split<LOGN>(Z, t, X, XM);
#pragma unroll
    for (int q = 0; q < 4; ++q) ym[q] = clamp_sqrt(pw(X[q]), floor_);
    ym[4] = clamp_sqrt(pw(XM), floor_);
    __syncthreads();
  }
  load_frame<LOGN>(x + b * a.T, a, f, window, buf0, t, active);
  __syncthreads();
  float2* Z = fft_half<LOGN>(buf0, buf1, t);
  float2 X[4], XM;
  real_split<LOGN>(Z, t, X, XM);
  __syncthreads();
  const float ca = coef[0], cb = coef[1];
  float2* Gb = Z;
  float2* other = (Z == buf0) ? buf1 : buf0;
#pragma unroll
  for (int q = 0; q < 5; ++q) {
    if (q == 4 && t != 0) break;
    const float2 Xq = q < 4 ? X[q] : XM;
    const float p = pw(Xq);
    const float xm = clamp_sqrt(p, floor_);
    const float lx = logf(xm), ly = logf(ym[q]);
    const float sg = lx > ly ? 1.f : (lx < ly ? -1.f : 0.f);
    const float gx = ca * (xm - ym[q]) + cb * sg / xm;
    const float s = (active && p >= floor_) ? gx / xm : 0.f;
    Gb[q < 4 ? t + q * G::TPF : G::M] = make_float2(s * Xq.x, s * Xq.y);
  }
  __syncthreads();
  const float2* R = c2r_grad<LOGN>(Gb, other, t);
  store_frame_grad<LOGN>(R, a, window, slab + (active ? fr : 0) * a.win, t, active);
}

__device__ __forceinline__ float log_k(float v, int kind) {
  return kind == SEL_LOG_E ? logf(v) : (kind == SEL_LOG_2 ? log2f(v) : log10f(v));
}
__device__ __forceinline__ float dlog_k(int kind) {
  return kind == SEL_LOG_E ? 1.f : (kind == SEL_LOG_2 ? 0.6931471805599453f : 2.302585092994046f);
}

struct MelArgs {
  const float* melmat;     // (K, nm)
  const int2* range;       // fwd: per-mel bin range; bwd: per-bin mel range
  int nm;
  float eps;
  int log_kind;
};

// log-mel forward (mel_loss.py:84-94): stft -> |X| (floor eps) -> melmat -> floor eps -> log.
template <int LOGN>
__global__ __launch_bounds__(Geo<LOGN>::BLOCK) void k_logmel_fwd(
    const float* __restrict__ x, FrameArgs a, const float* __restrict__ window, MelArgs ma,
    float* __restrict__ out) {
  FRAME_PROLOGUE(LOGN)
  load_frame<LOGN>(x + b * a.T, a, f, window, buf0, t, active);
  __syncthreads();
  float2* Z = fft_half<LOGN>(buf0, buf1, t);
  float2 X[4], XM;
  real_split<LOGN>(Z, t, X, XM);
  float* magb = reinterpret_cast<float*>((Z == buf0) ? buf1 : buf0);
#pragma unroll
  for (int q = 0; q < 4; ++q) magb[t + q * G::TPF] = clamp_sqrt(pw(X[q]), ma.eps);
  if (t == 0) magb[G::M] = clamp_sqrt(pw(XM), ma.eps);
  __syncthreads();
  if (!active) return;
  for (int m = t; m < ma.nm; m += G::TPF) {
    const int2 r = ma.range[m];
    float s = 0.f;
    for (int k = r.x; k < r.y; ++k) s = fmaf(magb[k], ma.melmat[k * ma.nm + m], s);
    out[(b * ma.nm + m) * a.F + f] = log_k(fmaxf(s, ma.eps), ma.log_kind);
  }
}

// log-mel backward. gsel: if ref != nullptr, upstream = g_scale * sign(gout - ref)
// (L1 backward, mel_loss.py:153); else upstream = gout.
template <int LOGN>
__global__ __launch_bounds__(Geo<LOGN>::BLOCK) void k_logmel_bwd(
    const float* __restrict__ x, FrameArgs a, const float* __restrict__ window, MelArgs ma,
    const int2* __restrict__ krange, const float* __restrict__ gout,
    const float* __restrict__ ref, const float* __restrict__ gscale, float gmul,
    float* __restrict__ slab) {
  FRAME_PROLOGUE(LOGN)
  load_frame<LOGN>(x + b * a.T, a, f, window, buf0, t, active);
  __syncthreads();
  float2* Z = fft_half<LOGN>(buf0, buf1, t);
  float2 X[4], XM;
  real_split<LOGN>(Z, t, X, XM);
  float2* other = (Z == buf0) ? buf1 : buf0;
  float* magb = reinterpret_cast<float*>(other);
  float* glin = magb + G::M + 4;
#pragma unroll
  for (int q = 0; q < 4; ++q) magb[t + q * G::TPF] = clamp_sqrt(pw(X[q]), ma.eps);
  if (t == 0) magb[G::M] = clamp_sqrt(pw(XM), ma.eps);
  __syncthreads();
  const float gs = ref ? gscale[0] * gmul : 0.f;
  for (int m = t; m < ma.nm; m += G::TPF) {
    float v = 0.f;
    if (active) {
      const int2 r = krange[m];
      float s = 0.f;
      for (int k = r.x; k < r.y; ++k) s = fmaf(magb[k], ma.melmat[k * ma.nm + m], s);
      const int64_t o = (b * ma.nm + m) * a.F + f;
      float up;
      if (ref) {
        const float d = gout[o] - ref[o];
        up = d > 0.f ? gs : (d < 0.f ? -gs : 0.f);
      } else {
        up = gout[o];
      }
      const float mel = fmaxf(s, ma.eps);
      v = (s >= ma.eps) ? up / (mel * dlog_k(ma.log_kind)) : 0.f;
    }
    glin[m] = v;
  }
  __syncthreads();
  float2* Gb = Z;
#pragma unroll
  for (int q = 0; q < 5; ++q) {
    if (q == 4 && t != 0) break;
    const int k = q < 4 ? t + q * G::TPF : G::M;
    const float2 Xq = q < 4 ? X[q] : XM;
    const int2 r = ma.range[k];
    float gmag = 0.f;
    for (int m = r.x; m < r.y; ++m) gmag = fmaf(ma.melmat[k * ma.nm + m], glin[m], gmag);
    const float p = pw(Xq);
    const float s = (active && p >= ma.eps) ? gmag / sqrtf(p) : 0.f;
    Gb[k] = make_float2(s * Xq.x, s * Xq.y);
  }
  __syncthreads();
  const float2* R = c2r_grad<LOGN>(Gb, other, t);
  store_frame_grad<LOGN>(R, a, window, slab + (active ? fr : 0) * a.win, t, active);
}

// Overlap-add of frame-gradient slabs + adjoint of the reflect pad -> g_x (B,T).
__device__ __forceinline__ float ola_at(const float* __restrict__ slab, const FrameArgs& a, int64_t i) {
  // frames f with 0 <= i - f*hop - left < win
  const int64_t r = i - a.left;
  if (r < 0) return 0.f;
  int64_t fhi = r / a.hop;
  int64_t flo = r - (a.win - 1);
  flo = flo <= 0 ? 0 : (flo + a.hop - 1) / a.hop;
  if (fhi > a.F - 1) fhi = a.F - 1;
  float s = 0.f;
  for (int64_t f = flo; f <= fhi; ++f) s += slab[f * a.win + (r - f * a.hop)];
  return s;
}

__global__ __launch_bounds__(256) void k_ola_fold(const float* __restrict__ slab, FrameArgs a,
                                                  float* __restrict__ gx) {
  const int64_t b = blockIdx.y;
  const int64_t t = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t >= a.T) return;
  const float* s = slab + b * int64_t(a.F) * a.win;
  float v = ola_at(s, a, t + a.P);
  if (t >= 1 && t <= a.P) v += ola_at(s, a, a.P - t);
  if (t >= a.T - 1 - a.P && t <= a.T - 2) v += ola_at(s, a, 2 * a.T - 2 + a.P - t);
  gx[b * a.T + t] = v;
}

// ---- reductions --------------------------------------------------------

// partial sums over (x_mag, y_mag) pairs: {sum (y-x)^2, sum y^2, sum |ln y - ln x|}
__global__ __launch_bounds__(256) void k_mag_pair_partials(const float* __restrict__ xm,
                                                           const float* __restrict__ ym, int64_t n,
                                                           double* __restrict__ partials) {
  __shared__ double red[16];
  float s1 = 0.f, s2 = 0.f, s3 = 0.f;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += int64_t(gridDim.x) * blockDim.x) {
    const float xv = xm[i], yv = ym[i];
    const float d = yv - xv;
    s1 += d * d;
    s2 += yv * yv;
    s3 += fabsf(logf(yv) - logf(xv));
  }
  const double r1 = block_sum<double>(s1, red);
  const double r2 = block_sum<double>(s2, red);
  const double r3 = block_sum<double>(s3, red);
  if (threadIdx.x == 0) {
    partials[3 * blockIdx.x + 0] = r1;
    partials[3 * blockIdx.x + 1] = r2;
    partials[3 * blockIdx.x + 2] = r3;
  }
}

__global__ __launch_bounds__(256) void k_abs_diff_partials(const float* __restrict__ a_,
                                                           const float* __restrict__ b_, int64_t n,
                                                           double* __restrict__ partials) {
  __shared__ double red[16];
  float s = 0.f;
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += int64_t(gridDim.x) * blockDim.x)
    s += fabsf(a_[i] - b_[i]);
  const double r = block_sum<double>(s, red);
  if (threadIdx.x == 0) partials[blockIdx.x] = r;
}

// Sum `np` partial vectors of width W -> sums[W] (double); optionally mean -> fout.
__global__ __launch_bounds__(256) void k_finish_partials(const double* __restrict__ partials, int np,
                                                         int W, double* __restrict__ sums,
                                                         float* __restrict__ fout, double inv_n) {
  __shared__ double red[16];
  for (int w = 0; w < W; ++w) {
    double s = 0.0;
    for (int i = threadIdx.x; i < np; i += blockDim.x) s += partials[i * W + w];
    s = block_sum<double>(s, red);
    if (threadIdx.x == 0) {
      if (sums) sums[w] = s;
      if (fout) fout[w] = float(s * inv_n);
    }
    __syncthreads();
  }
}

// {sc, mag} from sums (stft_loss.py:56, :77)
__global__ void k_stft_loss_finish(const double* __restrict__ sums, double inv_n, float* out2) {
  const float n1 = sqrtf(float(sums[0])), n2 = sqrtf(float(sums[1]));
  out2[0] = n1 / n2;
  out2[1] = float(sums[2] * inv_n);
}

// coef {a, b, c, d} for the magnitude-pair backward given upstream {g_sc, g_mag}.
__global__ void k_stft_loss_coef(const double* __restrict__ sums, double inv_n,
                                 const float* __restrict__ g_sc, const float* __restrict__ g_mag,
                                 float* coef) {
  const float n1 = sqrtf(float(sums[0])), n2 = sqrtf(float(sums[1]));
  const float gsc = g_sc ? g_sc[0] : 0.f, gmag = g_mag ? g_mag[0] : 0.f;
  // d||y-x||/dx = (x-y)/||y-x|| (0 when the norm is 0), then /n2
  const float a = n1 > 0.f ? gsc / (n1 * n2) : 0.f;
  coef[0] = a;
  coef[1] = float(gmag * inv_n);
  coef[2] = a;                                    // d/dy of ||y-x||/n2 numerator part
  coef[3] = n2 > 0.f ? -gsc * (n1 / n2) / (n2 * n2) : 0.f;  // -sc/n2^2 * y
}

__global__ __launch_bounds__(256) void k_mag_pair_bwd(const float* __restrict__ xm,
                                                      const float* __restrict__ ym, int64_t n,
                                                      const float* __restrict__ coef,
                                                      float* __restrict__ gx, float* __restrict__ gy) {
  const float ca = coef[0], cb = coef[1], cc = coef[2], cd = coef[3];
  for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += int64_t(gridDim.x) * blockDim.x) {
    const float xv = xm[i], yv = ym[i];
    const float lx = logf(xv), ly = logf(yv);
    const float sg = lx > ly ? 1.f : (lx < ly ? -1.f : 0.f);
    gx[i] = ca * (xv - yv) + cb * sg / xv;
    if (gy) gy[i] = cc * (yv - xv) + cd * yv - cb * sg / yv;
  }
}

}  // namespace spec
}  // namespace sel

// -------------------------------------------------------------------------
// C ABI
// -------------------------------------------------------------------------
using namespace sel;
using namespace sel::spec;

namespace {

int check_frame(int64_t B, int64_t T, int n_fft, int hop, int win, int& logn) {
  SEL_REQUIRE(initialized(), SEL_ERR_STATE, "sel_init() has not succeeded");
  SEL_REQUIRE(B >= 0 && T > 0, SEL_ERR_ARG, "bad signal shape (%lld, %lld)", (long long)B, (long long)T);
  SEL_REQUIRE(n_fft > 0 && (n_fft & (n_fft - 1)) == 0, SEL_ERR_UNSUPPORTED,
              "n_fft=%d: only powers of two are implemented", n_fft);
  logn = 0;
  while ((1 << logn) < n_fft) ++logn;
  SEL_REQUIRE(logn >= kMinLog && logn <= kMaxLog - 1, SEL_ERR_UNSUPPORTED,
              "n_fft=%d outside [256, 2048]", n_fft);
  SEL_REQUIRE(hop > 0, SEL_ERR_ARG, "hop must be > 0");
  SEL_REQUIRE(win > 0 && win <= n_fft, SEL_ERR_ARG, "win_length=%d must be in (0, n_fft=%d]", win, n_fft);
  // torch.stft(center=True, pad_mode='reflect') requires pad < input length
  SEL_REQUIRE(T > n_fft / 2, SEL_ERR_ARG,
              "reflect padding (%d) must be smaller than the signal length (%lld)", n_fft / 2,
              (long long)T);
  return SEL_OK;
}

FrameArgs frame_args(int64_t B, int64_t T, int n_fft, int hop, int win) {
  FrameArgs a;
  a.B = B;
  a.T = T;
  a.F = int(1 + T / hop);
  a.hop = hop;
  a.win = win;
  a.left = (n_fft - win) / 2;
  a.P = n_fft / 2;
  return a;
}

// dispatch helper: one template kernel family over LOGN in [8, 11]
#define SEL_FRAME_DISPATCH(logn, nframes, stream, KER, ...)                                  \
  do {                                                                                       \
    switch (logn) {                                                                          \
      case 8: {                                                                              \
        using G = Geo<8>;                                                                    \
        dim3 grid(unsigned((nframes + G::FPB - 1) / G::FPB));                                \
        if (grid.x) hipLaunchKernelGGL(KER<8>, grid, dim3(G::BLOCK), 0, stream, __VA_ARGS__);   \
      } break;                                                                               \
      case 9: {                                                                              \
        using G = Geo<9>;                                                                    \
        dim3 grid(unsigned((nframes + G::FPB - 1) / G::FPB));                                \
        if (grid.x) hipLaunchKernelGGL(KER<9>, grid, dim3(G::BLOCK), 0, stream, __VA_ARGS__);   \
      } break;                                                                               \
      case 10: {                                                                             \
        using G = Geo<10>;                                                                   \
        dim3 grid(unsigned((nframes + G::FPB - 1) / G::FPB));                                \
        if (grid.x) hipLaunchKernelGGL(KER<10>, grid, dim3(G::BLOCK), 0, stream, __VA_ARGS__);  \
      } break;                                                                               \
      case 11: {                                                                             \
        using G = Geo<11>;                                                                   \
        dim3 grid(unsigned((nframes + G::FPB - 1) / G::FPB));                                \
        if (grid.x) hipLaunchKernelGGL(KER<11>, grid, dim3(G::BLOCK), 0, stream, __VA_ARGS__);  \
      } break;                                                                               \
      default:                                                                               \
        ::sel::set_error("unsupported log2(n_fft)=%d", logn);                                \
        return SEL_ERR_UNSUPPORTED;                                                          \
    }                                                                                        \
    SEL_LAUNCH_CHECK();                                                                      \
  } while (0)

int frames_per_block(int logn) {
  switch (logn) {
    case 8: return Geo<8>::FPB;
    case 9: return Geo<9>::FPB;
    case 10: return Geo<10>::FPB;
    default: return Geo<11>::FPB;
  }
}

int64_t n_blocks(int logn, int64_t nframes) {
  const int fpb = frames_per_block(logn);
  return (nframes + fpb - 1) / fpb;
}

int ola(const float* slab, const FrameArgs& a, float* gx, hipStream_t s) {
  if (a.B == 0) return SEL_OK;
  dim3 grid(unsigned((a.T + 255) / 256), unsigned(a.B));
  hipLaunchKernelGGL(k_ola_fold, grid, dim3(256), 0, s, slab, a, gx);
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

size_t slab_bytes(int64_t B, int64_t T, int hop, int win) {
  return size_t(B) * size_t(1 + T / hop) * size_t(win) * sizeof(float);
}

constexpr int kReduceBlocks = 1024;

}  // namespace

extern "C" {

int sel_stft_mag_fwd(const float* x, int64_t B, int64_t T, int n_fft, int hop, int win_length,
                     const float* window, float pow_floor, float* mag, sel_stream_t stream) {
  int logn;
  if (int rc = check_frame(B, T, n_fft, hop, win_length, logn)) return rc;
  const FrameArgs a = frame_args(B, T, n_fft, hop, win_length);
  const int64_t nf = B * a.F;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  SEL_FRAME_DISPATCH(logn, nf, s, k_stft_mag_fwd, x, a, window, pow_floor, mag);
  return SEL_OK;
}

size_t sel_stft_bwd_workspace(int64_t B, int64_t T, int n_fft, int hop, int win_length) {
  (void)n_fft;
  return slab_bytes(B, T, hop, win_length);
}

int sel_stft_mag_bwd(const float* x, int64_t B, int64_t T, int n_fft, int hop, int win_length,
                     const float* window, float pow_floor, const float* g_mag, float* g_x, void* ws,
                     size_t ws_bytes, sel_stream_t stream) {
  int logn;
  if (int rc = check_frame(B, T, n_fft, hop, win_length, logn)) return rc;
  SEL_REQUIRE(ws_bytes >= slab_bytes(B, T, hop, win_length), SEL_ERR_WORKSPACE, "workspace too small");
  const FrameArgs a = frame_args(B, T, n_fft, hop, win_length);
  const int64_t nf = B * a.F;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  float* slab = static_cast<float*>(ws);
  SEL_FRAME_DISPATCH(logn, nf, s, k_stft_mag_bwd, x, a, window, pow_floor, g_mag, slab);
  return ola(slab, a, g_x, s);
}

size_t sel_mag_pair_workspace(int64_t n) {
  (void)n;
  return size_t(kReduceBlocks) * 3 * sizeof(double);
}

int sel_mag_pair_sums(const float* x_mag, const float* y_mag, int64_t n, double* sums, void* ws,
                      size_t ws_bytes, sel_stream_t stream) {
  SEL_REQUIRE(n > 0, SEL_ERR_ARG, "empty magnitude tensors");
  SEL_REQUIRE(ws_bytes >= sel_mag_pair_workspace(n), SEL_ERR_WORKSPACE, "workspace too small");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int nb = int(std::min<int64_t>(kReduceBlocks, (n + 255) / 256));
  double* part = static_cast<double*>(ws);
  hipLaunchKernelGGL(k_mag_pair_partials, dim3(nb), dim3(256), 0, s, x_mag, y_mag, n, part);
  SEL_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_finish_partials, dim3(1), dim3(256), 0, s, part, nb, 3, sums, nullptr, 0.0);
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

int sel_mag_pair_bwd(const float* x_mag, const float* y_mag, int64_t n, const float* coef,
                     float* g_x, float* g_y, sel_stream_t stream) {
  SEL_REQUIRE(n > 0, SEL_ERR_ARG, "empty magnitude tensors");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int nb = int(std::min<int64_t>(4096, (n + 255) / 256));
  hipLaunchKernelGGL(k_mag_pair_bwd, dim3(nb), dim3(256), 0, s, x_mag, y_mag, n, coef, g_x, g_y);
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

size_t sel_stft_loss_workspace(int64_t B, int64_t T, int n_fft, int hop, int win_length) {
  int logn = 0;
  while ((1 << logn) < n_fft) ++logn;
  if (logn < kMinLog || logn > kMaxLog - 1) return 0;
  const int64_t nf = B * (1 + T / hop);
  const size_t part = size_t(n_blocks(logn, nf)) * 3 * sizeof(double);
  const size_t slab = slab_bytes(B, T, hop, win_length);
  return part > slab ? part : slab;
}

int sel_stft_loss_fwd(const float* x, const float* y, int64_t B, int64_t T, int n_fft, int hop,
                      int win_length, const float* window, double* sums, void* ws, size_t ws_bytes,
                      sel_stream_t stream) {
  int logn;
  if (int rc = check_frame(B, T, n_fft, hop, win_length, logn)) return rc;
  SEL_REQUIRE(B > 0, SEL_ERR_ARG, "empty batch");
  SEL_REQUIRE(ws_bytes >= sel_stft_loss_workspace(B, T, n_fft, hop, win_length), SEL_ERR_WORKSPACE,
              "workspace too small");
  const FrameArgs a = frame_args(B, T, n_fft, hop, win_length);
  const int64_t nf = B * a.F;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  double* part = static_cast<double*>(ws);
  SEL_FRAME_DISPATCH(logn, nf, s, k_stft_loss_fwd, x, y, a, window, 1e-7f, part);
  const int nb = int(n_blocks(logn, nf));
  hipLaunchKernelGGL(k_finish_partials, dim3(1), dim3(256), 0, s, part, nb, 3, sums, nullptr, 0.0);
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

int sel_stft_loss_bwd(const float* x, const float* y, int64_t B, int64_t T, int n_fft, int hop,
                      int win_length, const float* window, const float* coef, float* g_x, void* ws,
                      size_t ws_bytes, sel_stream_t stream) {
  int logn;
  if (int rc = check_frame(B, T, n_fft, hop, win_length, logn)) return rc;
  SEL_REQUIRE(ws_bytes >= slab_bytes(B, T, hop, win_length), SEL_ERR_WORKSPACE, "workspace too small");
  const FrameArgs a = frame_args(B, T, n_fft, hop, win_length);
  const int64_t nf = B * a.F;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  float* slab = static_cast<float*>(ws);
  SEL_FRAME_DISPATCH(logn, nf, s, k_stft_loss_bwd, x, y, a, window, 1e-7f, coef, slab);
  return ola(slab, a, g_x, s);
}

int sel_stft_loss_finish(const double* sums, int64_t n, float* out2, sel_stream_t stream) {
  SEL_REQUIRE(n > 0, SEL_ERR_ARG, "n must be > 0");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(k_stft_loss_finish, dim3(1), dim3(1), 0, s, sums, 1.0 / double(n), out2);
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

int sel_stft_loss_coef(const double* sums, int64_t n, const float* g_sc, const float* g_mag,
                       float* coef, sel_stream_t stream) {
  SEL_REQUIRE(n > 0, SEL_ERR_ARG, "n must be > 0");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(k_stft_loss_coef, dim3(1), dim3(1), 0, s, sums, 1.0 / double(n), g_sc, g_mag,
                     coef);
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

int sel_logmel_fwd(const float* x, int64_t B, int64_t T, int n_fft, int hop, int win_length,
                   const float* window, const float* melmat, const int32_t* krange, int n_mels,
                   float eps, int log_kind, float* out, sel_stream_t stream) {
  int logn;
  if (int rc = check_frame(B, T, n_fft, hop, win_length, logn)) return rc;
  SEL_REQUIRE(n_mels > 0, SEL_ERR_ARG, "n_mels must be > 0");
  SEL_REQUIRE(log_kind >= SEL_LOG_E && log_kind <= SEL_LOG_10, SEL_ERR_ARG, "bad log kind");
  const FrameArgs a = frame_args(B, T, n_fft, hop, win_length);
  MelArgs ma{melmat, reinterpret_cast<const int2*>(krange), n_mels, eps, log_kind};
  const int64_t nf = B * a.F;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  SEL_FRAME_DISPATCH(logn, nf, s, k_logmel_fwd, x, a, window, ma, out);
  return SEL_OK;
}

size_t sel_l1_workspace(int64_t n) {
  (void)n;
  return size_t(kReduceBlocks) * sizeof(double);
}

int sel_l1_mean(const float* a, const float* b, int64_t n, float* out, void* ws, size_t ws_bytes,
                sel_stream_t stream) {
  SEL_REQUIRE(n > 0, SEL_ERR_ARG, "empty tensors");
  SEL_REQUIRE(ws_bytes >= sel_l1_workspace(n), SEL_ERR_WORKSPACE, "workspace too small");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int nb = int(std::min<int64_t>(kReduceBlocks, (n + 255) / 256));
  double* part = static_cast<double*>(ws);
  hipLaunchKernelGGL(k_abs_diff_partials, dim3(nb), dim3(256), 0, s, a, b, n, part);
  SEL_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_finish_partials, dim3(1), dim3(256), 0, s, part, nb, 1, nullptr, out,
                     1.0 / double(n));
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

size_t sel_logmel_bwd_workspace(int64_t B, int64_t T, int n_fft, int hop, int win_length) {
  (void)n_fft;
  return slab_bytes(B, T, hop, win_length);
}

int sel_logmel_bwd(const float* x, int64_t B, int64_t T, int n_fft, int hop, int win_length,
                   const float* window, const float* melmat, const int32_t* krange,
                   const int32_t* mrange, int n_mels, float eps, int log_kind, const float* g_out,
                   const float* ref, const float* g_scale, float g_mul, float* g_x, void* ws,
                   size_t ws_bytes, sel_stream_t stream) {
  int logn;
  if (int rc = check_frame(B, T, n_fft, hop, win_length, logn)) return rc;
  SEL_REQUIRE(n_mels > 0 && n_mels <= n_fft / 2 + 12, SEL_ERR_UNSUPPORTED,
              "n_mels=%d must be in (0, n_fft/2 + 12]", n_mels);
  SEL_REQUIRE(log_kind >= SEL_LOG_E && log_kind <= SEL_LOG_10, SEL_ERR_ARG, "bad log kind");
  SEL_REQUIRE(ws_bytes >= slab_bytes(B, T, hop, win_length), SEL_ERR_WORKSPACE, "workspace too small");
  SEL_REQUIRE(ref == nullptr || g_scale != nullptr, SEL_ERR_ARG, "g_scale required with ref");
  const FrameArgs a = frame_args(B, T, n_fft, hop, win_length);
  MelArgs ma{melmat, reinterpret_cast<const int2*>(mrange), n_mels, eps, log_kind};
  const int64_t nf = B * a.F;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  float* slab = static_cast<float*>(ws);
  SEL_FRAME_DISPATCH(logn, nf, s, k_logmel_bwd, x, a, window, ma,
                     reinterpret_cast<const int2*>(krange), g_out, ref, g_scale, g_mul, slab);
  return ola(slab, a, g_x, s);
}

}  // extern "C"
