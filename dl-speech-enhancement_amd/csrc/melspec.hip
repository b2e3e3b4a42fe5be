// Power-mel spectrogram of mel_spectrogram.py:38-44 (the eval Mel-L1 metric):
// torchaudio MelSpectrogram(48000) defaults — n_fft 400, hop 200, periodic Hann,
// center/reflect, onesided, spec = |X|^power (power 2), HTK filterbank without
// norm (the (K, n_mels) filterbank comes from the host), out (B, n_mels, F).
//
// n_fft = 400 is not a power of two, so this file carries its own mixed-radix
// FFT: a half-size (M = n_fft/2) complex Stockham autosort with radix-4/2/3/5
// passes in LDS, one wavefront per frame (4 frames per 256-lane workgroup),
// twiddles from sincospif.  Real split and the sparse mel projection (each
// filter only touches its nonzero bin range) follow in the same kernel; the
// block's 4 consecutive frames are written as one 16-B vector per mel row.
#include <cmath>

#include "sel_common.h"

namespace sel {
namespace melspec {

constexpr int FPB = 4;        // frames per block (one wave each)
constexpr int THREADS = 256;
constexpr int MAXM = 512;     // max half-size (n_fft <= 1024)
constexpr int MAXPASS = 12;

struct Plan {
  int M, npass;
  int radix[MAXPASS];
};

struct Args {
  int64_t B, T;
  int F, hop, win, left, P;  // P = n_fft / 2 reflect pad; left = window offset in the frame
  int n_mels;
  float power;
};

__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ float2 cmni(float2 a) { return make_float2(a.y, -a.x); }  // * -i
__device__ __forceinline__ float2 cis(float turns) {  // exp(2 pi i * turns)
  float s, c;
  sincospif(2.f * turns, &s, &c);
  return make_float2(c, s);
}

__device__ __forceinline__ int64_t reflect_index(int64_t j, int64_t T) {
  j = j < 0 ? -j : j;
  j = j >= T ? 2 * (T - 1) - j : j;
  return j;
}

// In-place small DFTs (forward, e^{-2 pi i nk/R}).
__device__ __forceinline__ void dft2(float2* v) {
  const float2 a = v[0], b = v[1];
  v[0] = cadd(a, b);
  v[1] = csub(a, b);
}
__device__ __forceinline__ void dft4(float2* v) {
  const float2 t0 = cadd(v[0], v[2]), t1 = csub(v[0], v[2]), t2 = cadd(v[1], v[3]), t3 = cmni(csub(v[1], v[3]));
  v[0] = cadd(t0, t2);
  v[1] = cadd(t1, t3);
  v[2] = csub(t0, t2);
  v[3] = csub(t1, t3);
}
__device__ __forceinline__ void dft3(float2* v) {
  const float c = -0.5f, s = -0.86602540378443864676f;  // cos/sin(-2pi/3)
  const float2 a = v[0], b = v[1], d = v[2];
  const float2 sum = cadd(b, d), dif = csub(b, d);
  v[0] = cadd(a, sum);
  const float2 m = make_float2(a.x + c * sum.x, a.y + c * sum.y);
  const float2 r = make_float2(-s * dif.y, s * dif.x);  // i*s*dif
  v[1] = cadd(m, r);
  v[2] = csub(m, r);
}
__device__ __forceinline__ void dft5(float2* v) {
  const float c1 = 0.30901699437494742410f, c2 = -0.80901699437494742410f;   // cos(2pi/5), cos(4pi/5)
  const float s1 = 0.95105651629515357212f, s2 = 0.58778525229247312917f;    // sin(2pi/5), sin(4pi/5)
  const float2 a = v[0];
  const float2 p1 = cadd(v[1], v[4]), m1 = csub(v[1], v[4]);
  const float2 p2 = cadd(v[2], v[3]), m2 = csub(v[2], v[3]);
  v[0] = cadd(a, cadd(p1, p2));
  const float2 r1 = make_float2(a.x + c1 * p1.x + c2 * p2.x, a.y + c1 * p1.y + c2 * p2.y);
  const float2 r2 = make_float2(a.x + c2 * p1.x + c1 * p2.x, a.y + c2 * p1.y + c1 * p2.y);
  // forward transform: -i * (s1*m1 + s2*m2) and -i * (s2*m1 - s1*m2)
  const float2 q1 = make_float2(s1 * m1.x + s2 * m2.x, s1 * m1.y + s2 * m2.y);
  const float2 q2 = make_float2(s2 * m1.x - s1 * m2.x, s2 * m1.y - s1 * m2.y);
  v[1] = cadd(r1, cmni(q1));
  v[4] = csub(r1, cmni(q1));
  v[2] = cadd(r2, cmni(q2));
  v[3] = csub(r2, cmni(q2));
}

template <int R>
__device__ __forceinline__ void stockham_pass(const float2* src, float2* dst, int M, int Ns, int lane) {
  const int nb = M / R;
  for (int j = lane; j < nb; j += 64) {
    const int k = j % Ns;
    float2 v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      v[r] = src[j + r * nb];
      if (r > 0 && Ns > 1) v[r] = cmul(v[r], cis(-float(k * r) / float(Ns * R)));
    }
    if constexpr (R == 2) dft2(v);
    if constexpr (R == 3) dft3(v);
    if constexpr (R == 4) dft4(v);
    if constexpr (R == 5) dft5(v);
    const int d = (j / Ns) * Ns * R + k;
#pragma unroll
    for (int r = 0; r < R; ++r) dst[d + r * Ns] = v[r];
  }
}

__global__ __launch_bounds__(THREADS) void k_power_mel_fwd(const float* __restrict__ x, Args a, Plan plan,
                                                           const float* __restrict__ window,
                                                           const float* __restrict__ fb,
                                                           const int32_t* __restrict__ krange,
                                                           float* __restrict__ out) {
  __shared__ float2 lds[FPB][2][MAXM + 8];
  __shared__ float spec[FPB][MAXM + 8];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int M = plan.M, N = 2 * M, K = M + 1;
  // the block owns frames [f0, f0 + FPB) of one signal
  const int fpb_per_sig = (a.F + FPB - 1) / FPB;
  const int64_t b = blockIdx.x / fpb_per_sig;
  const int f0 = int(blockIdx.x % fpb_per_sig) * FPB;
  const int f = f0 + w;
  const bool active = f < a.F;
  const float* xs = x + b * a.T;
  float2* src = lds[w][0];
  float2* dst = lds[w][1];

  // load: windowed, reflect-padded samples packed two per complex point
  const int64_t base = int64_t(f) * a.hop - a.P;
  for (int m = lane; m < M; m += 64) {
    float v0 = 0.f, v1 = 0.f;
    if (active) {
      const int w0 = 2 * m - a.left, w1 = w0 + 1;
      if (w0 >= 0 && w0 < a.win) v0 = window[w0] * xs[reflect_index(base + 2 * m, a.T)];
      if (w1 >= 0 && w1 < a.win) v1 = window[w1] * xs[reflect_index(base + 2 * m + 1, a.T)];
    }
    src[m] = make_float2(v0, v1);
  }
  __syncthreads();
  // mixed-radix Stockham (each wave owns its frame: wave-local barriers suffice,
  // but the LDS buffers are block-visible, so keep block barriers for clarity)
  int Ns = 1;
  for (int p = 0; p < plan.npass; ++p) {
    const int R = plan.radix[p];
    if (R == 4) stockham_pass<4>(src, dst, M, Ns, lane);
    else if (R == 2) stockham_pass<2>(src, dst, M, Ns, lane);
    else if (R == 5) stockham_pass<5>(src, dst, M, Ns, lane);
    else stockham_pass<3>(src, dst, M, Ns, lane);
    __syncthreads();
    float2* t = src;
    src = dst;
    dst = t;
    Ns *= R;
  }
  // real split -> |X_k|^power for k = 0..M
  for (int k = lane; k <= M; k += 64) {
    float2 X;
    if (k == 0 || k == M) {
      const float2 z0 = src[0];
      X = make_float2(k == 0 ? z0.x + z0.y : z0.x - z0.y, 0.f);
    } else {
      const float2 zk = src[k], zm = src[M - k];
      const float2 e = make_float2(0.5f * (zk.x + zm.x), 0.5f * (zk.y - zm.y));
      const float2 o = make_float2(0.5f * (zk.y + zm.y), -0.5f * (zk.x - zm.x));
      X = cadd(e, cmul(cis(-float(k) / float(N)), o));
    }
    const float mag = sqrtf(X.x * X.x + X.y * X.y);  // torch: spec.abs().pow(power)
    spec[w][k] = a.power == 2.f ? mag * mag : (a.power == 1.f ? mag : powf(mag, a.power));
  }
  __syncthreads();
  // sparse mel projection: thread -> (mel row, frame-in-block); vector store of the block's frames
  float4* o4 = reinterpret_cast<float4*>(out);
  for (int m = threadIdx.x; m < a.n_mels; m += THREADS) {
    const int lo = krange[2 * m], hi = krange[2 * m + 1];
    float acc[FPB] = {0.f, 0.f, 0.f, 0.f};
    for (int k = lo; k < hi; ++k) {
      const float wgt = fb[int64_t(k) * a.n_mels + m];
#pragma unroll
      for (int q = 0; q < FPB; ++q) acc[q] = fmaf(spec[q][k], wgt, acc[q]);
    }
    float* row = out + (b * a.n_mels + m) * a.F + f0;
    const bool vec = (f0 + FPB <= a.F) && ((reinterpret_cast<uintptr_t>(row) & 15) == 0);
    if (vec) {
      o4[(row - out) / 4] = make_float4(acc[0], acc[1], acc[2], acc[3]);
    } else {
#pragma unroll
      for (int q = 0; q < FPB; ++q)
        if (f0 + q < a.F) row[q] = acc[q];
    }
  }
  (void)K;
}

static bool make_plan(int M, Plan& p) {
  p.M = M;
  p.npass = 0;
  int r = M;
  while (r % 4 == 0 && p.npass < MAXPASS) { p.radix[p.npass++] = 4; r /= 4; }
  while (r % 2 == 0 && p.npass < MAXPASS) { p.radix[p.npass++] = 2; r /= 2; }
  while (r % 5 == 0 && p.npass < MAXPASS) { p.radix[p.npass++] = 5; r /= 5; }
  while (r % 3 == 0 && p.npass < MAXPASS) { p.radix[p.npass++] = 3; r /= 3; }
  return r == 1;
}

}  // namespace melspec
}  // namespace sel

using namespace sel;
using namespace sel::melspec;

extern "C" {

int sel_power_mel_fwd(const float* x, int64_t B, int64_t T, int n_fft, int hop, int win_length,
                      const float* window, const float* fb, const int32_t* krange, int n_mels, float power,
                      float* out, sel_stream_t stream) {
  SEL_REQUIRE(initialized(), SEL_ERR_STATE, "sel_init() not called");
  SEL_REQUIRE(x && window && fb && krange && out, SEL_ERR_ARG, "null pointer");
  SEL_REQUIRE(B > 0 && T > 0 && hop > 0 && n_mels > 0, SEL_ERR_ARG, "bad sizes");
  SEL_REQUIRE(n_fft >= 8 && n_fft % 2 == 0 && n_fft / 2 <= MAXM, SEL_ERR_UNSUPPORTED,
              "n_fft %d: need an even size <= %d", n_fft, 2 * MAXM);
  SEL_REQUIRE(win_length > 0 && win_length <= n_fft, SEL_ERR_ARG, "win_length %d > n_fft %d", win_length, n_fft);
  SEL_REQUIRE(T > n_fft / 2, SEL_ERR_ARG, "reflect pad %d needs T > pad (T=%lld)", n_fft / 2, (long long)T);
  SEL_REQUIRE(power > 0.f, SEL_ERR_UNSUPPORTED, "power must be > 0 (None = complex output not supported)");
  Plan plan;
  SEL_REQUIRE(make_plan(n_fft / 2, plan), SEL_ERR_UNSUPPORTED, "n_fft/2 = %d has prime factors other than 2,3,5",
              n_fft / 2);
  Args a;
  a.B = B;
  a.T = T;
  a.F = int(1 + T / hop);
  a.hop = hop;
  a.win = win_length;
  a.left = (n_fft - win_length) / 2;
  a.P = n_fft / 2;
  a.n_mels = n_mels;
  a.power = power;
  const int64_t blocks = B * ((a.F + FPB - 1) / FPB);
  SEL_REQUIRE(blocks < (int64_t(1) << 31), SEL_ERR_ARG, "batch too large");
  hipLaunchKernelGGL(k_power_mel_fwd, dim3(unsigned(blocks)), dim3(THREADS), 0,
                     reinterpret_cast<hipStream_t>(stream), x, a, plan, window, fb, krange, out);
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

}  // extern "C"
