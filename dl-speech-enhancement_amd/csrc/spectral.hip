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

__constant__ float2 g_tw[kTwTotal];  // constant address space: lane-uniform reads are scalar loads

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

// Wave-FFT geometry: a frame is owned by LPF = M/8 lanes (8 points per lane):
// a quarter / half / whole wave for n_fft 256 / 512 / 1024, so those
// transforms run without a block barrier, and two waves (s_barrier between
// passes) for 2048.  A 256-lane block holds FPB = 256/LPF frames per
// iteration and walks `iters` consecutive frame groups (window and twiddles
// stay in registers across them).
// LDS padding of a frame's complex slots: one pad slot per 2^SEL_PSH
#ifndef SEL_PSH
#define SEL_PSH 4
#endif

template <int LOGN>
struct Geo {
  static constexpr int N = 1 << LOGN;
  static constexpr int M = N / 2;
  static constexpr int PPL = fft_ppl(LOGN);  // complex points per lane
  static constexpr int LPF = M / PPL;         // lanes per frame
  static constexpr int FPB = 256 / LPF;       // frames per block iteration
  static constexpr int BLOCK = 256;
  static constexpr int NP = fft_npass(LOGN);
  static constexpr int R0 = fft_radix(LOGN, 0), R1 = fft_radix(LOGN, 1), R2 = fft_radix(LOGN, 2),
                       R3 = fft_radix(LOGN, 3);
  static constexpr int NS1 = R0, NS2 = R0 * R1, NS3 = R0 * R1 * R2;
  // complex slots per frame: M padded by pidx, + a spare slot (G_M in c2r_grad)
  static constexpr int PADN = M + (M >> SEL_PSH) + 2;
  static_assert(R0 * R1 * R2 * R3 == M && PPL == 8 && LPF <= 256, "wave FFT schedule");
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

// one pad slot per 8 complex values: the radix-8/16 Stockham stores (a lane's 8
// or 16 outputs contiguous, lanes 64-128 B apart) spread over all 64 banks
__device__ __forceinline__ int pidx(int i) { return i + (i >> SEL_PSH); }
// pidx(i + c) = pidx(i) + padc(c) whenever c is a multiple of 2^SEL_PSH
__host__ __device__ constexpr int padc(int c) { return c + (c >> SEL_PSH); }
// pidx(l + c) from pl = pidx(l): linear (an immediate offset) when the unrolled c allows it
__device__ __forceinline__ int padd(int pl, int l, int c) {
  return (c & ((1 << SEL_PSH) - 1)) == 0 ? pl + padc(c) : pidx(l + c);
}

// orders this lane's LDS accesses around cross-lane exchanges inside the wave
// (DS instructions of one wave execute in order; this stops the compiler from
// moving them across the exchange point)
__device__ __forceinline__ void wave_lds_fence() {
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

// exchange point of one frame's lanes: in-wave fence, or a block barrier when
// the frame spans two waves (n_fft 2048)
template <int LOGN>
__device__ __forceinline__ void frame_fence() {
  if constexpr (Geo<LOGN>::LPF > 64) __syncthreads();
  else wave_lds_fence();
}

// ---- in-register DFTs (forward, exp(-2 pi i nk/R)), natural-order output ----
__device__ __forceinline__ void dft2(float2& a0, float2& a1) {
  const float2 t = a0;
  a0 = cadd(t, a1);
  a1 = csub(t, a1);
}
__device__ __forceinline__ void dft4(float2& a0, float2& a1, float2& a2, float2& a3) {
  const float2 t0 = cadd(a0, a2), t1 = csub(a0, a2), t2 = cadd(a1, a3), t3 = cmni(csub(a1, a3));
  a0 = cadd(t0, t2);
  a1 = cadd(t1, t3);
  a2 = csub(t0, t2);
  a3 = csub(t1, t3);
}
constexpr float kS2 = 0.70710678118654752440f;  // sqrt(1/2)
constexpr float kC8 = 0.92387953251128675613f;  // cos(pi/8)
constexpr float kS8 = 0.38268343236508977173f;  // sin(pi/8)
// x * exp(-i pi/4), x * exp(-3i pi/4)
__device__ __forceinline__ float2 w8_1(float2 x) { return make_float2(kS2 * (x.x + x.y), kS2 * (x.y - x.x)); }
__device__ __forceinline__ float2 w8_3(float2 x) { return make_float2(kS2 * (x.y - x.x), -kS2 * (x.x + x.y)); }
__device__ __forceinline__ float2 cmulc(float2 x, float c, float s) {  // x * (c + i s)
  return make_float2(fmaf(x.x, c, -x.y * s), fmaf(x.x, s, x.y * c));
}

__device__ __forceinline__ void dft8(float2 (&a)[8]) {
  float2 b[4], c[4];
#pragma unroll
  for (int n = 0; n < 4; ++n) {
    b[n] = cadd(a[n], a[n + 4]);
    c[n] = csub(a[n], a[n + 4]);
  }
  c[1] = w8_1(c[1]);
  c[2] = cmni(c[2]);
  c[3] = w8_3(c[3]);
  dft4(b[0], b[1], b[2], b[3]);
  dft4(c[0], c[1], c[2], c[3]);
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    a[2 * m] = b[m];
    a[2 * m + 1] = c[m];
  }
}

__device__ __forceinline__ void dft16(float2 (&a)[16]) {
  float2 b[8], c[8];
#pragma unroll
  for (int n = 0; n < 8; ++n) {
    b[n] = cadd(a[n], a[n + 8]);
    c[n] = csub(a[n], a[n + 8]);
  }
  // c[n] *= exp(-2 pi i n / 16)
  c[1] = cmulc(c[1], kC8, -kS8);
  c[2] = w8_1(c[2]);
  c[3] = cmulc(c[3], kS8, -kC8);
  c[4] = cmni(c[4]);
  c[5] = cmulc(c[5], -kS8, -kC8);
  c[6] = w8_3(c[6]);
  c[7] = cmulc(c[7], -kC8, -kS8);
  dft8(b);
  dft8(c);
#pragma unroll
  for (int m = 0; m < 8; ++m) {
    a[2 * m] = b[m];
    a[2 * m + 1] = c[m];
  }
}

template <int R>
__device__ __forceinline__ void dft(float2 (&a)[R]) {
  if constexpr (R == 2) dft2(a[0], a[1]);
  else if constexpr (R == 4) dft4(a[0], a[1], a[2], a[3]);
  else if constexpr (R == 8) dft8(a);
  else dft16(a);
}

// Per-lane twiddles, loaded once per kernel: pass p's base twiddles
// W_{R*NS}^{r*(l mod NS)} (r = 1..R-1) and the split twiddle W_N^l.  A lane's
// other butterflies / bins differ by a lane-uniform factor read from the same
// tables (scalar loads): W^{r*(l + LPF*u mod NS)} = W^{r*l} * W^{r*(LPF*u mod NS)},
// W_N^{l + LPF*q} = W_N^l * W_N^{LPF*q}.
#ifndef SEL_SPLIT_TW_RES
#define SEL_SPLIT_TW_RES 1
#endif

template <int LOGN>
struct LaneTw {
  using G = Geo<LOGN>;
  // register-resident for PPL = 8; for PPL = 16 the pass twiddles are re-read
  // from the (L1-resident) table each frame, through a pointer made opaque per
  // use so the compiler cannot hoist them into registers it does not have
  static constexpr bool RES = G::PPL == 8;
  float2 p1[RES ? G::R1 - 1 : 1], p2[RES ? G::R2 - 1 : 1], p3[G::R3 > 1 ? G::R3 - 1 : 1], n;
  // W_N^{l + LPF*q} exactly rounded from the table, where a frame fits one wave
  // (at n_fft 2048 the 16 extra VGPRs cost a wave of occupancy: factorised)
  static constexpr bool NQ = SEL_SPLIT_TW_RES && G::LPF <= 64;
  float2 nq[NQ ? G::PPL : 1];
  const float2* g1;
  const float2* g2;
  // table offsets as constants (the recursive constexpr helpers are otherwise
  // emitted as device calls in the prologue)
  static constexpr int OFF1 = twp_off(LOGN, 1), OFF2 = twp_off(LOGN, 2), OFF3 = twp_off(LOGN, 3),
                       OFFN = tw_off(LOGN) + G::M;
  __device__ __forceinline__ void load(int l) {
    g1 = g_tw + OFF1 + (l & (G::NS1 - 1)) * (G::R1 - 1);
    g2 = g_tw + OFF2 + (l & (G::NS2 - 1)) * (G::R2 - 1);
    if constexpr (RES) {
#pragma unroll
      for (int r = 1; r < G::R1; ++r) p1[r - 1] = g1[r - 1];
#pragma unroll
      for (int r = 1; r < G::R2; ++r) p2[r - 1] = g2[r - 1];
    }
    if constexpr (G::R3 > 1) {
#pragma unroll
      for (int r = 1; r < G::R3; ++r) p3[r - 1] = g_tw[OFF3 + (l & (G::NS3 - 1)) * (G::R3 - 1) + r - 1];
    }
    n = g_tw[OFFN + l];
    if constexpr (NQ) {
#pragma unroll
      for (int q = 0; q < G::PPL; ++q) nq[q] = g_tw[OFFN + l + G::LPF * q];
    }
  }
  __device__ __forceinline__ const float2* t1() const {
    if constexpr (RES) return p1;
    const float2* p = g1;
    asm volatile("" : "+v"(p));
    return p;
  }
  __device__ __forceinline__ const float2* t2() const {
    if constexpr (RES) return p2;
    const float2* p = g2;
    asm volatile("" : "+v"(p));
    return p;
  }
};

// W_N^k for this lane's bin k = l + LPF*q
template <int LOGN>
__device__ __forceinline__ float2 split_tw(const LaneTw<LOGN>& tw, int q) {
  using G = Geo<LOGN>;
  if constexpr (LaneTw<LOGN>::NQ) return tw.nq[q];
  else return q == 0 ? tw.n : cmul(tw.n, g_tw[tw_off(LOGN) + G::M + G::LPF * q]);
}

// One Stockham pass (radix R, stride NS) from registers to the frame's LDS
// buffer.  Lane l's points are q = u + r*NB <-> butterfly j = l + LPF*u,
// input j + r*M/R; output (j - j%NS)*R + j%NS + r*NS.
template <int LOGN, int R, int NS, int PASS>
__device__ __forceinline__ void fft_pass_store(float2 (&v)[Geo<LOGN>::PPL], float2* z, int l, const float2* twb) {
  using G = Geo<LOGN>;
  constexpr int NB = G::PPL / R;
#pragma unroll
  for (int u = 0; u < NB; ++u) {
    const int j = l + G::LPF * u;
    const int k = j & (NS - 1);
    float2 a[R];
#pragma unroll
    for (int r = 0; r < R; ++r) a[r] = v[u + r * NB];
    if constexpr (NS > 1) {
      const int kf = (G::LPF * u) & (NS - 1);  // lane-uniform part of k
#pragma unroll
      for (int r = 1; r < R; ++r) {
        float2 t = twb[r - 1];
        constexpr int OFFP = twp_off(LOGN, PASS);
        if (NS > G::LPF && u > 0) t = cmul(t, g_tw[OFFP + kf * (R - 1) + r - 1]);
        a[r] = cmul(a[r], t);
      }
    }
    dft<R>(a);
    // padded destination pidx(base + r*NS): linear in r when 2^PSH | NS; for
    // NS == 1, base = 8j and the r < 8 outputs stay inside one 8-slot run
    const int base = (j - k) * R + k;
    const int pb = pidx(base);
#pragma unroll
    for (int r = 0; r < R; ++r) z[NS == 1 ? pb + r : padd(pb, base, r * NS)] = a[r];
  }
}

template <int LOGN, int R>
__device__ __forceinline__ void fft_pass_load(float2 (&v)[Geo<LOGN>::PPL], const float2* z, int l) {
  using G = Geo<LOGN>;
  constexpr int NB = G::PPL / R;
  const int pl = pidx(l);
#pragma unroll
  for (int u = 0; u < NB; ++u)
#pragma unroll
    for (int r = 0; r < R; ++r) v[u + r * NB] = z[padd(pl, l, G::LPF * u + r * (G::M / R))];
}

// Half-size complex FFT of the frame whose points m = l + LPF*q sit in v[q]
// (q < PPL); leaves Z in natural order in z[pidx(.)].  Wave-local: no barrier.
template <int LOGN>
__device__ __forceinline__ void fft_half(float2 (&v)[Geo<LOGN>::PPL], float2* z, int l, const LaneTw<LOGN>& tw) {
  using G = Geo<LOGN>;
  fft_pass_store<LOGN, G::R0, 1, 0>(v, z, l, nullptr);
  frame_fence<LOGN>();
  fft_pass_load<LOGN, G::R1>(v, z, l);
  frame_fence<LOGN>();
  fft_pass_store<LOGN, G::R1, G::NS1, 1>(v, z, l, tw.t1());
  frame_fence<LOGN>();
  fft_pass_load<LOGN, G::R2>(v, z, l);
  frame_fence<LOGN>();
  fft_pass_store<LOGN, G::R2, G::NS2, 2>(v, z, l, tw.t2());
  frame_fence<LOGN>();
  if constexpr (G::NP == 4) {
    fft_pass_load<LOGN, G::R3>(v, z, l);
    frame_fence<LOGN>();
    fft_pass_store<LOGN, G::R3, G::NS3, 3>(v, z, l, tw.p3);
    frame_fence<LOGN>();
  }
}

// This lane's window pairs (w(2m - left), w(2m + 1 - left)), m = l + LPF*q:
// register-resident for PPL = 8, re-read per frame (L1 hits) for PPL = 16,
// whose FFT working set leaves no room for them.
template <int LOGN, bool RESIDENT = (Geo<LOGN>::PPL == 8)>
struct Win {
  using G = Geo<LOGN>;
  float2 w[RESIDENT ? G::PPL : 1];
  const float* __restrict__ win;
  int left, n, l;
  __device__ __forceinline__ float2 fetch(int q) const {
    const int w0 = 2 * (l + G::LPF * q) - left, w1 = w0 + 1;
    return make_float2(w0 >= 0 && w0 < n ? win[w0] : 0.f, w1 >= 0 && w1 < n ? win[w1] : 0.f);
  }
  __device__ __forceinline__ void init(const float* window, const FrameArgs& a, int l_) {
    win = window;
    left = a.left;
    n = a.win;
    l = l_;
    if constexpr (RESIDENT) {
#pragma unroll
      for (int q = 0; q < G::PPL; ++q) w[q] = fetch(q);
    }
  }
  __device__ __forceinline__ float2 get(int q) const {
    if constexpr (RESIDENT) return w[q];
    else return fetch(q);
  }
};

// Raw sample pairs (x[2m], x[2m+1]) of frame f of signal b, reflect-padded,
// m = l + LPF*q.  Interior frames: one coalesced 8-B load per point off one
// base address; edge frames: per-sample reflected loads through a buffer
// resource over the whole (B, T) batch (32-bit offsets, one VGPR per address;
// the host keeps B*T*4 < 2^31).  Issued one frame ahead
// of the transform that consumes them.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t signal_rsrc(const float* x, const FrameArgs& a) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(x), 0, int(a.B * a.T * 4), 0x00020000);
}

template <int LOGN>
__device__ __forceinline__ void fetch_frame(const float* __restrict__ x, __amdgpu_buffer_rsrc_t xr, const FrameArgs& a,
                                            int64_t b, int f, int l, bool active, float2 (&raw)[Geo<LOGN>::PPL]) {
  using G = Geo<LOGN>;
  const int T = int(a.T);
  const int base = f * a.hop - a.P;
  const int sig = int(b) * T;
  const float* xs = x + sig + base;
  if (active && base >= 0 && base + G::N <= T && (reinterpret_cast<uintptr_t>(xs) & 7) == 0) {
    // (raw_buffer_load_b64 returned wrong pairs here on gfx950: plain 8-B global loads)
    const float2* x2 = reinterpret_cast<const float2*>(xs) + l;
#pragma unroll
    for (int q = 0; q < G::PPL; ++q) raw[q] = x2[G::LPF * q];
  } else if (active) {
#pragma unroll
    for (int q = 0; q < G::PPL; ++q) {
      // reflect(j) = min(|j|, 2(T-1) - |j|) for -(T-1) <= j <= 2(T-1)
      int n0 = abs(base + 2 * (l + G::LPF * q)), n1 = abs(base + 2 * (l + G::LPF * q) + 1);
      n0 = min(n0, 2 * (T - 1) - n0);
      n1 = min(n1, 2 * (T - 1) - n1);
      raw[q] = make_float2(__builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, (sig + n0) * 4, 0, 0)),
                           __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, (sig + n1) * 4, 0, 0)));
    }
  } else {
#pragma unroll
    for (int q = 0; q < G::PPL; ++q) raw[q] = make_float2(0.f, 0.f);
  }
}

template <int LOGN>
__device__ __forceinline__ void window_frame(const float2 (&raw)[Geo<LOGN>::PPL], const Win<LOGN>& wn,
                                             float2 (&v)[Geo<LOGN>::PPL]) {
#pragma unroll
  for (int q = 0; q < Geo<LOGN>::PPL; ++q) {
    const float2 w = wn.get(q);
    v[q] = make_float2(raw[q].x * w.x, raw[q].y * w.y);
  }
}

// Real split: X_k for this lane's bins k = l + LPF*q (q < PPL) and X_M (valid on l == 0).
template <int LOGN>
__device__ __forceinline__ void real_split(const float2* z, int l, const LaneTw<LOGN>& tw, float2 (&X)[Geo<LOGN>::PPL],
                                           float2& XM) {
  using G = Geo<LOGN>;
  constexpr int M = G::M;
  // LDS addressing off two per-lane bases: pidx(l + c) = pidx(l) + padc(c) and
  // pidx(M - l - c) = pidx(-l) + padc(M - c) (bin 0 pairs with itself)
  const int pl = pidx(l), pn = pidx(-l);
#pragma unroll
  for (int q = 0; q < G::PPL; ++q) {
    const int c = M - G::LPF * q;
    const int im = q == 0 ? (l == 0 ? 0 : padd(pn, -l, M)) : padd(pn, -l, c);
    const float2 zk = z[padd(pl, l, G::LPF * q)], zm = z[im];
    const float2 e = make_float2(0.5f * (zk.x + zm.x), 0.5f * (zk.y - zm.y));
    const float2 o = make_float2(0.5f * (zk.y + zm.y), -0.5f * (zk.x - zm.x));
    X[q] = cadd(e, cmul(split_tw<LOGN>(tw, q), o));  // k = 0: e + o = (z0.x + z0.y, 0)
    if (q == 0) XM = make_float2(zk.x - zk.y, 0.f);  // meaningful for k = 0 only
  }
  frame_fence<LOGN>();
}

// |X|^2 for bin pairs (forward-only epilogues): lane l's bins k = l + LPF*q and
// M - k (q < PPL/2) share zk, zm and one twiddle product, since
// X_{M-k} = conj(e_k - W^k o_k) while X_k = e_k + W^k o_k; p[q] <- |X_k|^2,
// p[PPL/2 + q] <- |X_{M-k}|^2 (k = 0 pairs with the Nyquist bin M), and pmid <-
// |X_{M/2}|^2 = |Z_{M/2}|^2 (valid on l == 0).
// |X_k|^2 and |X_{M-k}|^2 of one bin pair from Z_k, Z_{M-k} and W_N^k
__device__ __forceinline__ void pair_power(float2 zk, float2 zm, float2 w, float& pk, float& pm) {
  const float ex = zk.x + zm.x, ey = zk.y - zm.y;  // 2 e_k
  const float ox = zk.y + zm.y, oy = zm.x - zk.x;  // 2 o_k
  const float wox = w.x * ox - w.y * oy, woy = w.x * oy + w.y * ox;
  const float ax = ex + wox, ay = ey + woy, bx = ex - wox, by = ey - woy;
  pk = 0.25f * (ax * ax + ay * ay);
  pm = 0.25f * (bx * bx + by * by);
}

template <int LOGN>
__device__ __forceinline__ void split_pairs(const float2* z, int l, const LaneTw<LOGN>& tw,
                                            float (&p)[Geo<LOGN>::PPL], float& pmid) {
  using G = Geo<LOGN>;
  constexpr int M = G::M, H = G::PPL / 2;
  const int pl = pidx(l), pn = pidx(-l);
#pragma unroll
  for (int q = 0; q < H; ++q) {
    const int im = q == 0 ? (l == 0 ? 0 : padd(pn, -l, M)) : padd(pn, -l, M - G::LPF * q);
    pair_power(z[padd(pl, l, G::LPF * q)], z[im], split_tw<LOGN>(tw, q), p[q], p[H + q]);
  }
  const float2 zc = z[pidx(M / 2)];
  pmid = zc.x * zc.x + zc.y * zc.y;
  frame_fence<LOGN>();
}

// The last Stockham pass in registers: the same butterflies as
// fft_pass_store, written back to v in place (the pass's input point q = u +
// r*NB and output r of butterfly u share a register), so for the final pass
// (NS = M/R, j < NS) v[m] = Z[l + LPF*m].
template <int LOGN, int R, int NS, int PASS>
__device__ __forceinline__ void fft_pass_reg(float2 (&v)[Geo<LOGN>::PPL], int l, const float2* twb) {
  using G = Geo<LOGN>;
  constexpr int NB = G::PPL / R;
  static_assert(NS * R == G::M && NS >= G::LPF * NB, "final pass: j < NS");
#pragma unroll
  for (int u = 0; u < NB; ++u) {
    float2 a[R];
#pragma unroll
    for (int r = 0; r < R; ++r) a[r] = v[u + r * NB];
    const int kf = (G::LPF * u) & (NS - 1);
#pragma unroll
    for (int r = 1; r < R; ++r) {
      float2 t = twb[r - 1];
      constexpr int OFFP = twp_off(LOGN, PASS);
      if (NS > G::LPF && u > 0) t = cmul(t, g_tw[OFFP + kf * (R - 1) + r - 1]);
      a[r] = cmul(a[r], t);
    }
    dft<R>(a);
#pragma unroll
    for (int r = 0; r < R; ++r) v[u + r * NB] = a[r];
  }
}

__device__ __forceinline__ float2 bpermute2(int addr, float2 x) {
  return make_float2(__builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(addr, __builtin_bit_cast(int, x.x))),
                     __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(addr, __builtin_bit_cast(int, x.y))));
}

// FFT + bin-pair powers (split_pairs' outputs).  Where a frame fits one wave the
// last pass stays in registers: lane l's Z_{l+LPF m} pairs with Z_{M-l-LPF m},
// register 7 - m of lane LPF - l (lane 0: its own register (8 - m) mod 8), so 8
// ds_bpermute replace the last pass's LDS store and the pair reads.
#ifndef SEL_FFT_REGPAIRS
#define SEL_FFT_REGPAIRS 1
#endif
// REG = false keeps the LDS form (the fused loss forward: +16 VGPRs past the
// 4-wave budget with two spectra live, measured 195 -> 203 us at B = 512)
template <int LOGN, bool REG = true>
__device__ __forceinline__ void fft_pairs(float2 (&v)[Geo<LOGN>::PPL], float2* z, int l, const LaneTw<LOGN>& tw,
                                          float (&p)[Geo<LOGN>::PPL], float& pmid) {
  using G = Geo<LOGN>;
  if constexpr (SEL_FFT_REGPAIRS && REG && G::LPF <= 64 && G::NP == 3 && G::PPL == 8) {
    constexpr int H = G::PPL / 2;
    fft_pass_store<LOGN, G::R0, 1, 0>(v, z, l, nullptr);
    frame_fence<LOGN>();
    fft_pass_load<LOGN, G::R1>(v, z, l);
    frame_fence<LOGN>();
    fft_pass_store<LOGN, G::R1, G::NS1, 1>(v, z, l, tw.t1());
    frame_fence<LOGN>();
    fft_pass_load<LOGN, G::R2>(v, z, l);
    frame_fence<LOGN>();
    fft_pass_reg<LOGN, G::R2, G::NS2, 2>(v, l, tw.t2());
    const int lane = int(threadIdx.x % 64);
    const int addr = 4 * (lane - l + ((G::LPF - l) & (G::LPF - 1)));
#pragma unroll
    for (int q = 0; q < H; ++q) {
      const float2 pm = bpermute2(addr, v[7 - q]);
      const float2 zm = l == 0 ? v[(8 - q) & 7] : pm;
      pair_power(v[q], zm, split_tw<LOGN>(tw, q), p[q], p[H + q]);
    }
    pmid = v[4].x * v[4].x + v[4].y * v[4].y;
  } else {
    fft_half<LOGN>(v, z, l, tw);
    split_pairs<LOGN>(z, l, tw, p, pmid);
  }
}

// Gradient through real_split + FFT: given G_k for this lane's bins (Gq[q],
// k = l + LPF*q) and G_M (GM, on l == 0), r_n = Re sum_{k=0}^{M} G_k exp(+2 pi i k n / N)
// for this lane's points: out[q] = (r[2m], r[2m+1]), m = l + LPF*q.
template <int LOGN>
__device__ __forceinline__ void c2r_grad(float2 (&Gq)[Geo<LOGN>::PPL], float2 GM, float2* z, int l,
                                         const LaneTw<LOGN>& tw, float2 (&out)[Geo<LOGN>::PPL]) {
  using G = Geo<LOGN>;
  constexpr int M = G::M;
  const int pl = pidx(l);
#pragma unroll
  for (int q = 0; q < G::PPL; ++q) z[padd(pl, l, G::LPF * q)] = Gq[q];
  if (l == 0) z[G::PADN - 1] = GM;  // the spare slot (pidx never maps there)
  frame_fence<LOGN>();
  const int pn = pidx(-l);
#pragma unroll
  for (int q = 0; q < G::PPL; ++q) {
    const int k = l + G::LPF * q;
    // G_{M-k}; bin 0 pairs with G_M in the spare slot PADN - 1
    const int im = q == 0 ? (l == 0 ? G::PADN - 1 : padd(pn, -l, M)) : padd(pn, -l, M - G::LPF * q);
    const float2 gk = Gq[q], gm = z[im];
    float2 zp;
    if (k == 0) {
      zp = make_float2(gk.x + gm.x, gk.x - gm.x);
    } else {
      const float2 s = make_float2(gk.x + gm.x, gk.y - gm.y);  // gk + conj(gm)
      const float2 d = make_float2(gk.x - gm.x, gk.y + gm.y);  // gk - conj(gm)
      const float2 wd = cmul(conjf2(split_tw<LOGN>(tw, q)), d);  // W^-k * d
      zp = make_float2(0.5f * (s.x - wd.y), 0.5f * (s.y + wd.x));
    }
    out[q] = conjf2(zp);
  }
  frame_fence<LOGN>();
  fft_half<LOGN>(out, z, l, tw);
#pragma unroll
  for (int q = 0; q < G::PPL; ++q) {
    const float2 r = z[padd(pl, l, G::LPF * q)];
    out[q] = make_float2(r.x, -r.y);
  }
  frame_fence<LOGN>();
}

// Windowed frame-gradient slab row: slab[n - left] = w(n - left) * r_n.
template <int LOGN>
__device__ __forceinline__ void store_frame_grad(const float2 (&r)[Geo<LOGN>::PPL], const FrameArgs& a,
                                                 const Win<LOGN>& wn, float* __restrict__ slab, int l, bool active) {
  using G = Geo<LOGN>;
  if (!active) return;
#pragma unroll
  for (int q = 0; q < G::PPL; ++q) {
    const int w0 = 2 * (l + G::LPF * q) - a.left, w1 = w0 + 1;
    const float2 w = wn.get(q);
    if (w0 >= 0 && w0 < a.win) slab[w0] = w.x * r[q].x;
    if (w1 >= 0 && w1 < a.win) slab[w1] = w.y * r[q].y;
  }
}

// v_sqrt_f32 / v_rsq_f32 (1 ulp): the IEEE sqrtf expansion costs ~10 VALU per bin
__device__ __forceinline__ float clamp_sqrt(float p, float floor_) { return __builtin_amdgcn_sqrtf(fmaxf(p, floor_)); }
__device__ __forceinline__ float rsqrt_(float p) { return __builtin_amdgcn_rsqf(p); }
__device__ __forceinline__ float pw(float2 z) { return z.x * z.x + z.y * z.y; }

// -------------------------------------------------------------------------
// Kernels
// -------------------------------------------------------------------------

// register budget of the frame kernels: >= 2 waves per SIMD (<= 256 VGPRs; the
// 4-wave budget made hipcc spill, and the spilling builds computed wrong results)
#ifndef SEL_FFT_WAVES
#define SEL_FFT_WAVES 2
#endif
#define SEL_FFT_OCC __attribute__((amdgpu_waves_per_eu(SEL_FFT_WAVES)))

// Frame ownership: block b, iteration it -> frames (b*iters + it)*FPB + slot;
// the next frame's samples are fetched before the current one is transformed.
#define FRAME_PROLOGUE(LOGN, EXTRA_FLOATS) FRAME_PROLOGUE_X(LOGN, EXTRA_FLOATS, Geo<LOGN>::FPB)
// FPBV = frames per block iteration (block size / lanes per frame)
#define FRAME_PROLOGUE_X(LOGN, EXTRA_FLOATS, FPBV)                                  \
  using G = Geo<LOGN>;                                                              \
  extern __shared__ __align__(16) float2 lds_dyn[];                                 \
  const int slot = threadIdx.x / G::LPF, l = threadIdx.x % G::LPF;                  \
  float2* z = lds_dyn + slot * (G::PADN + (EXTRA_FLOATS) / 2);                      \
  const int nframes = int(a.B * a.F);                                               \
  const int fr0 = int(blockIdx.x) * iters * (FPBV) + slot;                          \
  Win<LOGN> wn;                                                                     \
  wn.init(window, a, l);                                                            \
  LaneTw<LOGN> tw;                                                                  \
  tw.load(l);

// A wave's current frame: flat index, signal, frame-in-signal (32-bit: the host
// keeps B*T < 2^29, so B*F < 2^31).  Consecutive iterations advance by FPB
// frames without a division.
struct FramePos {
  int fr, b, f;
  bool active;
  __device__ __forceinline__ void init(int fr_, int nframes, int F) {
    fr = fr_;
    active = fr < nframes;
    b = active ? fr / F : 0;
    f = active ? fr - b * F : 0;
  }
  __device__ __forceinline__ void advance(int step, int nframes, int F) {
    fr += step;
    f += step;
    while (f >= F) {  // step = FPB <= 16: a few rounds at most
      f -= F;
      ++b;
    }
    active = fr < nframes;
    if (!active) b = f = 0;
  }
};

// for it in [0, iters): P = this frame; RAW (and RAWY) hold its fetched samples on
// entry to the body, and the next frame's fetch is already in flight
#define FRAME_LOOP_BEGIN(X, RAW, PF)                                     \
  float2 RAW[G::PPL];                                                    \
  const __amdgpu_buffer_rsrc_t X##_rsrc = signal_rsrc(X, a);             \
  FramePos P;                                                            \
  P.init(fr0, nframes, a.F);                                             \
  if constexpr (PF) fetch_frame<LOGN>(X, X##_rsrc, a, P.b, P.f, l, P.active, RAW); \
  for (int it = 0; it < iters; ++it) {                                   \
    if constexpr (!(PF)) fetch_frame<LOGN>(X, X##_rsrc, a, P.b, P.f, l, P.active, RAW); \
    float2 v[G::PPL];                                                    \
    window_frame<LOGN>(RAW, wn, v);                                      \
    const FramePos cur = P;                                              \
    if (it + 1 < iters) {                                                \
      P.advance(G::FPB, nframes, a.F);                                   \
      if constexpr (PF) fetch_frame<LOGN>(X, X##_rsrc, a, P.b, P.f, l, P.active, RAW); \
    }                                                                    \
    const int64_t fr = cur.fr, b = cur.b;                                \
    const int f = cur.f;                                                 \
    const bool active = cur.active;                                      \
    (void)b;

// one-frame-ahead prefetch only where the registers allow it (PPL = 8, one signal)
#ifndef SEL_FFT_PF
#define SEL_FFT_PF 1
#endif
#define SEL_PF (SEL_FFT_PF && G::PPL == 8)

#define FRAME_LOOP_END }

// ---- hand-counted prefetch (|X| kernel) ----------------------------------
// Loads and stores share vmcnt on gfx950 and retire in issue order
// (MI355X_MICROARCH §vmcnt), but hipcc treats a counter with both pending as
// out of order and waits for vmcnt(0) before the prefetched samples are used:
// every frame then also waits for the previous frame's |X| stores to reach
// memory.  The prefetch is issued through inline asm (invisible to hipcc's
// counter model) and waited for by hand with vmcnt(kVmStores): in each
// iteration the stores of an active frame follow the next frame's loads.
#ifndef SEL_STFT_VMA
#define SEL_STFT_VMA 1
#endif
typedef float v2f_t __attribute__((ext_vector_type(2)));
// |X| stores issued after the prefetch by any wave whose frame is active
constexpr int kVmStores = 8;
// timing ablations of the |X| kernel: 1 no |X| stores, 2 no FFT,
// 4 no sample loads, 8 per-wave clock stamps over the first rows; 0 in every build
#ifndef SEL_STFT_ABL
#define SEL_STFT_ABL 0
#endif

template <int LOGN>
__device__ __forceinline__ void fetch_frame_vm(const float* __restrict__ x, __amdgpu_buffer_rsrc_t xr,
                                               const FrameArgs& a, int b, int f, int l, bool active,
                                               v2f_t (&raw)[8]) {
  using G = Geo<LOGN>;
  static_assert(G::PPL == 8 && G::LPF * 8 * 3 < 4096, "immediate offsets");
  constexpr int S = G::LPF * 8;  // bytes between a lane's consecutive points
  const int T = int(a.T);
  const int base = f * a.hop - a.P;
  const int sig = b * T;
  const float* xs = x + sig + base;
  if (active && base >= 0 && base + G::N <= T && (reinterpret_cast<uintptr_t>(xs) & 7) == 0) {
    if constexpr (G::LPF * 8 * 7 >= 4096) {  // n_fft 2048: points 4-7 off a second base address
      const float2* p = reinterpret_cast<const float2*>(xs) + l;
      const float2* p4 = p + 4 * G::LPF;
      asm volatile(
          "global_load_dwordx2 %0, %8, off\n\t"
          "global_load_dwordx2 %1, %8, off offset:%10\n\t"
          "global_load_dwordx2 %2, %8, off offset:%11\n\t"
          "global_load_dwordx2 %3, %8, off offset:%12\n\t"
          "global_load_dwordx2 %4, %9, off\n\t"
          "global_load_dwordx2 %5, %9, off offset:%10\n\t"
          "global_load_dwordx2 %6, %9, off offset:%11\n\t"
          "global_load_dwordx2 %7, %9, off offset:%12"
          : "=&v"(raw[0]), "=&v"(raw[1]), "=&v"(raw[2]), "=&v"(raw[3]), "=&v"(raw[4]), "=&v"(raw[5]),
            "=&v"(raw[6]), "=&v"(raw[7])
          : "v"(p), "v"(p4), "i"(S), "i"(2 * S), "i"(3 * S)
          : "memory");
    } else {
      const float2* p = reinterpret_cast<const float2*>(xs) + l;
      asm volatile(
          "global_load_dwordx2 %0, %8, off\n\t"
          "global_load_dwordx2 %1, %8, off offset:%9\n\t"
          "global_load_dwordx2 %2, %8, off offset:%10\n\t"
          "global_load_dwordx2 %3, %8, off offset:%11\n\t"
          "global_load_dwordx2 %4, %8, off offset:%12\n\t"
          "global_load_dwordx2 %5, %8, off offset:%13\n\t"
          "global_load_dwordx2 %6, %8, off offset:%14\n\t"
          "global_load_dwordx2 %7, %8, off offset:%15"
          : "=&v"(raw[0]), "=&v"(raw[1]), "=&v"(raw[2]), "=&v"(raw[3]), "=&v"(raw[4]), "=&v"(raw[5]),
            "=&v"(raw[6]), "=&v"(raw[7])
          : "v"(p), "i"(S), "i"(2 * S), "i"(3 * S), "i"(4 * S), "i"(5 * S), "i"(6 * S), "i"(7 * S)
          : "memory");
    }
  } else if (active) {
    unsigned o[16];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      int n0 = abs(base + 2 * (l + G::LPF * q)), n1 = abs(base + 2 * (l + G::LPF * q) + 1);
      n0 = min(n0, 2 * (T - 1) - n0);
      n1 = min(n1, 2 * (T - 1) - n1);
      o[2 * q] = unsigned(sig + n0) * 4u;
      o[2 * q + 1] = unsigned(sig + n1) * 4u;
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      float r[8];
      asm volatile(
          "buffer_load_dword %0, %8, %16, 0 offen\n\t"
          "buffer_load_dword %1, %9, %16, 0 offen\n\t"
          "buffer_load_dword %2, %10, %16, 0 offen\n\t"
          "buffer_load_dword %3, %11, %16, 0 offen\n\t"
          "buffer_load_dword %4, %12, %16, 0 offen\n\t"
          "buffer_load_dword %5, %13, %16, 0 offen\n\t"
          "buffer_load_dword %6, %14, %16, 0 offen\n\t"
          "buffer_load_dword %7, %15, %16, 0 offen"
          : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3]), "=&v"(r[4]), "=&v"(r[5]), "=&v"(r[6]),
            "=&v"(r[7])
          : "v"(o[8 * h]), "v"(o[8 * h + 1]), "v"(o[8 * h + 2]), "v"(o[8 * h + 3]), "v"(o[8 * h + 4]),
            "v"(o[8 * h + 5]), "v"(o[8 * h + 6]), "v"(o[8 * h + 7]), "s"(xr)
          : "memory");
#pragma unroll
      for (int q = 0; q < 4; ++q) raw[4 * h + q] = v2f_t{r[2 * q], r[2 * q + 1]};
    }
  } else {
#pragma unroll
    for (int q = 0; q < 8; ++q) raw[q] = v2f_t{0.f, 0.f};
  }
}

// the prefetched samples are in registers once at most N younger vector-memory
// operations are pending; the "+v" ties keep every use of raw[] below this point
template <int N>
__device__ __forceinline__ void vm_wait_raw(v2f_t (&raw)[8]) {
  asm volatile("s_waitcnt vmcnt(%8)"
               : "+v"(raw[0]), "+v"(raw[1]), "+v"(raw[2]), "+v"(raw[3]), "+v"(raw[4]), "+v"(raw[5]), "+v"(raw[6]),
                 "+v"(raw[7])
               : "i"(N)
               : "memory");
}

// Frames of wave unit u (FPW consecutive frames, lane slot sw): the unit index
// is wave-uniform, so the division by F runs on the scalar unit.
__device__ __forceinline__ FramePos unit_pos(int u, int FPW, int sw, int nframes, int F) {
  FramePos p;
  const int base = u * FPW, b0 = base / F;
  p.fr = base + sw;
  p.active = p.fr < nframes;
  p.b = b0;
  p.f = base - b0 * F + sw;
  while (p.f >= F) {  // sw < FPW <= 4: at most a few rounds
    p.f -= F;
    ++p.b;
  }
  if (!p.active) p.b = p.f = 0;
  return p;
}

// Block size of the |X| kernel where a frame fits one wave: one 1024-lane block
// per CU.  The SQ arbitrates issue by priority, then age, so with a static
// frame split the first-dispatched waves of a SIMD finish early and the CU ends
// on one or two latency-bound waves (per-wave stamps at B = 512, 1024/120/600:
// blocks of 4 waves took 51.7 / 57.1 / 65.5 / 73.2 us by dispatch rank on their
// CU); in one block the CU's 16 waves draw frames from one LDS counter and
// finish together.
#ifndef SEL_STFT_BS
#define SEL_STFT_BS 1024
#endif
template <int LOGN>
constexpr int mag_block() {
  return (SEL_STFT_VMA && Geo<LOGN>::LPF <= 64) ? SEL_STFT_BS : 256;
}

// |X| leaves as streaming (non-temporal) stores: the magnitudes (4/5 of the
// kernel's bytes) are written once and not read back by this launch, so they
// should not displace the signal rows in the caches (SEL_STFT_NT=0: plain stores)
#ifndef SEL_STFT_NT
#define SEL_STFT_NT 1
#endif
__device__ __forceinline__ void mag_store(float* p, float v) {
  if constexpr (SEL_STFT_NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

template <int LOGN, int BS = mag_block<LOGN>()>
__global__ __launch_bounds__(BS) SEL_FFT_OCC void k_stft_mag_fwd(const float* __restrict__ x, FrameArgs a,
                                                     const float* __restrict__ window, float floor_,
                                                     float* __restrict__ mag, int iters) {
  constexpr int FPBB = BS / Geo<LOGN>::LPF;
  FRAME_PROLOGUE_X(LOGN, 0, FPBB)
  constexpr int K = G::M + 1, H = G::PPL / 2;
  if constexpr (SEL_STFT_VMA && G::PPL == 8 && G::LPF <= 64) {
    // wave units of FPW frames; the block owns units [ub, ue) and its waves
    // take them in turn from an LDS counter (first one each by wave index)
    constexpr int FPW = 64 / G::LPF, WPB = BS / 64;
    __shared__ unsigned s_next;
    if (threadIdx.x == 0) s_next = 0;
    __syncthreads();
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x / 64), sw = (threadIdx.x % 64) / G::LPF;
    const int ub = int(blockIdx.x) * iters * WPB;
    const int ue = min(ub + iters * WPB, (nframes + FPW - 1) / FPW);
    v2f_t raw[8];
    const __amdgpu_buffer_rsrc_t xr = signal_rsrc(x, a);
    int u = ub + wid;
    FramePos P = unit_pos(u, FPW, sw, nframes, a.F);
    if (u < ue) fetch_frame_vm<LOGN>(x, xr, a, P.b, P.f, l, P.active && !(SEL_STFT_ABL & 4), raw);
    vm_wait_raw<0>(raw);
    [[maybe_unused]] uint64_t t0 = 0, r0 = 0;
    if constexpr ((SEL_STFT_ABL & 8) != 0) {
      t0 = __builtin_amdgcn_s_memtime();
      r0 = __builtin_amdgcn_s_memrealtime();
    }
    while (u < ue) {
      float2 v[G::PPL];
#pragma unroll
      for (int q = 0; q < G::PPL; ++q) {
        const float2 w = wn.get(q);
        v[q] = make_float2(raw[q].x * w.x, raw[q].y * w.y);
      }
      unsigned tk = 0;
      if (threadIdx.x % 64 == 0) tk = atomicAdd(&s_next, 1u);
      const int un = ub + WPB + __builtin_amdgcn_readlane(int(tk), 0);
      const bool pf = un < ue;
      const FramePos cur = P;
      if (pf) {
        P = unit_pos(un, FPW, sw, nframes, a.F);
        fetch_frame_vm<LOGN>(x, xr, a, P.b, P.f, l, P.active && !(SEL_STFT_ABL & 4), raw);
      }
      float pwr[G::PPL], pmid;
      if constexpr ((SEL_STFT_ABL & 2) != 0) {
#pragma unroll
        for (int q = 0; q < G::PPL; ++q) pwr[q] = v[q].x * v[q].x + v[q].y * v[q].y;
        pmid = pwr[0];
      } else {
        fft_pairs<LOGN>(v, z, l, tw, pwr, pmid);
      }
      if (cur.active && !(SEL_STFT_ABL & 1)) {
        float* out = mag + int64_t(cur.fr) * K;
#pragma unroll
        for (int q = 0; q < H; ++q) {
          mag_store(&out[l + G::LPF * q], clamp_sqrt(pwr[q], floor_));
          mag_store(&out[G::M - l - G::LPF * q], clamp_sqrt(pwr[H + q], floor_));
        }
        if (l == 0) mag_store(&out[G::M / 2], clamp_sqrt(pmid, floor_));
      }
      if (pf) vm_wait_raw<(SEL_STFT_ABL & 1) ? 0 : kVmStores>(raw);
      u = un;
    }
    if constexpr ((SEL_STFT_ABL & 8) != 0) {  // per-wave shader-clock / 100 MHz stamps over the frame loop
      const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
      __syncthreads();
      if (threadIdx.x % 64 == 0) {
        uint64_t* st = reinterpret_cast<uint64_t*>(mag) + (size_t(blockIdx.x) * (BS / 64) + threadIdx.x / 64) * 8;
        st[0] = t0;
        st[1] = t1;
        st[2] = r0;
        st[3] = r1;
        st[4] = __builtin_amdgcn_s_getreg(0xF804);  // HW_ID: simd [5:4], cu [11:8], sh [12], se [15:13]
        st[5] = __builtin_amdgcn_s_getreg((15 << 11) | 20);  // XCC_ID
        st[6] = blockIdx.x;
        st[7] = 0x5354465453544654ull;  // record marker
      }
    }
  } else {
    static_assert(BS == 256, "FRAME_LOOP_BEGIN advances by Geo::FPB");
    FRAME_LOOP_BEGIN(x, raw, SEL_PF)
    (void)f;
    fft_half<LOGN>(v, z, l, tw);
    float pwr[G::PPL], pmid;
    split_pairs<LOGN>(z, l, tw, pwr, pmid);
    if (active) {
      float* out = mag + fr * K;
#pragma unroll
      for (int q = 0; q < H; ++q) {
        out[l + G::LPF * q] = clamp_sqrt(pwr[q], floor_);
        out[G::M - l - G::LPF * q] = clamp_sqrt(pwr[H + q], floor_);
      }
      if (l == 0) out[G::M / 2] = clamp_sqrt(pmid, floor_);
    }
    FRAME_LOOP_END
  }
}

template <int LOGN>
__global__ __launch_bounds__(256) SEL_FFT_OCC void k_stft_mag_bwd(const float* __restrict__ x, FrameArgs a,
                                                      const float* __restrict__ window, float floor_,
                                                      const float* __restrict__ gmag, float* __restrict__ slab,
                                                      int iters) {
  FRAME_PROLOGUE(LOGN, 0)
  FRAME_LOOP_BEGIN(x, raw, false)
  (void)f;
  fft_half<LOGN>(v, z, l, tw);
  float2 X[G::PPL], XM;
  real_split<LOGN>(z, l, tw, X, XM);
  constexpr int K = G::M + 1;
  const float* gm = gmag + (active ? fr : 0) * K;
#pragma unroll
  for (int q = 0; q < G::PPL; ++q) {
    const float p = pw(X[q]);
    const float s = (active && p >= floor_) ? gm[l + G::LPF * q] * rsqrt_(p) : 0.f;
    X[q] = make_float2(s * X[q].x, s * X[q].y);
  }
  {
    const float p = pw(XM);
    const float s = (active && l == 0 && p >= floor_) ? gm[G::M] * rsqrt_(p) : 0.f;
    XM = make_float2(s * XM.x, s * XM.y);
  }
  c2r_grad<LOGN>(X, XM, z, l, tw, v);
  store_frame_grad<LOGN>(v, a, wn, slab + (active ? fr : 0) * a.win, l, active);
  FRAME_LOOP_END
}

// |Y| of the reference signal's frame (windowed points in v) into ym[]
// (PPL bins + bin M on l == 0)
template <int LOGN, bool PAIRED>
__device__ __forceinline__ void ref_mag(float2 (&v)[Geo<LOGN>::PPL], int l, float2* z, const LaneTw<LOGN>& tw,
                                        float floor_, float (&ym)[Geo<LOGN>::PPL + 1]) {
  using G = Geo<LOGN>;
  if constexpr (PAIRED) {  // split_pairs' bins (the fused forward)
    float pwr[G::PPL], pmid;
    fft_pairs<LOGN, false>(v, z, l, tw, pwr, pmid);
#pragma unroll
    for (int q = 0; q < G::PPL; ++q) ym[q] = clamp_sqrt(pwr[q], floor_);
    ym[G::PPL] = clamp_sqrt(pmid, floor_);
  } else {  // real_split's bins k = l + LPF*q, then M (the backward)
    fft_half<LOGN>(v, z, l, tw);
    float2 X[G::PPL], XM;
    real_split<LOGN>(z, l, tw, X, XM);
#pragma unroll
    for (int q = 0; q < G::PPL; ++q) ym[q] = clamp_sqrt(pw(X[q]), floor_);
    ym[G::PPL] = clamp_sqrt(pw(XM), floor_);
  }
}

// the reference signal's windowed frame at the current position (no prefetch)
#define Y_FRAME(VY)                                                        \
  float2 VY[G::PPL];                                                       \
  {                                                                        \
    float2 rawy[G::PPL];                                                   \
    fetch_frame<LOGN>(y, y_rsrc, a, cur.b, cur.f, l, cur.active, rawy);    \
    window_frame<LOGN>(rawy, wn, VY);                                      \
  }

// Fused STFT loss forward: both signals' spectra, block partial sums
// {sum (ym-xm)^2, sum ym^2, sum |ln ym - ln xm|} (stft_loss.py:56, :77).
template <int LOGN>
__global__ __launch_bounds__(256) SEL_FFT_OCC void k_stft_loss_fwd(const float* __restrict__ x, const float* __restrict__ y,
                                                       FrameArgs a, const float* __restrict__ window,
                                                       float floor_, double* __restrict__ partials, int iters) {
  FRAME_PROLOGUE(LOGN, 0)
  __shared__ double red[16];
  float s1 = 0.f, s2 = 0.f, s3 = 0.f;
  const __amdgpu_buffer_rsrc_t y_rsrc = signal_rsrc(y, a);
  FRAME_LOOP_BEGIN(x, raw, false)
  (void)f;
  (void)fr;
  Y_FRAME(vy)
  float ym[G::PPL + 1];
  ref_mag<LOGN, true>(vy, l, z, tw, floor_, ym);
  float pwr[G::PPL], pmid;
  fft_pairs<LOGN, false>(v, z, l, tw, pwr, pmid);  // same bin pairing as ref_mag's ym
  if (active) {
#pragma unroll
    for (int q = 0; q <= G::PPL; ++q) {
      if (q == G::PPL && l != 0) break;
      const float xm = clamp_sqrt(q < G::PPL ? pwr[q] : pmid, floor_);
      const float d = ym[q] - xm;
      s1 += d * d;
      s2 += ym[q] * ym[q];
      s3 += fabsf(logf(ym[q]) - logf(xm));
    }
  }
  FRAME_LOOP_END
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
__global__ __launch_bounds__(256) SEL_FFT_OCC void k_stft_loss_bwd(const float* __restrict__ x, const float* __restrict__ y,
                                                       FrameArgs a, const float* __restrict__ window,
                                                       float floor_, const float* __restrict__ coef,
                                                       float* __restrict__ slab, int iters) {
  FRAME_PROLOGUE(LOGN, 0)
  const float ca = coef[0], cb = coef[1];
  const __amdgpu_buffer_rsrc_t y_rsrc = signal_rsrc(y, a);
  FRAME_LOOP_BEGIN(x, raw, false)
  (void)f;
  Y_FRAME(vy)
  float ym[G::PPL + 1];
  ref_mag<LOGN, false>(vy, l, z, tw, floor_, ym);
  fft_half<LOGN>(v, z, l, tw);
  float2 X[G::PPL + 1];
  real_split<LOGN>(z, l, tw, reinterpret_cast<float2(&)[G::PPL]>(X), X[G::PPL]);
#pragma unroll
  for (int q = 0; q <= G::PPL; ++q) {
    const float p = pw(X[q]);
    const float xm = clamp_sqrt(p, floor_);
    const float lx = logf(xm), ly = logf(ym[q]);
    const float sg = lx > ly ? 1.f : (lx < ly ? -1.f : 0.f);
    const float gx = ca * (xm - ym[q]) + cb * sg / xm;
    const bool ok = active && p >= floor_ && (q < G::PPL || l == 0);
    const float s = ok ? gx / xm : 0.f;
    X[q] = make_float2(s * X[q].x, s * X[q].y);
  }
  c2r_grad<LOGN>(reinterpret_cast<float2(&)[G::PPL]>(X), X[G::PPL], z, l, tw, v);
  store_frame_grad<LOGN>(v, a, wn, slab + (active ? fr : 0) * a.win, l, active);
  FRAME_LOOP_END
}

__device__ __forceinline__ float log_k(float v, int kind) {
  return kind == SEL_LOG_E ? logf(v) : (kind == SEL_LOG_2 ? log2f(v) : log10f(v));
}
__device__ __forceinline__ float dlog_k(int kind) {
  return kind == SEL_LOG_E ? 1.f : (kind == SEL_LOG_2 ? 0.6931471805599453f : 2.302585092994046f);
}

// sum over k in [k0, k1) of a[k] * w[k * ld + m]: one fmaf chain in ascending
// k (the order the single loop used, so results are bit-identical), with the
// loads issued eight at a time so their latencies overlap (the top mel filters
// at n_fft 2048 span ~70 bins; one dependent global load per bin left the
// lane on a ~70-deep latency chain)
__device__ __forceinline__ float mel_dot(const float* a, const float* __restrict__ w, int ld, int m, int k0,
                                        int k1) {
  float s = 0.f;
  int k = k0;
  for (; k + 8 <= k1; k += 8) {
    float av[8], wv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      av[u] = a[k + u];
      wv[u] = w[(k + u) * ld + m];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) s = fmaf(av[u], wv[u], s);
  }
  for (; k < k1; ++k) s = fmaf(a[k], w[k * ld + m], s);
  return s;
}

struct MelArgs {
  const float* melmat;     // (K, nm)
  const int2* range;       // fwd: per-mel bin range; bwd: per-bin mel range
  int nm;
  float eps;
  int log_kind;
};

// The filterbank's nonzero band staged in LDS once per block: mel m's weights
// over its bins [kr_m.x, kr_m.y) at wl[m * wmax + (k - kr_m.x)], wmax = the
// widest filter.  The per-frame mel sums then read LDS instead of one global
// load per (bin, mel) — at n_fft 2048 the top filters span ~70 bins, and that
// chain of L2 round trips was most of the log-mel kernels' time (the same
// fmaf order and weights: bit-identical results).  Needs nm * wmax <= cap
// floats (kMelCap, or the host's smaller grant); otherwise the block keeps
// reading melmat from global (returns 0).
constexpr int kMelCap = 6144;  // 24 KB: 80 filters x 76 bins (n_fft 2048) fit
__device__ __forceinline__ int stage_mel(const float* __restrict__ melmat, const int2* __restrict__ krange, int nm,
                                         int2* kr_l, float* wl, int cap) {
  __shared__ int s_wmax;
  const int tid = threadIdx.x;
  if (tid == 0) s_wmax = 0;
  __syncthreads();
  int w = 0;
  for (int m = tid; m < nm; m += blockDim.x) {
    const int2 r = krange[m];
    kr_l[m] = r;
    w = max(w, r.y - r.x);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) w = max(w, __shfl_xor(w, o, 64));
  if ((tid & 63) == 0) atomicMax(&s_wmax, w);
  __syncthreads();
  const int wmax = s_wmax;
  if (wmax <= 0 || int64_t(nm) * wmax > cap) return 0;
  const int total = nm * wmax;
  for (int i0 = 0; i0 < total; i0 += 8 * int(blockDim.x)) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {  // eight loads in flight per lane
      const int i = i0 + u * int(blockDim.x) + tid;
      const int m = i / wmax, j = i - m * wmax;
      const int2 r = i < total ? kr_l[m] : make_int2(0, 0);
      v[u] = r.x + j < r.y ? melmat[int64_t(r.x + j) * nm + m] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = i0 + u * int(blockDim.x) + tid;
      if (i < total) wl[i] = v[u];
    }
  }
  __syncthreads();
  return wmax;
}

// LDS bytes of the staged filterbank after the frame slots
inline size_t mel_lds_bytes(int nm) { return (size_t(nm) * sizeof(int2) + 15) / 16 * 16 + size_t(kMelCap) * 4; }

// log-mel forward (mel_loss.py:84-94): stft -> |X| (floor eps) -> melmat -> floor eps -> log.
// Frame loop on the |X| kernel's memory schedule: the next frame's samples are
// requested through inline asm (fetch_frame_vm, invisible to hipcc's counter
// model) and waited for by hand with vmcnt(MS), MS = the fixed number of log-mel
// stores each lane issues per frame after that request (one per mel slot m = l +
// LPF*i, i < MS; slots past n_mels or of an inactive frame go to RU_OOB and are
// dropped).  hipcc's own wait there was vmcnt(0): every frame also waited for
// the previous frame's stores to reach memory.
template <int LOGN>
__global__ __launch_bounds__(256) SEL_FFT_OCC void k_logmel_fwd(const float* __restrict__ x, FrameArgs a,
                                                    const float* __restrict__ window, MelArgs ma,
                                                    float* __restrict__ out, int iters) {
  FRAME_PROLOGUE(LOGN, 0)
  constexpr int MS = (G::M + 12 + G::LPF - 1) / G::LPF;  // mel slots per lane (n_mels <= n_fft/2 + 12)
  float* magb = reinterpret_cast<float*>(z);
  int2* kr_l = reinterpret_cast<int2*>(lds_dyn + G::FPB * G::PADN);
  float* wl = reinterpret_cast<float*>(kr_l) + (ma.nm * 2 + 3) / 4 * 4;
  const int wmax = stage_mel(ma.melmat, ma.range, ma.nm, kr_l, wl, kMelCap);
  const __amdgpu_buffer_rsrc_t xr = signal_rsrc(x, a);
  // the host keeps B * n_mels * F * 4 <= RU_OOB (ru_region_ok)
  const __amdgpu_buffer_rsrc_t orr =
      __builtin_amdgcn_make_buffer_rsrc(out, 0, int(a.B * ma.nm * a.F * 4), 0x00020000);
  v2f_t raw[8];
  FramePos P;
  P.init(fr0, nframes, a.F);
  fetch_frame_vm<LOGN>(x, xr, a, P.b, P.f, l, P.active, raw);
  vm_wait_raw<0>(raw);
  for (int it = 0; it < iters; ++it) {
    float2 v[G::PPL];
#pragma unroll
    for (int q = 0; q < G::PPL; ++q) {
      const float2 w = wn.get(q);
      v[q] = make_float2(raw[q].x * w.x, raw[q].y * w.y);
    }
    const FramePos cur = P;
    const bool pf = it + 1 < iters;
    if (pf) {
      P.advance(G::FPB, nframes, a.F);
      fetch_frame_vm<LOGN>(x, xr, a, P.b, P.f, l, P.active, raw);
    }
    float pwr[G::PPL], pmid;
    fft_pairs<LOGN>(v, z, l, tw, pwr, pmid);
#pragma unroll
    for (int q = 0; q < G::PPL / 2; ++q) {
      magb[l + G::LPF * q] = clamp_sqrt(pwr[q], ma.eps);
      magb[G::M - l - G::LPF * q] = clamp_sqrt(pwr[G::PPL / 2 + q], ma.eps);
    }
    if (l == 0) magb[G::M / 2] = clamp_sqrt(pmid, ma.eps);
    frame_fence<LOGN>();
#pragma unroll
    for (int i = 0; i < MS; ++i) {
      const int m = l + G::LPF * i;
      const bool ok = cur.active && m < ma.nm;
      float val = 0.f;
      if (ok) {
        float s;
        if (wmax) {
          const int2 r = kr_l[m];
          s = mel_dot(magb, wl + m * wmax - r.x, 1, 0, r.x, r.y);
        } else {
          const int2 r = ma.range[m];
          s = mel_dot(magb, ma.melmat, ma.nm, m, r.x, r.y);
        }
        val = log_k(fmaxf(s, ma.eps), ma.log_kind);
      }
      const int off = ok ? int(((int64_t(cur.b) * ma.nm + m) * a.F + cur.f) * 4) : RU_OOB;
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, val), orr, off, 0, 0);
    }
    frame_fence<LOGN>();
    if (pf) vm_wait_raw<MS>(raw);
  }
}

// log-mel backward. gsel: if ref != nullptr, upstream = g_scale * sign(gout - ref)
// (L1 backward, mel_loss.py:153); else upstream = gout.  Each frame owns
// PADN complex slots (spectrum, then |X|, then G) + nm floats (dL/dmel).
template <int LOGN>
__global__ __launch_bounds__(256) SEL_FFT_OCC void k_logmel_bwd(const float* __restrict__ x, FrameArgs a,
                                                    const float* __restrict__ window, MelArgs ma,
                                                    const int2* __restrict__ krange, const float* __restrict__ gout,
                                                    const float* __restrict__ ref, const float* __restrict__ gscale,
                                                    float gmul, float* __restrict__ slab, int iters, int glin_floats) {
  FRAME_PROLOGUE(LOGN, glin_floats)
  float* magb = reinterpret_cast<float*>(z);
  float* glin = reinterpret_cast<float*>(z + G::PADN);
  int2* kr_l = reinterpret_cast<int2*>(lds_dyn + G::FPB * (G::PADN + glin_floats / 2));
  float* wl = reinterpret_cast<float*>(kr_l) + (ma.nm * 2 + 3) / 4 * 4;
  const int wmax = stage_mel(ma.melmat, krange, ma.nm, kr_l, wl, kMelCap);
  const float gs = ref ? gscale[0] * gmul : 0.f;
  FRAME_LOOP_BEGIN(x, raw, false)
  // upstream gradient of mel m of this frame
  auto upstream = [&](int m) {
    const int64_t o = (b * ma.nm + m) * a.F + f;
    if (ref) {
      const float d = gout[o] - ref[o];
      return d > 0.f ? gs : (d < 0.f ? -gs : 0.f);
    }
    return gout[o];
  };
  // the first mel of this lane: loaded here, in flight across the transform
  const float up0 = active && l < ma.nm ? upstream(l) : 0.f;
  fft_half<LOGN>(v, z, l, tw);
  float2 X[G::PPL + 1];
  real_split<LOGN>(z, l, tw, reinterpret_cast<float2(&)[G::PPL]>(X), X[G::PPL]);
#pragma unroll
  for (int q = 0; q < G::PPL; ++q) magb[l + G::LPF * q] = clamp_sqrt(pw(X[q]), ma.eps);
  if (l == 0) magb[G::M] = clamp_sqrt(pw(X[G::PPL]), ma.eps);
  frame_fence<LOGN>();
  for (int m = l; m < ma.nm; m += G::LPF) {
    float gv = 0.f;
    if (active) {
      float s;
      if (wmax) {
        const int2 r = kr_l[m];
        s = mel_dot(magb, wl + m * wmax - r.x, 1, 0, r.x, r.y);
      } else {
        const int2 r = krange[m];
        s = mel_dot(magb, ma.melmat, ma.nm, m, r.x, r.y);
      }
      const float up = m == l ? up0 : upstream(m);
      const float mel = fmaxf(s, ma.eps);
      gv = (s >= ma.eps) ? up / (mel * dlog_k(ma.log_kind)) : 0.f;
    }
    glin[m] = gv;
  }
  frame_fence<LOGN>();
#pragma unroll
  for (int q = 0; q <= G::PPL; ++q) {
    const int k = q < G::PPL ? l + G::LPF * q : G::M;
    const int2 r = ma.range[k];
    float gmag = 0.f;
    if (wmax) {
      for (int m = r.x; m < r.y; ++m) {  // melmat[k][m] is 0 outside mel m's band
        const int2 km = kr_l[m];
        const float wv = k >= km.x && k < km.y ? wl[m * wmax + k - km.x] : 0.f;
        gmag = fmaf(wv, glin[m], gmag);
      }
    } else {
      for (int m = r.x; m < r.y; ++m) gmag = fmaf(ma.melmat[k * ma.nm + m], glin[m], gmag);
    }
    const float p = pw(X[q]);
    const bool ok = active && p >= ma.eps && (q < G::PPL || l == 0);
    const float s = ok ? gmag * rsqrt_(p) : 0.f;
    X[q] = make_float2(s * X[q].x, s * X[q].y);
  }
  frame_fence<LOGN>();  // magb / glin reads done before c2r overwrites the slots
  c2r_grad<LOGN>(reinterpret_cast<float2(&)[G::PPL]>(X), X[G::PPL], z, l, tw, v);
  store_frame_grad<LOGN>(v, a, wn, slab + (active ? fr : 0) * a.win, l, active);
  FRAME_LOOP_END
}

// Fused log-mel L1 (mel_loss.py:151-154): loss = mean |logmel(x) - logmel(y)|
// and, with slab != nullptr, its gradient w.r.t. x for a unit upstream, in one
// pass per frame position: y's FFT and log-mels (parked in the frame's
// dL/dmel LDS slots), then x's FFT and log-mels, |d| into the loss partial, and
// the adjoint of x's path (sign(d) / n through log, the mel projection, |X|
// and the FFT) into the frame-gradient slab, as k_logmel_bwd does from stored
// log-mels.  The separate path ran three frame transforms per position (x and y
// forward, x again in the backward) and stored and re-read both log-mel
// tensors; this one runs three in one launch (y, x, x's adjoint) with no
// log-mel tensor in memory, and the backward is one scale by the upstream.
template <int LOGN>
__global__ __launch_bounds__(256) SEL_FFT_OCC void k_mel_l1(const float* __restrict__ x, const float* __restrict__ y,
                                                FrameArgs a, const float* __restrict__ window, MelArgs ma,
                                                const int2* __restrict__ krange, float inv_n,
                                                double* __restrict__ partials, float* __restrict__ slab, int iters,
                                                int glin_floats) {
  FRAME_PROLOGUE(LOGN, glin_floats)
  __shared__ double red[16];
  float* magb = reinterpret_cast<float*>(z);
  float* glin = reinterpret_cast<float*>(z + G::PADN);
  int2* kr_l = reinterpret_cast<int2*>(lds_dyn + G::FPB * (G::PADN + glin_floats / 2));
  float* wl = reinterpret_cast<float*>(kr_l) + (ma.nm * 2 + 3) / 4 * 4;
  // per-bin mel ranges (mrange) after the filterbank: the adjoint's per-bin
  // loop reads them from LDS, not one global load per bin and frame
  int2* mr_l = reinterpret_cast<int2*>(wl + kMelCap);
  for (int k = threadIdx.x; k <= G::M; k += blockDim.x) mr_l[k] = ma.range[k];
  const int wmax = stage_mel(ma.melmat, krange, ma.nm, kr_l, wl, kMelCap);  // (its barriers cover mr_l)
  const __amdgpu_buffer_rsrc_t x_rsrc = signal_rsrc(x, a);
  const __amdgpu_buffer_rsrc_t y_rsrc = signal_rsrc(y, a);
  const float dl = dlog_k(ma.log_kind);
  auto mel_of = [&](int m) {  // sum_k melmat[k][m] |X_k| from magb
    if (wmax) {
      const int2 r = kr_l[m];
      return mel_dot(magb, wl + m * wmax - r.x, 1, 0, r.x, r.y);
    }
    const int2 r = krange[m];
    return mel_dot(magb, ma.melmat, ma.nm, m, r.x, r.y);
  };
  float lsum = 0.f;
  FramePos P;
  P.init(fr0, nframes, a.F);
  for (int it = 0; it < iters; ++it) {
  const FramePos cur = P;
  if (it + 1 < iters) P.advance(G::FPB, nframes, a.F);
  const bool active = cur.active;
  // both frames requested together (one exposed latency per position)
  float2 raw[G::PPL], rawy[G::PPL];
  fetch_frame<LOGN>(x, x_rsrc, a, cur.b, cur.f, l, cur.active, raw);
  fetch_frame<LOGN>(y, y_rsrc, a, cur.b, cur.f, l, cur.active, rawy);
  float2 v[G::PPL];
  // y: log-mels of this lane's slots, parked in the frame's dL/dmel slots
  // (glin[m]: read back and overwritten by the same lane in x's pass)
  {
    float2 vy[G::PPL];
    window_frame<LOGN>(rawy, wn, vy);
    float pwr[G::PPL], pmid;
    fft_pairs<LOGN, false>(vy, z, l, tw, pwr, pmid);
#pragma unroll
    for (int q = 0; q < G::PPL / 2; ++q) {
      magb[l + G::LPF * q] = clamp_sqrt(pwr[q], ma.eps);
      magb[G::M - l - G::LPF * q] = clamp_sqrt(pwr[G::PPL / 2 + q], ma.eps);
    }
    if (l == 0) magb[G::M / 2] = clamp_sqrt(pmid, ma.eps);
    frame_fence<LOGN>();
    for (int m = l; m < ma.nm; m += G::LPF) glin[m] = active ? log_k(fmaxf(mel_of(m), ma.eps), ma.log_kind) : 0.f;
    frame_fence<LOGN>();  // magb reads done before x's transform overwrites the slots
  }
  // x: log-mels, |d|, and dL/dmel = sign(d) / n through the log
  window_frame<LOGN>(raw, wn, v);
  fft_half<LOGN>(v, z, l, tw);
  float2 X[G::PPL + 1];
  real_split<LOGN>(z, l, tw, reinterpret_cast<float2(&)[G::PPL]>(X), X[G::PPL]);
#pragma unroll
  for (int q = 0; q < G::PPL; ++q) magb[l + G::LPF * q] = clamp_sqrt(pw(X[q]), ma.eps);
  if (l == 0) magb[G::M] = clamp_sqrt(pw(X[G::PPL]), ma.eps);
  frame_fence<LOGN>();
  for (int m = l; m < ma.nm; m += G::LPF) {
    float gv = 0.f;
    if (active) {
      const float sm = mel_of(m);
      const float mel = fmaxf(sm, ma.eps);
      const float d = log_k(mel, ma.log_kind) - glin[m];
      lsum += fabsf(d);
      const float up = d > 0.f ? inv_n : (d < 0.f ? -inv_n : 0.f);
      gv = (sm >= ma.eps) ? up / (mel * dl) : 0.f;
    }
    glin[m] = gv;
  }
  if (slab) {  // the gradient (launch-uniform)
    frame_fence<LOGN>();
#pragma unroll
    for (int q = 0; q <= G::PPL; ++q) {
      const int k = q < G::PPL ? l + G::LPF * q : G::M;
      const int2 r = mr_l[k];
      float gmag = 0.f;
      if (wmax) {
        for (int m = r.x; m < r.y; ++m) {  // melmat[k][m] is 0 outside mel m's band
          const int2 km = kr_l[m];
          const float wv = k >= km.x && k < km.y ? wl[m * wmax + k - km.x] : 0.f;
          gmag = fmaf(wv, glin[m], gmag);
        }
      } else {
        for (int m = r.x; m < r.y; ++m) gmag = fmaf(ma.melmat[k * ma.nm + m], glin[m], gmag);
      }
      const float p = pw(X[q]);
      const bool ok = active && p >= ma.eps && (q < G::PPL || l == 0);
      const float sc = ok ? gmag * rsqrt_(p) : 0.f;
      X[q] = make_float2(sc * X[q].x, sc * X[q].y);
    }
    frame_fence<LOGN>();  // magb / glin reads done before c2r overwrites the slots
    c2r_grad<LOGN>(reinterpret_cast<float2(&)[G::PPL]>(X), X[G::PPL], z, l, tw, v);
    store_frame_grad<LOGN>(v, a, wn, slab + (active ? cur.fr : 0) * a.win, l, active);
  } else {
    frame_fence<LOGN>();  // glin / magb reads done before the next frame's transform
  }
  }
  const double r = block_sum<double>(double(lsum), red);
  if (threadIdx.x == 0) partials[blockIdx.x] = r;
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
// inv_n == 0: the element count is sums[3] (the data-parallel exchange's
// all-reduced count, kept on device: no host sync)
__global__ void k_stft_loss_finish(const double* __restrict__ sums, double inv_n, float* out2) {
  if (inv_n == 0.0) inv_n = 1.0 / sums[3];
  const float n1 = sqrtf(float(sums[0])), n2 = sqrtf(float(sums[1]));
  out2[0] = n1 / n2;
  out2[1] = float(sums[2] * inv_n);
}

// coef {a, b, c, d} for the magnitude-pair backward given upstream {g_sc, g_mag}.
__global__ void k_stft_loss_coef(const double* __restrict__ sums, double inv_n,
                                 const float* __restrict__ g_sc, const float* __restrict__ g_mag,
                                 float* coef) {
  if (inv_n == 0.0) inv_n = 1.0 / sums[3];  // k_stft_loss_finish
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
  // frame loads address the batch through 32-bit buffer offsets
  SEL_REQUIRE(B * T < (int64_t(1) << 29), SEL_ERR_UNSUPPORTED,
              "batch of %lld x %lld samples exceeds 2 GiB per call: split the batch", (long long)B, (long long)T);
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

// Launch plan of the wave-FFT kernels: FPB frames per block iteration, `iters`
// iterations per block (enough blocks to fill 256 CUs 8 deep first).
// Frame groups per block.  A block pays a fixed prologue (per-lane twiddles and
// window from the tables, the first frame's fetch) before its frame loop
// pipelines, and blocks of one launch take near-equal time, so a grid slightly
// larger than the resident-block capacity (`slots`) costs a whole extra round
// for its tail.  Default: one round, iters = ceil(groups / slots) (measured at
// B = 512, 1024/120/600: 117 us at 8 iters -> 98-100 us).  tune key 14: -1 = the
// earlier rule (<= 8 iters, >= 2048 groups per iter), > 0 = fixed iters.
template <int LOGN>
unsigned frame_grid(int64_t nframes, int& iters, int64_t slots = 0, int fpb = Geo<LOGN>::FPB) {
  const int64_t groups = (nframes + fpb - 1) / fpb;
  if (tune(14) > 0) {
    iters = tune(14);
  } else if (tune(14) == -1 || slots <= 0) {
    iters = int(std::max<int64_t>(1, std::min<int64_t>(8, groups / 2048)));
  } else {
    iters = int(std::max<int64_t>(1, (groups + slots - 1) / slots));
  }
  return unsigned((groups + iters - 1) / iters);
}

// grid of the last SEL_FRAME_DISPATCH on this thread (per-block partial counts)
thread_local unsigned t_last_frame_grid = 0;

// resident-block capacity of a frame kernel at `lds` bytes per block (cached
// per call site by the dispatch macro)
template <typename KerT>
int64_t frame_slots(KerT ker, size_t lds, int block = 256) {
  int dev = 0, cus = 0, per_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, ker, block, lds) != hipSuccess)
    return 0;
  return int64_t(cus) * per_cu;
}

// dispatch helper: one template kernel family over LOGN in [8, 11]; the kernel's
// trailing arguments are (iters, ...EXTRA); EXTRA_FLOATS = per-frame LDS floats
// beyond the spectrum slots
#define SEL_FRAME_CASE(L, nframes, stream, extra, KER, ...)                                   \
  case L: {                                                                                   \
    using G = Geo<L>;                                                                         \
    int iters;                                                                                \
    const size_t lds = size_t(G::FPB) * (G::PADN * sizeof(float2) + size_t(extra) * sizeof(float)); \
    static const int64_t slots = frame_slots(KER<L>, lds);                                    \
    const unsigned grid = frame_grid<L>(nframes, iters, slots);                               \
    t_last_frame_grid = grid;                                                                 \
    if (grid) hipLaunchKernelGGL(KER<L>, dim3(grid), dim3(256), lds, stream, __VA_ARGS__, iters); \
  } break;

#define SEL_FRAME_DISPATCH_X(logn, nframes, stream, extra, KER, ...)                          \
  do {                                                                                       \
    switch (logn) {                                                                          \
      SEL_FRAME_CASE(8, nframes, stream, extra, KER, __VA_ARGS__)                            \
      SEL_FRAME_CASE(9, nframes, stream, extra, KER, __VA_ARGS__)                            \
      SEL_FRAME_CASE(10, nframes, stream, extra, KER, __VA_ARGS__)                           \
      SEL_FRAME_CASE(11, nframes, stream, extra, KER, __VA_ARGS__)                           \
      default:                                                                               \
        ::sel::set_error("unsupported log2(n_fft)=%d", logn);                                \
        return SEL_ERR_UNSUPPORTED;                                                          \
    }                                                                                        \
    SEL_LAUNCH_CHECK();                                                                      \
  } while (0)

#define SEL_FRAME_DISPATCH(logn, nframes, stream, KER, ...) \
  SEL_FRAME_DISPATCH_X(logn, nframes, stream, 0, KER, __VA_ARGS__)

// upper bound on the block count of any launch plan (workspace sizing)
int64_t n_blocks(int logn, int64_t nframes) {
  int fpb;
  switch (logn) {
    case 8: fpb = Geo<8>::FPB; break;
    case 9: fpb = Geo<9>::FPB; break;
    case 10: fpb = Geo<10>::FPB; break;
    default: fpb = Geo<11>::FPB;
  }
  return (nframes + fpb - 1) / fpb;
}

int ola(const float* slab, const FrameArgs& a, float* gx, hipStream_t s) {
  if (a.B == 0) return SEL_OK;
  dim3 grid(unsigned((a.T + 255) / 256), unsigned(a.B));
  hipLaunchKernelGGL(k_ola_fold, grid, dim3(256), 0, s, slab, a, gx);
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

// (0 for an invalid shape: the call it sizes fails its own check_frame)
size_t slab_bytes(int64_t B, int64_t T, int hop, int win) {
  if (B < 0 || T < 0 || hop <= 0 || win <= 0) return 0;
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
  switch (logn) {
#define SEL_MAG_CASE(L)                                                                                   \
    case L: {                                                                                             \
      constexpr int BS = mag_block<L>(), FPBB = BS / Geo<L>::LPF;                                         \
      int iters;                                                                                          \
      const size_t lds = size_t(FPBB) * Geo<L>::PADN * sizeof(float2);                                    \
      static const int64_t slots = frame_slots(k_stft_mag_fwd<L, BS>, lds, BS);                           \
      const unsigned grid = frame_grid<L>(nf, iters, slots, FPBB);                                        \
      if (grid) hipLaunchKernelGGL((k_stft_mag_fwd<L, BS>), dim3(grid), dim3(BS), lds, s, x, a, window, pow_floor, \
                                   mag, iters);                                                           \
    } break;
    SEL_MAG_CASE(8)
    SEL_MAG_CASE(9)
    SEL_MAG_CASE(10)
    SEL_MAG_CASE(11)
#undef SEL_MAG_CASE
    default:
      ::sel::set_error("unsupported log2(n_fft)=%d", logn);
      return SEL_ERR_UNSUPPORTED;
  }
  SEL_LAUNCH_CHECK();
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
  if (logn < kMinLog || logn > kMaxLog - 1 || B < 0 || T < 0 || hop <= 0 || win_length <= 0) return 0;
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
  const int nb = int(t_last_frame_grid);  // one partial triple per block of that launch
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
  SEL_REQUIRE(n >= 0 && sums && out2, SEL_ERR_ARG, "n must be >= 0 (0: the count is sums[3])");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(k_stft_loss_finish, dim3(1), dim3(1), 0, s, sums, n ? 1.0 / double(n) : 0.0, out2);
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

int sel_stft_loss_coef(const double* sums, int64_t n, const float* g_sc, const float* g_mag,
                       float* coef, sel_stream_t stream) {
  SEL_REQUIRE(n >= 0 && sums && coef, SEL_ERR_ARG, "n must be >= 0 (0: the count is sums[3])");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(k_stft_loss_coef, dim3(1), dim3(1), 0, s, sums, n ? 1.0 / double(n) : 0.0, g_sc, g_mag,
                     coef);
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

int sel_logmel_fwd(const float* x, int64_t B, int64_t T, int n_fft, int hop, int win_length,
                   const float* window, const float* melmat, const int32_t* krange, int n_mels,
                   float eps, int log_kind, float* out, sel_stream_t stream) {
  int logn;
  if (int rc = check_frame(B, T, n_fft, hop, win_length, logn)) return rc;
  SEL_REQUIRE(n_mels > 0 && n_mels <= n_fft / 2 + 12, SEL_ERR_UNSUPPORTED,
              "n_mels=%d must be in (0, n_fft/2 + 12]", n_mels);
  SEL_REQUIRE(log_kind >= SEL_LOG_E && log_kind <= SEL_LOG_10, SEL_ERR_ARG, "bad log kind");
  const FrameArgs a = frame_args(B, T, n_fft, hop, win_length);
  SEL_REQUIRE(ru_region_ok(B * int64_t(n_mels) * a.F * 4), SEL_ERR_UNSUPPORTED,
              "log-mel output of %lld bytes past the 32-bit store range", (long long)(B * int64_t(n_mels) * a.F * 4));
  MelArgs ma{melmat, reinterpret_cast<const int2*>(krange), n_mels, eps, log_kind};
  const int64_t nf = B * a.F;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  switch (logn) {
#define SEL_LOGMEL_FWD_CASE(L)                                                                          \
    case L: {                                                                                           \
      using G = Geo<L>;                                                                                 \
      int iters;                                                                                        \
      const size_t lds = size_t(G::FPB) * G::PADN * sizeof(float2) + mel_lds_bytes(n_mels);             \
      const unsigned grid = frame_grid<L>(nf, iters, frame_slots(k_logmel_fwd<L>, lds));               \
      if (grid) hipLaunchKernelGGL(k_logmel_fwd<L>, dim3(grid), dim3(256), lds, s, x, a, window, ma, out, iters); \
    } break;
    SEL_LOGMEL_FWD_CASE(8)
    SEL_LOGMEL_FWD_CASE(9)
    SEL_LOGMEL_FWD_CASE(10)
    SEL_LOGMEL_FWD_CASE(11)
#undef SEL_LOGMEL_FWD_CASE
    default:
      ::sel::set_error("unsupported log2(n_fft)=%d", logn);
      return SEL_ERR_UNSUPPORTED;
  }
  SEL_LAUNCH_CHECK();
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

size_t sel_mel_l1_workspace(int64_t B, int64_t T, int n_fft, int hop, int win_length) {
  int logn = 0;
  while ((1 << logn) < n_fft) ++logn;
  if (logn < kMinLog || logn > kFftMaxLog || B < 0 || T < 0 || hop <= 0 || win_length <= 0) return 0;
  const size_t part = (size_t(n_blocks(logn, B * (1 + T / hop))) * sizeof(double) + 255) & ~size_t(255);
  return part + slab_bytes(B, T, hop, win_length);
}

int sel_mel_l1_fwd_grad(const float* x, const float* y, int64_t B, int64_t T, int n_fft, int hop, int win_length,
                        const float* window, const float* melmat, const int32_t* krange, const int32_t* mrange,
                        int n_mels, float eps, int log_kind, float* loss, float* g_x, void* ws, size_t ws_bytes,
                        sel_stream_t stream) {
  int logn;
  if (int rc = check_frame(B, T, n_fft, hop, win_length, logn)) return rc;
  SEL_REQUIRE(B > 0 && x && y && loss, SEL_ERR_ARG, "mel L1 needs a non-empty batch, x, y and loss");
  SEL_REQUIRE(n_mels > 0 && n_mels <= n_fft / 2 + 12, SEL_ERR_UNSUPPORTED,
              "n_mels=%d must be in (0, n_fft/2 + 12]", n_mels);
  SEL_REQUIRE(log_kind >= SEL_LOG_E && log_kind <= SEL_LOG_10, SEL_ERR_ARG, "bad log kind");
  SEL_REQUIRE(ws_bytes >= sel_mel_l1_workspace(B, T, n_fft, hop, win_length), SEL_ERR_WORKSPACE,
              "workspace too small");
  const FrameArgs a = frame_args(B, T, n_fft, hop, win_length);
  MelArgs ma{melmat, reinterpret_cast<const int2*>(mrange), n_mels, eps, log_kind};
  const int64_t nf = B * a.F;
  const double n = double(nf) * n_mels;  // elements of each log-mel tensor
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  double* part = static_cast<double*>(ws);
  float* slab = g_x ? reinterpret_cast<float*>(static_cast<char*>(ws) +
                                               ((size_t(n_blocks(logn, nf)) * sizeof(double) + 255) & ~size_t(255)))
                    : nullptr;
  const int glin = (n_mels + 3) / 4 * 4;
  unsigned grid = 0;
  switch (logn) {
#define SEL_MEL_L1_CASE(L)                                                                              \
    case L: {                                                                                           \
      using G = Geo<L>;                                                                                 \
      int iters;                                                                                        \
      const size_t lds = size_t(G::FPB) * (G::PADN * sizeof(float2) + size_t(glin) * sizeof(float)) +   \
                         mel_lds_bytes(n_mels) + size_t(G::M + 1) * sizeof(int2);                       \
      grid = frame_grid<L>(nf, iters, frame_slots(k_mel_l1<L>, lds));                                   \
      if (grid)                                                                                         \
        hipLaunchKernelGGL(k_mel_l1<L>, dim3(grid), dim3(256), lds, s, x, y, a, window, ma,             \
                           reinterpret_cast<const int2*>(krange), float(1.0 / n), part, slab, iters, glin); \
    } break;
    SEL_MEL_L1_CASE(8)
    SEL_MEL_L1_CASE(9)
    SEL_MEL_L1_CASE(10)
    SEL_MEL_L1_CASE(11)
#undef SEL_MEL_L1_CASE
    default:
      ::sel::set_error("unsupported log2(n_fft)=%d", logn);
      return SEL_ERR_UNSUPPORTED;
  }
  SEL_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_finish_partials, dim3(1), dim3(256), 0, s, part, int(grid), 1, nullptr, loss, 1.0 / n);
  SEL_LAUNCH_CHECK();
  return g_x ? ola(slab, a, g_x, s) : SEL_OK;
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
  // per-frame dL/dmel floats after the spectrum slots; iters is passed before it
  const int glin = (n_mels + 3) / 4 * 4;
  switch (logn) {
#define SEL_LOGMEL_BWD_CASE(L)                                                                          \
    case L: {                                                                                           \
      using G = Geo<L>;                                                                                 \
      int iters;                                                                                        \
      const size_t lds = size_t(G::FPB) * (G::PADN * sizeof(float2) + size_t(glin) * sizeof(float)) +   \
                         mel_lds_bytes(n_mels);                                                         \
      const unsigned grid = frame_grid<L>(nf, iters, frame_slots(k_logmel_bwd<L>, lds));               \
      if (grid)                                                                                         \
        hipLaunchKernelGGL(k_logmel_bwd<L>, dim3(grid), dim3(256), lds, s, x, a, window, ma,           \
                           reinterpret_cast<const int2*>(krange), g_out, ref, g_scale, g_mul, slab, iters, \
                           glin);                                                                       \
    } break;
    SEL_LOGMEL_BWD_CASE(8)
    SEL_LOGMEL_BWD_CASE(9)
    SEL_LOGMEL_BWD_CASE(10)
    SEL_LOGMEL_BWD_CASE(11)
#undef SEL_LOGMEL_BWD_CASE
    default:
      ::sel::set_error("unsupported log2(n_fft)=%d", logn);
      return SEL_ERR_UNSUPPORTED;
  }
  SEL_LAUNCH_CHECK();
  return ola(slab, a, g_x, s);
}

}  // extern "C"
