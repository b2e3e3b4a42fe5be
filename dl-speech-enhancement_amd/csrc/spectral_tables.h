// FFT twiddle-table layout shared by sel_runtime.hip (host fill) and spectral.hip.
#pragma once
#include <hip/hip_runtime.h>

namespace sel {
namespace spec {

// n_fft = 2^L, L in [kMinLog, kMaxLog].  Per L: twM[M] = exp(-2 pi i k / M)
// (the half-size complex FFT), then twN[M+1] = exp(-2 pi i k / N) (real-FFT
// split), M = N/2.
constexpr int kMinLog = 8;
constexpr int kMaxLog = 12;

__host__ __device__ constexpr int tw_off(int L) {
  return ((1 << L) - (1 << kMinLog)) + (L - kMinLog);
}
constexpr int kTwBase = tw_off(kMaxLog + 1);

// Wave-FFT radix schedule of the half-size (M = N/2) complex FFT: PPL = 8
// points per lane, a frame on M/8 lanes (one wave up to n_fft 1024, two at
// 2048), Stockham passes of radix R0..R(NP-1): 8*8*{2,4,8} for n_fft 256..1024
// and 8*8*8*2 for 2048.  Pass p > 0 uses per-pass twiddles
// twp[k*(R-1) + r-1] = exp(-2 pi i r k / (R*Ns)), k < Ns = R0*..*R(p-1).
__host__ __device__ constexpr int fft_ppl(int) { return 8; }
__host__ __device__ constexpr int fft_npass(int L) { return L >= 11 ? 4 : 3; }
__host__ __device__ constexpr int fft_radix(int L, int p) {
  return p < 2 ? 8 : (p == 2 ? (L == 8 ? 2 : (L == 9 ? 4 : 8)) : (p == 3 && L >= 11 ? 2 : 1));
}
__host__ __device__ constexpr int fft_ns(int L, int p) {
  return p == 0 ? 1 : fft_ns(L, p - 1) * fft_radix(L, p - 1);
}
__host__ __device__ constexpr int twp_size(int L, int p) { return fft_ns(L, p) * (fft_radix(L, p) - 1); }
__host__ __device__ constexpr int twp_lsize(int L) { return twp_size(L, 1) + twp_size(L, 2) + twp_size(L, 3); }
__host__ __device__ constexpr int twp_loff(int L) { return L == kMinLog ? kTwBase : twp_loff(L - 1) + twp_lsize(L - 1); }
__host__ __device__ constexpr int twp_off(int L, int p) {  // p in {1, 2, 3}
  return twp_loff(L) + (p >= 2 ? twp_size(L, 1) : 0) + (p >= 3 ? twp_size(L, 2) : 0);
}
constexpr int kFftMaxLog = 11;  // largest n_fft the wave FFT serves (2048)
constexpr int kTwTotal = twp_loff(kFftMaxLog) + twp_lsize(kFftMaxLog);

hipError_t upload_twiddles(const float2* host, size_t count);

}  // namespace spec
}  // namespace sel
