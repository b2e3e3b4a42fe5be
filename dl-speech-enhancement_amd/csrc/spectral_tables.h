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
constexpr int kTwTotal = tw_off(kMaxLog + 1);

hipError_t upload_twiddles(const float2* host, size_t count);

}  // namespace spec
}  // namespace sel
