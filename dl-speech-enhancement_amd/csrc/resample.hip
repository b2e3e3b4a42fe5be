// On-device band-limited resampling for the data pipeline:
// dataloader/AudioDataset.py:25-36 calls torchaudio.functional.resample(audio,
// orig_sr, sr) with its defaults (sinc_interp_hann, lowpass_filter_width 6,
// rolloff 0.99).  torchaudio 2.1.1 (requirements.txt) is absent here; this is a
// restatement of its published algorithm (torchaudio/functional/functional.py
// _get_sinc_resample_kernel / _apply_sinc_resample_kernel):
//   g = gcd(orig, new); o = orig/g; n = new/g
//   base = min(o, n) * rolloff;  w = ceil(lowpass_filter_width * o / base)
//   taps i in [0, 2w + o): t(p, i) = (i - w)/o - p/n, p in [0, n)      (phase p)
//   t *= base; clamp to +-lpw; window = cos(pi t / (2 lpw))^2; t *= pi
//   K[p][i] = (t == 0 ? 1 : sin(t)/t) * window * base / o
//   y[f*n + p] = sum_i xpad[f*o + i] K[p][i],  xpad = (w zeros, x, w + o zeros)
//   output length ceil(n * len / o).
// The caller owns the tap table (sel_resample_kernel fills a host array; copy
// it to the device) like every other buffer of this ABI.
#include <algorithm>
#include <cmath>
#include <numeric>

#include "sel_common.h"

namespace sel {
namespace resample {

struct Plan {
  int o, n, w, taps;
};

Plan plan(int orig_freq, int new_freq, int lpw, float rolloff) {
  const int g = std::gcd(orig_freq, new_freq);
  Plan p;
  p.o = orig_freq / g;
  p.n = new_freq / g;
  const double base = double(std::min(p.o, p.n)) * double(rolloff);
  p.w = int(std::ceil(double(lpw) * double(p.o) / base));
  p.taps = 2 * p.w + p.o;
  return p;
}

// One thread per output sample: its phase's taps from LDS (or, for tables
// beyond 48 KB, e.g. 22.05 -> 24 kHz's 160 x 161, straight from L1/L2), its
// window of input samples through L1 (neighbouring outputs share them).
constexpr int kLdsTable = 12288;     // n * taps floats staged in LDS (48 KB)
constexpr int kMaxTable = 1 << 20;   // larger tables are read from the cache

template <bool LDS>
__global__ __launch_bounds__(256) void k_resample(const float* __restrict__ x, int64_t len, Plan p,
                                                  const float* __restrict__ table, int64_t out_len,
                                                  float* __restrict__ y) {
  extern __shared__ float taps_lds[];
  const float* taps = table;
  if constexpr (LDS) {
    const int tsize = p.n * p.taps;
    for (int i = threadIdx.x; i < tsize; i += blockDim.x) taps_lds[i] = table[i];
    __syncthreads();
    taps = taps_lds;
  }
  const int64_t wav = blockIdx.y;
  const int64_t j = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (j >= out_len) return;
  const int64_t f = j / p.n;
  const int ph = int(j - f * p.n);
  const float* xs = x + wav * len;
  const float* k = taps + ph * p.taps;
  const int64_t s0 = f * p.o - p.w;  // xpad index f*o + i  <->  x index f*o + i - w
  float acc = 0.f;
  if (s0 >= 0 && s0 + p.taps <= len) {
    for (int i = 0; i < p.taps; ++i) acc = fmaf(xs[s0 + i], k[i], acc);
  } else {
    for (int i = 0; i < p.taps; ++i) {
      const int64_t s = s0 + i;
      if (s >= 0 && s < len) acc = fmaf(xs[s], k[i], acc);
    }
  }
  y[wav * out_len + j] = acc;
}

}  // namespace resample
}  // namespace sel

using namespace sel;
using namespace sel::resample;

extern "C" {

int sel_resample_plan(int orig_freq, int new_freq, int lowpass_filter_width, float rolloff, int* phases,
                      int* taps) {
  SEL_REQUIRE(orig_freq > 0 && new_freq > 0, SEL_ERR_ARG, "sample rates must be > 0");
  SEL_REQUIRE(lowpass_filter_width > 0 && rolloff > 0.f && rolloff <= 1.f, SEL_ERR_ARG,
              "lowpass_filter_width must be > 0 and rolloff in (0, 1]");
  const Plan p = plan(orig_freq, new_freq, lowpass_filter_width, rolloff);
  SEL_REQUIRE(p.n * p.taps <= kMaxTable, SEL_ERR_UNSUPPORTED, "resampling ratio %d/%d needs %d taps (> %d)", p.n,
              p.o, p.n * p.taps, kMaxTable);
  if (phases) *phases = p.n;
  if (taps) *taps = p.taps;
  return SEL_OK;
}

int64_t sel_resample_out_len(int64_t len, int orig_freq, int new_freq) {
  const int g = std::gcd(orig_freq, new_freq);
  const int64_t o = orig_freq / g, n = new_freq / g;
  return (n * len + o - 1) / o;  // ceil(n * len / o)
}

/* host-side tap table [phases][taps] (fp32, computed in double, rounded once) */
int sel_resample_kernel(int orig_freq, int new_freq, int lowpass_filter_width, float rolloff, float* table) {
  int nph, ntaps;
  if (int rc = sel_resample_plan(orig_freq, new_freq, lowpass_filter_width, rolloff, &nph, &ntaps)) return rc;
  const Plan p = plan(orig_freq, new_freq, lowpass_filter_width, rolloff);
  const double base = double(std::min(p.o, p.n)) * double(rolloff);
  const double lpw = double(lowpass_filter_width);
  for (int ph = 0; ph < p.n; ++ph)
    for (int i = 0; i < p.taps; ++i) {
      double t = (double(i - p.w) / p.o - double(ph) / p.n) * base;
      t = std::min(lpw, std::max(-lpw, t));
      const double c = std::cos(t * M_PI / lpw / 2.0);
      const double win = c * c;
      t *= M_PI;
      const double s = t == 0.0 ? 1.0 : std::sin(t) / t;
      table[ph * p.taps + i] = float(s * win * base / p.o);
    }
  return SEL_OK;
}

int sel_resample(const float* x, int64_t n_wavs, int64_t len, int orig_freq, int new_freq, int lowpass_filter_width,
                 float rolloff, const float* table, float* y, sel_stream_t stream) {
  SEL_REQUIRE(initialized(), SEL_ERR_STATE, "sel_init() has not succeeded");
  int nph, ntaps;
  if (int rc = sel_resample_plan(orig_freq, new_freq, lowpass_filter_width, rolloff, &nph, &ntaps)) return rc;
  SEL_REQUIRE(n_wavs >= 0 && len > 0, SEL_ERR_ARG, "bad waveform shape (%lld, %lld)", (long long)n_wavs,
              (long long)len);
  SEL_REQUIRE(n_wavs <= 65535, SEL_ERR_UNSUPPORTED, "at most 65535 waveforms per call");
  const Plan p = plan(orig_freq, new_freq, lowpass_filter_width, rolloff);
  const int64_t out_len = sel_resample_out_len(len, orig_freq, new_freq);
  if (n_wavs == 0) return SEL_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  dim3 grid(unsigned((out_len + 255) / 256), unsigned(n_wavs));
  if (p.n * p.taps <= kLdsTable)
    hipLaunchKernelGGL(k_resample<true>, grid, dim3(256), size_t(p.n) * p.taps * sizeof(float), s, x, len, p, table,
                       out_len, y);
  else
    hipLaunchKernelGGL(k_resample<false>, grid, dim3(256), 0, s, x, len, p, table, out_len, y);
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

}  // extern "C"
