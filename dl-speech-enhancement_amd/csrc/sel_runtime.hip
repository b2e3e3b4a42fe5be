// Library-level state of libsel.so: error reporting, init, version.
#include <cmath>
#include <mutex>
#include <string>
#include <vector>

#include "sel_common.h"
#include "spectral_tables.h"

namespace sel {

static thread_local char g_err[1024] = "";
static std::once_flag g_once;
static int g_init_status = SEL_ERR_STATE;

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

bool initialized() { return g_init_status == SEL_OK; }

static int g_tune[16] = {0};
int tune(int key) { return (key >= 0 && key < 16) ? g_tune[key] : 0; }

static int do_init() {
  // FFT twiddles, computed in double on the host and rounded once to fp32.
  std::vector<float2> tw(spec::kTwTotal);
  for (int L = spec::kMinLog; L <= spec::kMaxLog; ++L) {
    const int N = 1 << L, M = N / 2;
    float2* twM = tw.data() + spec::tw_off(L);
    float2* twN = twM + M;
    for (int k = 0; k < M; ++k) {
      const double a = -2.0 * M_PI * double(k) / double(M);
      twM[k] = make_float2(float(std::cos(a)), float(std::sin(a)));
    }
    for (int k = 0; k <= M; ++k) {
      const double a = -2.0 * M_PI * double(k) / double(N);
      twN[k] = make_float2(float(std::cos(a)), float(std::sin(a)));
    }
  }
  for (int L = spec::kMinLog; L <= spec::kFftMaxLog; ++L) {
    for (int p = 1; p < spec::fft_npass(L); ++p) {
      const int R = spec::fft_radix(L, p), Ns = spec::fft_ns(L, p);
      float2* t = tw.data() + spec::twp_off(L, p);
      for (int k = 0; k < Ns; ++k)
        for (int r = 1; r < R; ++r) {
          const double a = -2.0 * M_PI * double(r) * double(k) / double(R * Ns);
          t[k * (R - 1) + r - 1] = make_float2(float(std::cos(a)), float(std::sin(a)));
        }
    }
  }
  SEL_HIP(spec::upload_twiddles(tw.data(), tw.size()));
  return SEL_OK;
}

}  // namespace sel

extern "C" {

int sel_init(void) {
  std::call_once(sel::g_once, [] { sel::g_init_status = sel::do_init(); });
  return sel::g_init_status;
}

const char* sel_last_error(void) { return sel::g_err; }

int sel_version(void) { return 1; }

int sel_tune(int key, int value) {
  if (key < 0 || key >= 16) return -1;
  const int prev = sel::g_tune[key];
  sel::g_tune[key] = value;
  return prev;
}

}  // extern "C"
