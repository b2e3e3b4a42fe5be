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

constexpr int kTuneKeys = 128;
static int g_tune[kTuneKeys] = {0};
int tune(int key) { return (key >= 0 && key < kTuneKeys) ? g_tune[key] : 0; }

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
  if (key < 0 || key >= sel::kTuneKeys) return -1;
  const int prev = sel::g_tune[key];
  sel::g_tune[key] = value;
  return prev;
}

int sel_tune_get(int key) { return (key >= 0 && key < sel::kTuneKeys) ? sel::g_tune[key] : -1; }

}  // extern "C"

// ---------------------------------------------------------------------------
// Probe behind spectral.hip's frame loads (tests/test_gpu_spectral.py):
// out[2i], out[2i+1] = the pair a raw_buffer_load_b64 returns at byte offset 4i
// of x, through the same buffer resource the STFT kernels build (num_records
// n*4, word3 0x00020000 = CK's gfx9 value).  mode 0 takes the two dwords out of
// the returned vector as scalars; mode 1 writes __builtin_bit_cast(float, v[1])
// — the form round 1 used.  ROCm 7.2's clang lowers a bit_cast of an
// ext_vector ELEMENT lvalue to a load from the vector's base address, so mode 1
// returns element 0 twice (one buffer_load_dword + v_mov in the ISA): that, not
// the hardware or the descriptor, was the "wrong pairs" of the r1 workaround.
// ---------------------------------------------------------------------------
namespace {
typedef unsigned int probe_u2 __attribute__((ext_vector_type(2)));
__global__ void k_probe_buffer_b64(const float* __restrict__ x, int n, int mode, float* __restrict__ out) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(x), 0, n * 4, 0x00020000);
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i + 1 < n; i += gridDim.x * blockDim.x) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b64(r, i * 4, 0, 0);
    if (mode == 0) {
      const probe_u2 u = v;
      const unsigned e0 = u.x, e1 = u.y;
      out[2 * i] = __builtin_bit_cast(float, e0);
      out[2 * i + 1] = __builtin_bit_cast(float, e1);
    } else {
      out[2 * i] = __builtin_bit_cast(float, v[0]);
      out[2 * i + 1] = __builtin_bit_cast(float, v[1]);
    }
  }
}
}  // namespace

extern "C" int sel_probe_buffer_b64(const float* x, int n, int mode, float* out, sel_stream_t stream) {
  SEL_REQUIRE(x && out && n >= 2 && n < (1 << 28) && (mode == 0 || mode == 1), SEL_ERR_ARG, "bad probe arguments");
  hipLaunchKernelGGL(k_probe_buffer_b64, dim3((n + 255) / 256), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     x, n, mode, out);
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}

// ---------------------------------------------------------------------------
// Measurement denominator for the STFT roofline (bench.py stft_kernel): a
// float4 stream copy, 4 independent 16-B loads in flight per thread, one
// resident round of workgroups striding over the buffer (the guide's
// "measured copy" shape), so a kernel's GB/s can be set against what this box's
// HBM sustains for a plain read + write of the same bytes.
// ---------------------------------------------------------------------------
namespace {
// grid-stride form (mode 1, the round-1 probe): 4 x 16-B loads in flight per thread
__global__ __launch_bounds__(256) void k_probe_copy_f4(const float4* __restrict__ src, float4* __restrict__ dst,
                                                       int64_t n) {
  const int64_t stride = int64_t(gridDim.x) * 256 * 4;
  for (int64_t i = int64_t(blockIdx.x) * 256 * 4 + threadIdx.x; i < n; i += stride) {
    float4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (i + u * 256 < n) v[u] = src[i + u * 256];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (i + u * 256 < n) dst[i + u * 256] = v[u];
  }
}
// one-shot form (default): every workgroup copies one contiguous 256 x U x 16-B
// piece (no loop, U loads in flight per thread), the grid covers the buffer;
// NT: nontemporal loads and stores (the copied bytes are not re-read)
template <int U, bool NT>
__global__ __launch_bounds__(256) void k_probe_copy_once(const float4* __restrict__ src, float4* __restrict__ dst,
                                                         int64_t n) {
  const int64_t i = int64_t(blockIdx.x) * 256 * U + threadIdx.x;
  float4 v[U];
  // every workgroup but the last: loads with no per-element guard (a guarded
  // load compiles to a branch with its own vmcnt(0): the loads then go out one
  // at a time)
  if (int64_t(blockIdx.x + 1) * 256 * U <= n) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (NT) {
        const float4* p = src + i + u * 256;
        v[u] = make_float4(__builtin_nontemporal_load(&p->x), __builtin_nontemporal_load(&p->y),
                           __builtin_nontemporal_load(&p->z), __builtin_nontemporal_load(&p->w));
      } else {
        v[u] = src[i + u * 256];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (NT) {
        float4* p = dst + i + u * 256;
        __builtin_nontemporal_store(v[u].x, &p->x);
        __builtin_nontemporal_store(v[u].y, &p->y);
        __builtin_nontemporal_store(v[u].z, &p->z);
        __builtin_nontemporal_store(v[u].w, &p->w);
      } else {
        dst[i + u * 256] = v[u];
      }
    }
    return;
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if (i + u * 256 < n) {
      if (NT) {
        const float4* p = src + i + u * 256;
        v[u] = make_float4(__builtin_nontemporal_load(&p->x), __builtin_nontemporal_load(&p->y),
                           __builtin_nontemporal_load(&p->z), __builtin_nontemporal_load(&p->w));
      } else {
        v[u] = src[i + u * 256];
      }
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if (i + u * 256 < n) {
      if (NT) {
        float4* p = dst + i + u * 256;
        __builtin_nontemporal_store(v[u].x, &p->x);
        __builtin_nontemporal_store(v[u].y, &p->y);
        __builtin_nontemporal_store(v[u].z, &p->z);
        __builtin_nontemporal_store(v[u].w, &p->w);
      } else {
        dst[i + u * 256] = v[u];
      }
    }
  }
}
}  // namespace

// mode (tune key 49), 1 GiB each way, tools/copy_probe.py (two runs):
//   0 (default) = one-shot, one 16-B piece per thread, nontemporal: 6.40 TB/s
//   1 = the grid-stride form over `blocks` workgroups (the round-1..4 probe,
//       4.7-5.1 TB/s at 4-32 blocks per CU)
//   2 / 3 = one-shot, 8 pieces per thread, plain / nontemporal (5.44-5.49 / 5.83)
//   4 = one-shot, 4 per thread, plain (5.72-5.77)
//   5 / 6 / 7 = one-shot, 2 / 4 / 16 per thread, nontemporal (6.00-6.03 /
//       5.97-6.03 / 5.08-5.15)
extern "C" int sel_probe_copy_f4(const void* src, void* dst, int64_t n16, int blocks, sel_stream_t stream) {
  SEL_REQUIRE(src && dst && n16 > 0 && blocks > 0, SEL_ERR_ARG, "bad copy probe arguments");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const float4* in = static_cast<const float4*>(src);
  float4* out = static_cast<float4*>(dst);
  const int mode = sel::tune(49);
  // the one-shot forms' grid of (n16 / (256 U)) workgroups must fit the
  // unsigned grid dimension for the U actually launched (U >= 1: checked at U = 1)
  SEL_REQUIRE((n16 + 255) / 256 < (int64_t(1) << 31), SEL_ERR_ARG, "copy probe buffer too large");
  auto once = [&](auto kern, int U) {
    const int64_t g = (n16 + 256 * U - 1) / (256 * U);
    hipLaunchKernelGGL(kern, dim3(unsigned(g)), dim3(256), 0, s, in, out, n16);
  };
  switch (mode) {
    case 1: hipLaunchKernelGGL(k_probe_copy_f4, dim3(unsigned(blocks)), dim3(256), 0, s, in, out, n16); break;
    case 2: once(k_probe_copy_once<8, false>, 8); break;
    case 3: once(k_probe_copy_once<8, true>, 8); break;
    case 4: once(k_probe_copy_once<4, false>, 4); break;
    case 5: once(k_probe_copy_once<2, true>, 2); break;
    case 6: once(k_probe_copy_once<4, true>, 4); break;
    case 7: once(k_probe_copy_once<16, true>, 16); break;
    default: once(k_probe_copy_once<1, true>, 1); break;
  }
  SEL_LAUNCH_CHECK();
  return SEL_OK;
}
