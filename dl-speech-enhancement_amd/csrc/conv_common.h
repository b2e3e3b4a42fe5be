// Helpers shared by the conv-stack translation units (conv.hip, conv_wss.hip).
#pragma once
#include "sel_common.h"

namespace sel {
namespace conv {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float to_f(float v) { return v; }
__device__ __forceinline__ float to_f(__bf16 v) { return float(v); }
template <typename T> __device__ __forceinline__ T from_f(float v);
template <> __device__ __forceinline__ float from_f<float>(float v) { return v; }
template <> __device__ __forceinline__ __bf16 from_f<__bf16>(float v) { return __bf16(v); }

__device__ __forceinline__ float elu(float v) { return v > 0.f ? v : expm1f(v); }
__device__ __forceinline__ float elu_grad(float v) { return v > 0.f ? 1.f : expf(v); }
// bf16 path: the result is rounded to bf16 (8-bit mantissa), so the hardware
// exp (v_exp_f32, a few ulp of fp32) replaces the libm expm1/exp range reduction.
__device__ __forceinline__ float elu_fast(float v) { return v > 0.f ? v : __expf(v) - 1.f; }
// v > 0 ? 1 : exp(v) as one min: exp(v) >= 1 exactly when v >= 0 (monotone
// hardware exp, exp(0) = 1), so the result is bit-identical to the select
__device__ __forceinline__ float elu_grad_fast(float v) { return fminf(__expf(v), 1.f); }

// elu_fast over 8 bf16 (round-to-nearest back to bf16), with the log2(e) scale
// and the -1 as packed fp32 ops: per element the same arithmetic as elu_fast
// (exp(v) = v_exp_f32(v * log2 e), as __expf lowers), so bit-identical
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint4 elu8(uint4 w) {
  const unsigned in[4] = {w.x, w.y, w.z, w.w};
  unsigned o[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const f32x2 f = {__uint_as_float(in[q] << 16), __uint_as_float(in[q] & 0xffff0000u)};
    const f32x2 t = f * 1.44269502f;
    f32x2 e = {__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)};
    e = e - 1.f;
    // x > 0 ? x : e as ONE v_med3_f32 (median of x, e, 0): for x > 0, e > x > 0;
    // for x <= 0, x <= e <= 0 (e^x >= 1 + x) — the same value as the select
    // for every input but -0.0 (the select gives +0 = e, med3 -0 or +0: equal)
    const f32x2 r = {__builtin_amdgcn_fmed3f(f.x, e.x, 0.f), __builtin_amdgcn_fmed3f(f.y, e.y, 0.f)};
    o[q] = __builtin_bit_cast(unsigned, __builtin_convertvector(r, bf16x2));  // v_cvt_pk_bf16_f32
  }
  return make_uint4(o[0], o[1], o[2], o[3]);
}

struct Args {
  int64_t rows;
  int T, C, N, K, dil, pad, pad_mode, in_elu, bias_period;
  // discriminator layers on the warp-specialised kernel (sel_dconv_desc; the
  // generator's own descriptors set tin_valid = tin_pitch = tout_valid = T,
  // ldx = C, ldo = N, epi = 0): input rows valid / allocated per sequence and
  // row pitches, output rows computed per sequence (later rows written as
  // zeros), epilogue 1 = (v + bias + res) * LeakyReLU'(aux), LeakyReLU if act
  int tin_valid, tin_pitch, ldx, ldo, tout_valid, epi, act;
  float slope;
  // > 0: flat tiling of all sequences' rows as one row space (equal input and
  // output pitch seq_pitch, zero gaps between sequences): input rows valid where
  // row % seq_pitch < tin_valid, outputs where row % seq_pitch < tout_valid
  int seq_pitch;
};

typedef float floatx16 __attribute__((ext_vector_type(16)));
constexpr int F4_HALOMAX = 64;

// XCD-aware block order for multi-column-tile launches (1-D grid of
// row tiles x ncol): workgroups are dealt round-robin over the 8 XCDs, so the
// ncol column tiles of one row tile are given ids 8 apart (one XCD, adjacent in
// that XCD's dispatch order) and share the input tile through its L2 instead
// of each XCD fetching it from HBM.  ncol == 0 means a 2-D (row, column) grid.
__device__ __forceinline__ void xcd_tile(int ncol, int64_t& mt, int& nt) {
  if (ncol == 0) {
    mt = blockIdx.x;
    nt = blockIdx.y;
    return;
  }
  const int64_t L = blockIdx.x;
  const int64_t mtiles = int64_t(gridDim.x) / ncol;
  const int64_t full = (mtiles / 8) * 8 * ncol;
  if (L < full) {
    const int64_t q = L >> 3;
    nt = int(q % ncol);
    mt = (q / ncol) * 8 + (L & 7);
  } else {
    const int64_t r = L - full;
    nt = int(r % ncol);
    mt = (mtiles / 8) * 8 + r / ncol;
  }
}

// s_waitcnt vmcnt(N) alone (expcnt / lgkmcnt left at their no-wait maxima)
template <int N>
__device__ __forceinline__ void ws_wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

typedef __attribute__((address_space(3))) void* lds_ptr_t;

}  // namespace conv
}  // namespace sel

namespace sel {
namespace conv {
// conv_wss.hip: sample-tile warp-specialised kernel (T <= 400)
bool wss_geometry(const Args& a, int& S, int& tm, int& BN);  // strips per tile, tile rows, channels
bool wss_geometry(const Args& a, int& S, int& tm);
bool wss_ok(const Args& a);
int wss_spt(const Args& a);  // samples per sample-tile (1, or 400 / T for short T)
bool wss_pw_ok(const Args& a);  // the fused RU128 forward on k_conv_wss (PW epilogue)
int launch_wss_pw(const Args& a, const void* x, const void* w1, const float* b1, const void* w2, const float* b2,
                  void* h, void* out, hipStream_t s);
bool wss_ok_out(const Args& a, bool out_f32);  // wss_ok and an instance for that output type
template <typename TO>
int launch_wss(const Args& a, const void* in, const void* wp, const float* bias, const void* aux, const void* res,
               void* out, hipStream_t s);
}  // namespace conv
}  // namespace sel
