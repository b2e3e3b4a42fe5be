// Shared helpers for libsel.so (gfx950 only; no CUDA, no dual paths).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <cstdarg>
#include <cstdint>
#include <cstdio>

#include "../../include/sel.h"

namespace sel {

void set_error(const char* fmt, ...);
bool initialized();
int tune(int key);

constexpr int kWave = 64;

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Block-wide sum for blockDim.x a multiple of 64 (<= 1024).  `red` needs >= 16 slots.
template <typename T>
__device__ __forceinline__ T block_sum(T v, T* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  T s = 0;
  if (threadIdx.x < 64) {
    s = (threadIdx.x < (blockDim.x >> 6)) ? red[threadIdx.x] : T(0);
    s = wave_sum(s);
  }
  return s;  // valid in thread 0 (and the whole first wave)
}

// Branch-free staging loads for the persistent tile loops: a bf16 tensor
// region as a buffer resource (bytes <= RU_OOB: ru_region_ok, checked by the dispatch predicates)
// and a 16-B load from it.  RU_OOB is past any region's bytes, so a load there
// returns zeros and touches no memory: rows outside the sample / span and a
// dead next-tile request take it instead of a branch around the load, and the
// compiler then counts the request exactly (a conditional request makes every
// later wait on an earlier load fall back to vmcnt(0) behind it).
constexpr int RU_OOB = 0x7ffffff0;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t ru_rsrc(const __bf16* base, int64_t elems) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<__bf16*>(base), 0, int(elems * 2), 0x00020000);
}
__device__ __forceinline__ uint4 ru_bload(__amdgpu_buffer_rsrc_t rs, int byte_off) {
  return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, byte_off, 0, 0));
}
// Host-side predicate of every dispatch that builds such a resource: the
// region's bytes must end at or before RU_OOB, so an RU_OOB request lies past
// it (a region reaching into [RU_OOB, 2^31) would turn a dead request into a
// real load).
inline bool ru_region_ok(int64_t bytes) { return bytes >= 0 && bytes <= RU_OOB; }

}  // namespace sel

#define SEL_REQUIRE(cond, code, ...)      \
  do {                                    \
    if (!(cond)) {                        \
      ::sel::set_error(__VA_ARGS__);      \
      return (code);                      \
    }                                     \
  } while (0)

#define SEL_HIP(expr)                                                                   \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess) {                                                             \
      ::sel::set_error("%s:%d %s -> %s", __FILE__, __LINE__, #expr, hipGetErrorString(e_)); \
      return SEL_ERR_HIP;                                                               \
    }                                                                                   \
  } while (0)

#define SEL_LAUNCH_CHECK() SEL_HIP(hipGetLastError())
