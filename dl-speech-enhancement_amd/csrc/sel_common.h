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
