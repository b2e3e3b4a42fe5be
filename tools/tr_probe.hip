// Probe of ds_read_b64_tr_b16 lane semantics on gfx950 (debug tool, not product).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef short v4i16 __attribute__((ext_vector_type(4)));
__global__ void k(short* out) {
  __shared__ short lds[4 * 64];  // 4 rows x 64 cols
  for (int i = threadIdx.x; i < 256; i += 64) lds[i] = short(i);  // value = row*64 + col
  __syncthreads();
  const int l = threadIdx.x, g = l >> 4, i = l & 15, q = i >> 2, p = i & 3;
  // group g reads rows 0..3, columns 16g .. 16g+15 ; lane 4q+p supplies row q, col 16g+4p
  v4i16 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) v4i16*)(lds + q * 64 + 16 * g + 4 * p));
  for (int e = 0; e < 4; ++e) out[l * 4 + e] = v[e];
}
int main() {
  short* d;
  hipMalloc(&d, 256 * 2);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  short h[256];
  hipMemcpy(h, d, 512, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int l = 0; l < 64; ++l) {
    const int g = l >> 4, i = l & 15;
    for (int e = 0; e < 4; ++e) {
      const int expect = e * 64 + 16 * g + i;  // row e, column 16g+i
      if (h[l * 4 + e] != expect) ++bad;
    }
  }
  printf("lane0: %d %d %d %d  lane5: %d %d %d %d  lane17: %d %d %d %d\n", h[0], h[1], h[2], h[3], h[20], h[21],
         h[22], h[23], h[68], h[69], h[70], h[71]);
  printf("tr16 probe: %s (%d mismatches)\n", bad ? "MISMATCH" : "OK (lane i of group gets column i, row e in element e)", bad);
  return 0;
}
