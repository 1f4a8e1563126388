// Semantics probe for the gfx950 lane-swap builtins (v_permlane16/32_swap_b32) used by the MFMA depthwise transposes.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned* out) {
  unsigned l = threadIdx.x;
  unsigned a = 1000 + l, b = 2000 + l;
  auto r32 = __builtin_amdgcn_permlane32_swap(a, b, false, false);
  auto r16 = __builtin_amdgcn_permlane16_swap(a, b, false, false);
  out[l] = r32[0]; out[64 + l] = r32[1]; out[128 + l] = r16[0]; out[192 + l] = r16[1];
}
int main() {
  unsigned* d; hipMalloc(&d, 256 * 4);
  k<<<1, 64>>>(d);
  unsigned h[256]; hipMemcpy(h, d, 1024, hipMemcpyDeviceToHost);
  for (int l : {0, 1, 15, 16, 17, 31, 32, 33, 47, 48, 63})
    printf("lane %2d: p32 first %u second %u | p16 first %u second %u\n", l, h[l], h[64 + l], h[128 + l], h[192 + l]);
  return 0;
}
