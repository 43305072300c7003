// Determines v_permlane32_swap_b32 operand semantics on gfx950 (which operand's low half
// is exchanged with which operand's high half).  Not product code.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned* o) {
  unsigned a = 100 + threadIdx.x, b = 200 + threadIdx.x;
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1\n\ts_nop 1" : "+v"(a), "+v"(b));
  o[threadIdx.x] = a; o[64 + threadIdx.x] = b;
}
int main() {
  unsigned* d; unsigned h[128];
  (void)hipMalloc(&d, 512);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  (void)hipMemcpy(h, d, 512, hipMemcpyDeviceToHost);
  printf("vdst lanes 0,31,32,63: %u %u %u %u\n", h[0], h[31], h[32], h[63]);
  printf("vsrc lanes 0,31,32,63: %u %u %u %u\n", h[64], h[95], h[96], h[127]);
  return 0;
}
