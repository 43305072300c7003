// Does gfx950 execute the GFX9 wavefront-wide DPP shifts (wave_shl:1 = 0x130, wave_shr:1 =
// 0x138)?  The assembler takes them; the one-element-per-wave kernel (fate_amd/csrc/
// wide_dev.h) would use them for its cross-lane hand-off instead of row_shl:1 plus
// v_readlane/v_writelane patches at the 16-lane row ends.
//   hipcc --offload-arch=gfx950 -O3 -o dpp_wave_probe dpp_wave_probe.hip && ./dpp_wave_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void k(int* o) {
  const int x = 100 + (int)threadIdx.x;
  o[threadIdx.x] = __builtin_amdgcn_update_dpp(0, x, 0x130, 0xf, 0xf, true);       // wave_shl:1
  o[64 + threadIdx.x] = __builtin_amdgcn_update_dpp(0, x, 0x138, 0xf, 0xf, true);  // wave_shr:1
}

int main() {
  int* d = nullptr;
  int h[128];
  if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 2;
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 2;
  int shl_next = 1, shr_prev = 1;
  for (int i = 0; i < 64; ++i) {
    if (h[i] != (i + 1 < 64 ? 100 + i + 1 : 0)) shl_next = 0;
    if (h[64 + i] != (i > 0 ? 100 + i - 1 : 0)) shr_prev = 0;
  }
  printf("wave_shl:1 lanes:");
  for (int i = 0; i < 64; ++i) printf(" %d", h[i]);
  printf("\nwave_shr:1 lanes:");
  for (int i = 0; i < 64; ++i) printf(" %d", h[64 + i]);
  printf("\nwave_shl:1 is lane i <- lane i+1: %s; wave_shr:1 is lane i <- lane i-1: %s\n", shl_next ? "yes" : "no",
         shr_prev ? "yes" : "no");
  return 0;
}
