// Verifies DPP lane-movement semantics used by mont27_dev.h (row_shl:1, row_shr:1,
// quad_perm broadcasts) on gfx950.  Not product code.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(int* o) {
  int x = 1000 + threadIdx.x;
  o[threadIdx.x] = __builtin_amdgcn_update_dpp(-1, x, 0x101, 0xf, 0xf, false);        // row_shl:1
  o[64 + threadIdx.x] = __builtin_amdgcn_update_dpp(-1, x, 0x111, 0xf, 0xf, false);   // row_shr:1
  o[128 + threadIdx.x] = __builtin_amdgcn_update_dpp(-1, x, 0x00, 0xf, 0xf, false);   // quad_perm [0,0,0,0]
  o[192 + threadIdx.x] = __builtin_amdgcn_update_dpp(-1, x, 0xA0, 0xf, 0xf, false);   // quad_perm [0,0,2,2]
  o[256 + threadIdx.x] = __builtin_amdgcn_update_dpp(-1, x, 0x101, 0xf, 0xf, true);   // row_shl:1 bound_ctrl
}
int main() {
  int* d; int h[320];
  (void)hipMalloc(&d, sizeof(h));
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  const char* nm[] = {"row_shl1", "row_shr1", "qp0000", "qp0022", "row_shl1_bc"};
  for (int t = 0; t < 5; ++t) {
    printf("%-12s", nm[t]);
    for (int l : {0, 1, 2, 3, 4, 14, 15, 16, 17, 31, 32, 63}) printf(" %d:%d", l, h[t * 64 + l]);
    printf("\n");
  }
  return 0;
}
