// Probe: operand/result lane maps of v_mfma_i32_32x32x32_i8 on gfx950, checked with exact
// integer data against a host matmul (A and B asymmetric).  Hypothesis under test:
//   A: lane l holds A[row l&31][k = 16*(l>>5) + j] in byte j (j = 0..15) of its 16-byte fragment
//   B: lane l holds B[k = 16*(l>>5) + j][col l&31] in byte j
//   C: lane l, register r holds C[row (r&3) + 8*(r>>2) + 4*(l>>5)][col l&31]
// hipcc --offload-arch=gfx950 -O3 -o /tmp/mfma_i8_map tools/probe/mfma_i8_map.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

__global__ void k(const int8_t* A, const int8_t* B, int* C) {
  const int l = threadIdx.x, r = l & 31, h = l >> 5;
  union { v4i v; int8_t b[16]; } a, bb;
  for (int j = 0; j < 16; ++j) {
    a.b[j] = A[r * 32 + 16 * h + j];
    bb.b[j] = B[(16 * h + j) * 32 + r];
  }
  v16i c = {0};
  c = __builtin_amdgcn_mfma_i32_32x32x32_i8(a.v, bb.v, c, 0, 0, 0);
  for (int reg = 0; reg < 16; ++reg) {
    const int row = (reg & 3) + 8 * (reg >> 2) + 4 * h;
    C[row * 32 + r] = c[reg];
  }
}

int main() {
  int8_t hA[32 * 32], hB[32 * 32];
  int hC[32 * 32], ref[32 * 32];
  srand(7);
  for (int i = 0; i < 1024; ++i) { hA[i] = (int8_t)(rand() % 255 - 127); hB[i] = (int8_t)(rand() % 255 - 127); }
  for (int i = 0; i < 32; ++i)
    for (int j = 0; j < 32; ++j) {
      int s = 0;
      for (int kk = 0; kk < 32; ++kk) s += hA[i * 32 + kk] * hB[kk * 32 + j];
      ref[i * 32 + j] = s;
    }
  int8_t *dA, *dB; int* dC;
  hipMalloc(&dA, 1024); hipMalloc(&dB, 1024); hipMalloc(&dC, 4096);
  hipMemcpy(dA, hA, 1024, hipMemcpyHostToDevice);
  hipMemcpy(dB, hB, 1024, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dC);
  hipMemcpy(hC, dC, 4096, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 1024; ++i) if (hC[i] != ref[i]) { if (bad < 5) printf("mismatch at %d,%d: %d vs %d\n", i / 32, i % 32, hC[i], ref[i]); ++bad; }
  printf("i8 32x32x32 map hypothesis: %s (%d mismatches)\n", bad ? "WRONG" : "OK", bad);
  return bad ? 1 : 0;
}
