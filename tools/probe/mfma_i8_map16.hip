// Probe: operand/result lane maps of v_mfma_i32_16x16x64_i8 on gfx950 (exact integer check).
// Hypothesis: A: lane l holds A[row l&15][k = 16*(l>>4) + j] in byte j; B: B[k = 16*(l>>4) + j][col l&15];
//             C: lane l, register r holds C[row 4*(l>>4) + r][col l&15].
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

typedef int v4i __attribute__((ext_vector_type(4)));

__global__ void k(const int8_t* A, const int8_t* B, int* C) {
  const int l = threadIdx.x, r = l & 15, g = l >> 4;
  union { v4i v; int8_t b[16]; } a, bb;
  for (int j = 0; j < 16; ++j) {
    a.b[j] = A[r * 64 + 16 * g + j];
    bb.b[j] = B[(16 * g + j) * 16 + r];
  }
  v4i c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_i32_16x16x64_i8(a.v, bb.v, c, 0, 0, 0);
  for (int reg = 0; reg < 4; ++reg) C[(4 * g + reg) * 16 + r] = c[reg];
}

int main() {
  int8_t hA[16 * 64], hB[64 * 16];
  int hC[256], ref[256];
  srand(11);
  for (int i = 0; i < 1024; ++i) { hA[i] = (int8_t)(rand() % 255 - 127); hB[i] = (int8_t)(rand() % 255 - 127); }
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j) {
      int s = 0;
      for (int kk = 0; kk < 64; ++kk) s += hA[i * 64 + kk] * hB[kk * 16 + j];
      ref[i * 16 + j] = s;
    }
  int8_t *dA, *dB; int* dC;
  (void)hipMalloc(&dA, 1024); (void)hipMalloc(&dB, 1024); (void)hipMalloc(&dC, 1024);
  (void)hipMemcpy(dA, hA, 1024, hipMemcpyHostToDevice);
  (void)hipMemcpy(dB, hB, 1024, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dC);
  (void)hipMemcpy(hC, dC, 1024, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 256; ++i) if (hC[i] != ref[i]) { if (bad < 5) printf("mismatch %d,%d: %d vs %d\n", i / 16, i % 16, hC[i], ref[i]); ++bad; }
  printf("i8 16x16x64 map hypothesis: %s (%d mismatches)\n", bad ? "WRONG" : "OK", bad);
  return bad ? 1 : 0;
}
