// Probe: Montgomery-product throughput of the real kernel code (mont_dev.h / mont2_dev.h)
// as a function of waves per SIMD.  Not product code.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include "mont2_dev.h"  // the round-1 32-bit two-lane engine, kept with the probe

using namespace fphe;

template <int L>
__global__ __launch_bounds__(256) void k_tpi1(const u32* __restrict__ N, u32 n0inv, u32* out, int reps) {
  extern __shared__ u32 lds[];
  const int lane = threadIdx.x & 63;
  const u32 wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  u32* slot = lds + wib * L * 64 + lane;
  u32 A[L];
#pragma unroll
  for (int j = 0; j < L; ++j) A[j] = (j == L - 1) ? 0u : (0x9e3779b9u * (threadIdx.x + 1) + j * 0x85ebca6bu);
#pragma unroll 1
  for (int r = 0; r < reps; ++r) mont_sqr<L>(A, slot, N, n0inv);
  u32 s = 0;
#pragma unroll
  for (int j = 0; j < L; ++j) s ^= A[j];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int LL>
__global__ __launch_bounds__(256) void k_tpi2(const u32* __restrict__ N, u32 n0inv, u32* out, int reps) {
  extern __shared__ u32 lds[];
  const int lane = threadIdx.x & 63, e = lane & 31, h = lane >> 5;
  const u32 wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  u32* bcol = lds + wib * (2 * LL * 32) + e;
  const u32 hoff = half_off<LL>(h);
  u32 NV[LL], A[LL];
#pragma unroll
  for (int j = 0; j < LL; ++j) {
    NV[j] = N[h * LL + j];
    A[j] = (h == 1 && j == LL - 1) ? 0u : (0x9e3779b9u * (threadIdx.x + 1) + j * 0x85ebca6bu);
  }
#pragma unroll 1
  for (int r = 0; r < reps; ++r) mont_sqr2<LL>(A, bcol, NV, n0inv, hoff);
  u32 s = 0;
#pragma unroll
  for (int j = 0; j < LL; ++j) s ^= A[j];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

static uint32_t neg_inv32(uint32_t m0) {
  uint32_t x = 1;
  for (int i = 0; i < 5; ++i) x *= 2u - m0 * x;
  return 0u - x;
}

template <typename K>
static void run(const char* name, K kern, int L, int tpi, size_t lds_per_block, int cus, const u32* N, u32 n0inv,
                u32* out) {
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_per_block);
  const int reps = 40;
  for (int bpc = 1; bpc <= 4; ++bpc) {
    if (lds_per_block * bpc > 160 * 1024) break;
    const int blocks = cus * bpc;
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), lds_per_block, 0, N, n0inv, out, 2);
    (void)hipDeviceSynchronize();
    hipEvent_t a, b;
    (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), lds_per_block, 0, N, n0inv, out, reps);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms; (void)hipEventElapsedTime(&ms, a, b);
    const double elems = (double)blocks * 256 / tpi;
    const double mac = elems * reps * (2.0 * L * L + L);
    printf("%-8s L=%3d tpi=%d blocks/CU=%d  %.3f ms  %.2f TMAC32/s  %.3e montmul/s\n", name, L, tpi, bpc, ms,
           mac / (ms * 1e-3) / 1e12, elems * reps / (ms * 1e-3));
  }
}

int main() {
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, 0);
  const int cus = prop.multiProcessorCount;
  std::vector<u32> hN(128);
  for (int j = 0; j < 128; ++j) hN[j] = 0x9e3779b1u * (j + 7) | 1u;
  hN[127] |= 0x80000000u;
  u32 *N, *out;
  (void)hipMalloc(&N, 128 * 4);
  (void)hipMalloc(&out, (size_t)cus * 4 * 256 * 4);
  (void)hipMemcpy(N, hN.data(), 128 * 4, hipMemcpyHostToDevice);
  const u32 ninv = neg_inv32(hN[0]);
  // modulus views: the top limb of each L-limb prefix is forced to have its top bit set
  run("tpi1", k_tpi1<32>, 32, 1, 4 * 32 * 64 * 4, cus, N, ninv, out);
  run("tpi1", k_tpi1<64>, 64, 1, 4 * 64 * 64 * 4, cus, N, ninv, out);
  run("tpi1", k_tpi1<128>, 128, 1, 4 * 128 * 64 * 4, cus, N, ninv, out);
  run("tpi2", k_tpi2<32>, 64, 2, 4 * 64 * 32 * 4, cus, N, ninv, out);
  run("tpi2", k_tpi2<64>, 128, 2, 4 * 128 * 32 * 4, cus, N, ninv, out);
  return 0;
}
