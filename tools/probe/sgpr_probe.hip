// Probe: does the carry-out SGPR of v_mad_u64_u32 limit its issue rate?  The same 8
// independent MAD chains with the carry-out in vcc (every MAD writes the same SGPR pair),
// in 8 distinct explicit SGPR pairs, and v_fma_f64 (no SGPR write) for reference, at 1, 2,
// 3 and 8 waves per SIMD.  Not product code.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define ITERS 16384
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void k_vcc(uint64_t* out, uint32_t a0, uint32_t b0) {
  uint64_t c0 = threadIdx.x, c1 = c0 + 1, c2 = c0 + 2, c3 = c0 + 3, c4 = c0 + 4, c5 = c0 + 5, c6 = c0 + 6, c7 = c0 + 7;
  uint32_t a = a0 + threadIdx.x, b = b0 ^ threadIdx.x;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(
        "v_mad_u64_u32 %0, vcc, %8, %9, %0\n\t"
        "v_mad_u64_u32 %1, vcc, %8, %9, %1\n\t"
        "v_mad_u64_u32 %2, vcc, %8, %9, %2\n\t"
        "v_mad_u64_u32 %3, vcc, %8, %9, %3\n\t"
        "v_mad_u64_u32 %4, vcc, %8, %9, %4\n\t"
        "v_mad_u64_u32 %5, vcc, %8, %9, %5\n\t"
        "v_mad_u64_u32 %6, vcc, %8, %9, %6\n\t"
        "v_mad_u64_u32 %7, vcc, %8, %9, %7\n\t"
        : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(c4), "+v"(c5), "+v"(c6), "+v"(c7)
        : "v"(a), "v"(b) : "vcc");
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = c0 + c1 + c2 + c3 + c4 + c5 + c6 + c7;
}

__global__ void k_sgprs(uint64_t* out, uint32_t a0, uint32_t b0) {
  uint64_t c0 = threadIdx.x, c1 = c0 + 1, c2 = c0 + 2, c3 = c0 + 3, c4 = c0 + 4, c5 = c0 + 5, c6 = c0 + 6, c7 = c0 + 7;
  uint32_t a = a0 + threadIdx.x, b = b0 ^ threadIdx.x;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(
        "v_mad_u64_u32 %0, s[40:41], %8, %9, %0\n\t"
        "v_mad_u64_u32 %1, s[42:43], %8, %9, %1\n\t"
        "v_mad_u64_u32 %2, s[44:45], %8, %9, %2\n\t"
        "v_mad_u64_u32 %3, s[46:47], %8, %9, %3\n\t"
        "v_mad_u64_u32 %4, s[48:49], %8, %9, %4\n\t"
        "v_mad_u64_u32 %5, s[50:51], %8, %9, %5\n\t"
        "v_mad_u64_u32 %6, s[52:53], %8, %9, %6\n\t"
        "v_mad_u64_u32 %7, s[54:55], %8, %9, %7\n\t"
        : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(c4), "+v"(c5), "+v"(c6), "+v"(c7)
        : "v"(a), "v"(b)
        : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53", "s54", "s55");
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = c0 + c1 + c2 + c3 + c4 + c5 + c6 + c7;
}

// two SGPR pairs alternating
__global__ void k_sgpr2(uint64_t* out, uint32_t a0, uint32_t b0) {
  uint64_t c0 = threadIdx.x, c1 = c0 + 1, c2 = c0 + 2, c3 = c0 + 3, c4 = c0 + 4, c5 = c0 + 5, c6 = c0 + 6, c7 = c0 + 7;
  uint32_t a = a0 + threadIdx.x, b = b0 ^ threadIdx.x;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(
        "v_mad_u64_u32 %0, s[40:41], %8, %9, %0\n\t"
        "v_mad_u64_u32 %1, s[42:43], %8, %9, %1\n\t"
        "v_mad_u64_u32 %2, s[40:41], %8, %9, %2\n\t"
        "v_mad_u64_u32 %3, s[42:43], %8, %9, %3\n\t"
        "v_mad_u64_u32 %4, s[40:41], %8, %9, %4\n\t"
        "v_mad_u64_u32 %5, s[42:43], %8, %9, %5\n\t"
        "v_mad_u64_u32 %6, s[40:41], %8, %9, %6\n\t"
        "v_mad_u64_u32 %7, s[42:43], %8, %9, %7\n\t"
        : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(c4), "+v"(c5), "+v"(c6), "+v"(c7)
        : "v"(a), "v"(b) : "s40", "s41", "s42", "s43");
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = c0 + c1 + c2 + c3 + c4 + c5 + c6 + c7;
}

__global__ void k_fma(double* out, double a0, double b0) {
  double c0 = threadIdx.x, c1 = c0 + 1, c2 = c0 + 2, c3 = c0 + 3, c4 = c0 + 4, c5 = c0 + 5, c6 = c0 + 6, c7 = c0 + 7;
  double a = a0 + threadIdx.x, b = b0 * threadIdx.x;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(
        "v_fma_f64 %0, %8, %9, %0\n\t"
        "v_fma_f64 %1, %8, %9, %1\n\t"
        "v_fma_f64 %2, %8, %9, %2\n\t"
        "v_fma_f64 %3, %8, %9, %3\n\t"
        "v_fma_f64 %4, %8, %9, %4\n\t"
        "v_fma_f64 %5, %8, %9, %5\n\t"
        "v_fma_f64 %6, %8, %9, %6\n\t"
        "v_fma_f64 %7, %8, %9, %7\n\t"
        : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(c4), "+v"(c5), "+v"(c6), "+v"(c7)
        : "v"(a), "v"(b));
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = c0 + c1 + c2 + c3 + c4 + c5 + c6 + c7;
}

template <typename F>
static float time_it(F launch) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  launch();
  hipDeviceSynchronize();
  hipEventRecord(a);
  for (int r = 0; r < 20; ++r) launch();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms / 20;
}

int main() {
  hipDeviceProp_t prop;
  CHK(hipGetDeviceProperties(&prop, 0));
  const int threads = 256;
  void* buf;
  CHK(hipMalloc(&buf, (size_t)prop.multiProcessorCount * 8 * threads * 8));
  for (int bpc : {1, 2, 3, 8}) {
    const int blocks = prop.multiProcessorCount * bpc;
    const double ops = (double)blocks * threads * ITERS * 8;
#define RUN(NAME, KER, T)                                                                                   \
  {                                                                                                         \
    float ms = time_it([&] { hipLaunchKernelGGL(KER, dim3(blocks), dim3(threads), 0, 0, (T*)buf, (T)3, (T)5); }); \
    printf("%d waves/SIMD %-10s %8.3f ms  %.1f lane-op/clk/CU (nominal clk)\n", bpc, NAME, ms,             \
           ops / (ms * 1e-3) / prop.multiProcessorCount / (prop.clockRate * 1e3));                          \
  }
    RUN("mad vcc", k_vcc, uint64_t)
    RUN("mad 8sgpr", k_sgprs, uint64_t)
    RUN("mad 2sgpr", k_sgpr2, uint64_t)
    RUN("fma_f64", k_fma, double)
  }
  CHK(hipFree(buf));
  return 0;
}
