// Step-0 probe: integer-MAD vs FP64-FMA issue rates on gfx950.
// Decides the limb arithmetic of the modexp kernels. Not product code.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define ITERS 16384
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int CHAINS>
__global__ void k_mad_u64(uint64_t* out, uint32_t a0, uint32_t b0) {
  uint64_t acc[CHAINS];
  uint32_t a = a0 + threadIdx.x, b = b0 ^ threadIdx.x;
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) acc[c] = c + threadIdx.x;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c)
      asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc[c]) : "v"(a), "v"(b) : "vcc");
  }
  uint64_t s = 0;
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) s += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int CHAINS>
__global__ void k_fma_f64(double* out, double a0, double b0) {
  double acc[CHAINS];
  double a = a0 + threadIdx.x, b = b0 * threadIdx.x;
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) acc[c] = c + threadIdx.x;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c)
      asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(acc[c]) : "v"(a), "v"(b));
  }
  double s = 0;
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) s += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int CHAINS>
__global__ void k_mul_lo(uint32_t* out, uint32_t a0, uint32_t b0) {
  uint32_t acc[CHAINS];
  uint32_t b = b0 ^ threadIdx.x;
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) acc[c] = c + threadIdx.x + a0;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c)
      asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(acc[c]) : "v"(b));
  }
  uint32_t s = 0;
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) s += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int CHAINS>
__global__ void k_mul_hi(uint32_t* out, uint32_t a0, uint32_t b0) {
  uint32_t acc[CHAINS];
  uint32_t b = b0 ^ threadIdx.x;
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) acc[c] = c + threadIdx.x + a0;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c)
      asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(acc[c]) : "v"(b));
  }
  uint32_t s = 0;
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) s += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int CHAINS>
__global__ void k_mad_u24(uint32_t* out, uint32_t a0, uint32_t b0) {
  uint32_t acc[CHAINS];
  uint32_t a = (a0 + threadIdx.x) & 0xffffff, b = (b0 ^ threadIdx.x) & 0xffffff;
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) acc[c] = c + threadIdx.x;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c)
      asm volatile("v_mad_u32_u24 %0, %1, %2, %0" : "+v"(acc[c]) : "v"(a), "v"(b));
  }
  uint32_t s = 0;
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) s += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int CHAINS>
__global__ void k_addc(uint32_t* out, uint32_t a0, uint32_t b0) {
  uint32_t acc[CHAINS];
  uint32_t b = b0 ^ threadIdx.x;
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) acc[c] = c + threadIdx.x + a0;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c)
      asm volatile("v_addc_co_u32 %0, vcc, %0, %1, vcc" : "+v"(acc[c]) : "v"(b) : "vcc");
  }
  uint32_t s = 0;
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) s += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}


template <int CHAINS>
__global__ void k_add_u32(uint32_t* out, uint32_t a0, uint32_t b0) {
  uint32_t acc[CHAINS];
  uint32_t b = b0 ^ threadIdx.x;
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) acc[c] = c + threadIdx.x + a0;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c)
      asm volatile("v_add_u32 %0, %0, %1" : "+v"(acc[c]) : "v"(b));
  }
  uint32_t s = 0;
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) s += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
template <int CHAINS>
__global__ void k_mad_u64_sep(uint64_t* out, uint32_t a0, uint32_t b0) {
  // each chain with its own carry-out SGPR pair
  uint64_t acc[CHAINS];
  uint32_t a = a0 + threadIdx.x, b = b0 ^ threadIdx.x;
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) acc[c] = c + threadIdx.x;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) {
      uint64_t cc;
      asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc[c]), "=s"(cc) : "v"(a), "v"(b));
    }
  }
  uint64_t s = 0;
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) s += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename F>
static float time_it(F launch) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  launch();
  hipDeviceSynchronize();
  hipEventRecord(a);
  for (int r = 0; r < 20; ++r) launch();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  return ms / 20;
}

int main() {
  hipDeviceProp_t prop;
  CHK(hipGetDeviceProperties(&prop, 0));
  printf("device %s CUs=%d clock=%d kHz\n", prop.gcnArchName, prop.multiProcessorCount, prop.clockRate);
  const int threads = 256;
  void* buf; CHK(hipMalloc(&buf, (size_t)prop.multiProcessorCount * 8 * threads * 8));
  for (int bpc : {8, 1}) {
  const int blocks = prop.multiProcessorCount * bpc;
  printf("--- %d blocks/CU of 256 threads (%d waves/SIMD)\n", bpc, bpc);
  const double total_lane_ops_per_chain = (double)blocks * threads * ITERS;
#define RUN(NAME, KER, T, CH) { \
    float ms = time_it([&] { hipLaunchKernelGGL((KER<CH>), dim3(blocks), dim3(threads), 0, 0, (T*)buf, (T)3, (T)5); }); \
    double ops = total_lane_ops_per_chain * CH; \
    double per_cu_clk = ops / (ms * 1e-3) / prop.multiProcessorCount / (prop.clockRate * 1e3); \
    printf("%-16s chains=%2d  %8.3f ms  %.3e lane-op/s  %.1f lane-op/clk/CU (nominal clk)\n", NAME, CH, ms, ops / (ms * 1e-3), per_cu_clk); }
  RUN("v_add_u32", k_add_u32, uint32_t, 8)
  RUN("v_mad_u32_u24", k_mad_u24, uint32_t, 8)
  RUN("v_mad_u64_u32", k_mad_u64, uint64_t, 1)
  RUN("v_mad_u64_u32", k_mad_u64, uint64_t, 8)
  RUN("v_mad_u64 sep", k_mad_u64_sep, uint64_t, 8)
  RUN("v_fma_f64", k_fma_f64, double, 1)
  RUN("v_fma_f64", k_fma_f64, double, 8)
  RUN("v_mul_lo_u32", k_mul_lo, uint32_t, 8)
  RUN("v_mul_hi_u32", k_mul_hi, uint32_t, 8)
  RUN("v_addc_co_u32", k_addc, uint32_t, 8)
  }
  CHK(hipFree(buf));
  return 0;
}
