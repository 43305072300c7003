// Shader clock over the course of a full-chip v_mad_u64_u32 burst (DESIGN.md §3, round 4:
// why a 15 ms fold launch runs at a lower clock than a 50 ms one).  Every CU runs 2 waves per
// SIMD of independent mad chains (the engines' occupancy); wave 0 of block 0 samples
// clock64() (shader clock) and wall_clock64() (constant-rate counter) every kIters
// iterations and stores the pairs with ordinary vector stores.  The host prints the clock in
// 1 ms bins from the start of the launch.  Two launches: after ~300 ms idle, and right
// after the first (warm).
//
//   hipcc --offload-arch=gfx950 -O3 -o clock_probe clock_probe.hip && ./clock_probe [ms]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <unistd.h>
#include <vector>

constexpr int kIters = 64;  // mad rounds between samples
constexpr int kMaxSamples = 1 << 16;

__global__ __launch_bounds__(256) void k_burst(uint64_t* samples, int nsamples, uint32_t seed, uint64_t* sink) {
  uint64_t acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = seed + threadIdx.x + i;
  uint32_t a = seed ^ threadIdx.x, b = seed * 7 + blockIdx.x;
  const bool rec = blockIdx.x == 0 && threadIdx.x < 64;
  for (int s = 0; s < nsamples; ++s) {
    for (int k = 0; k < kIters; ++k) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        uint64_t r;
        asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(acc[i]) : "vcc");
        acc[i] = r;
      }
    }
    if (rec && threadIdx.x == 0) {
      samples[2 * s] = clock64();
      samples[2 * s + 1] = wall_clock64();
    }
  }
  uint64_t t = 0;
  for (int i = 0; i < 8; ++i) t ^= acc[i];
  if (t == 0x123456789abcdefull) sink[0] = t;
}

int main(int argc, char** argv) {
  const double ms = argc > 1 ? atof(argv[1]) : 100.0;
  int dev = 0, cus = 0, wall_khz = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  (void)hipDeviceGetAttribute(&wall_khz, hipDeviceAttributeWallClockRate, dev);
  uint64_t *d = nullptr, *sink = nullptr;
  if (hipMalloc(&d, 2 * kMaxSamples * sizeof(uint64_t)) != hipSuccess || hipMalloc(&sink, 8) != hipSuccess) return 1;
  // calibrate samples per ms with a short launch
  const int grid = cus * 2;  // 2 blocks of 4 waves per CU = 2 waves per SIMD
  int ns = 200;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(k_burst, dim3(grid), dim3(256), 0, 0, d, ns, 1u, sink);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(k_burst, dim3(grid), dim3(256), 0, 0, d, ns, 2u, sink);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float cal = 0;
  (void)hipEventElapsedTime(&cal, e0, e1);
  ns = (int)(ns * ms / cal);
  if (ns > kMaxSamples) ns = kMaxSamples;
  std::vector<uint64_t> h(2 * ns);
  for (int run = 0; run < 2; ++run) {
    if (run == 0) usleep(300000);  // idle first
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(k_burst, dim3(grid), dim3(256), 0, 0, d, ns, 3u + run, sink);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float t = 0;
    (void)hipEventElapsedTime(&t, e0, e1);
    (void)hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost);
    printf("run %d (%s): %.2f ms, %d samples, wall clock %d kHz\n", run, run ? "right after the first" : "after 300 ms idle",
           t, ns, wall_khz);
    const double w0 = (double)h[1];
    int s0 = 0;
    double next = 1.0;
    for (int s = 1; s < ns; ++s) {
      const double tw = ((double)h[2 * s + 1] - w0) / wall_khz;  // ms since the first sample
      if (tw >= next || s == ns - 1) {
        const double dc = (double)(h[2 * s] - h[2 * s0]);
        const double dw = ((double)h[2 * s + 1] - (double)h[2 * s0 + 1]) / (wall_khz * 1e3);
        printf("  %7.1f ms  %.3f GHz\n", tw, dc / dw / 1e9);
        s0 = s;
        next = tw < 10 ? tw + 1.0 : tw + 5.0;
      }
    }
  }
  return 0;
}
