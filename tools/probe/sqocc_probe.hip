// Squaring throughput of the 27-bit engine (mont27_dev.h mont_sqr, TPI = 4) at 2 and 3
// waves/SIMD register budgets: issue rate in Tmad/s (v_mad_u64_u32 per second, the mad
// count of NL rows x TPI lanes x (20 + 38)), and a check that both builds agree.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "../../fate_amd/csrc/mont27_dev.h"
using namespace fphe;
using namespace fphe::r27;

template <int TPI, int OCC>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OCC))) void k_sq(const u32* __restrict__ Nl,
                                                                                        u32 np, u32* io, int iters) {
  using G = Geo<TPI>;
  constexpr int E = G::E;
  extern __shared__ u32 lds[];
  G g;
  const u32 wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  u32* bcol = lds + wib * G::NL * E + g.e;
  const u32 qoff = lds_qoff<TPI>(g.q);
  Mod<TPI> N;
  N.init(Nl, g.q);
  const size_t base = ((size_t)blockIdx.x * 256 + threadIdx.x) * LL;
  L27 A;
#pragma unroll
  for (int j = 0; j < LL; ++j) A.set(j, io[base + j]);
#pragma unroll 1
  for (int it = 0; it < iters; ++it) sqr<TPI>(A, bcol, qoff, N, np, g.q);
  finalize<TPI>(A, N, g.q);
#pragma unroll
  for (int j = 0; j < LL; ++j) io[base + j] = A[j];
}

template <int OCC>
double run(int blocks, int iters, const u32* dN, u32 np, u32* io, const u32* init, size_t n) {
  constexpr int TPI = 4, NL = LL * TPI;
  (void)hipMemcpy(io, init, n * 4, hipMemcpyHostToDevice);
  const size_t lds = 4 * NL * (64 / TPI) * 4;
  hipLaunchKernelGGL((k_sq<TPI, OCC>), dim3(blocks), dim3(256), lds, 0, dN, np, io, 2);
  (void)hipMemcpy(io, init, n * 4, hipMemcpyHostToDevice);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  (void)hipEventRecord(a);
  hipLaunchKernelGGL((k_sq<TPI, OCC>), dim3(blocks), dim3(256), lds, 0, dN, np, io, iters);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  const double prods = (double)blocks * 256 / TPI * iters;
  const double mads = prods * NL * TPI * (20 + 38);
  printf("OCC=%d blocks=%d: %.3f ms, %.3e sqr/s, %.2f Tmad/s\n", OCC, blocks, ms, prods / (ms * 1e-3),
         mads / (ms * 1e-3) / 1e12);
  return ms;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 400;
  constexpr int TPI = 4, NL = LL * TPI;
  u32 hN[NL];
  srand(1);
  for (int j = 0; j < NL; ++j) hN[j] = ((u32)rand() ^ ((u32)rand() << 16)) & MASK;
  hN[0] |= 1;
  hN[NL - 1] &= MASK >> 3;
  u32 inv = 1;
  for (int i = 0; i < 5; ++i) inv *= 2 - hN[0] * inv;
  const u32 np = (0u - inv) & MASK;
  const int maxblocks = 256 * 6;
  const size_t n = (size_t)maxblocks * 256 * LL;
  u32* init = (u32*)malloc(n * 4);
  for (size_t i = 0; i < n; ++i) init[i] = ((u32)rand() ^ ((u32)rand() << 16)) & MASK;
  for (size_t i = 0; i < n; i += (size_t)LL * TPI) init[i + LL * TPI - 1] &= MASK >> 4;  // < N-ish
  u32 *dN, *io;
  (void)hipMalloc(&dN, NL * 4);
  (void)hipMalloc(&io, n * 4);
  (void)hipMemcpy(dN, hN, NL * 4, hipMemcpyHostToDevice);
  u32* out2 = (u32*)malloc(n * 4);
  u32* out3 = (u32*)malloc(n * 4);
  // warm the clock up first (a cold chip ramps over the first tens of ms)
  run<2>(256 * 2, iters * 4, dN, np, io, init, n);
  for (int rep = 0; rep < 2; ++rep) {
    run<2>(256 * 2, iters, dN, np, io, init, n);
    (void)hipMemcpy(out2, io, (size_t)256 * 2 * 256 * LL * 4, hipMemcpyDeviceToHost);
    run<3>(256 * 3, iters, dN, np, io, init, n);
    (void)hipMemcpy(out3, io, (size_t)256 * 2 * 256 * LL * 4, hipMemcpyDeviceToHost);
    printf("  outputs (first 512 blocks) %s\n", memcmp(out2, out3, (size_t)256 * 2 * 256 * LL * 4) ? "DIFFER" : "agree");
    run<2>(256 * 4, iters, dN, np, io, init, n);
    run<3>(256 * 6, iters, dN, np, io, init, n);
  }
  return 0;
}
