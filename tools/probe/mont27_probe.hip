// Throughput/codegen probe for the 27-bit engine (mont27_dev.h): `iters` squarings per
// element, TPI lanes per element.  Output: product count and kernel time.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include "../../fate_amd/csrc/mont27_dev.h"
using namespace fphe;
using namespace fphe::r27;

template <int TPI>
__global__ __launch_bounds__(256) void k_sq(const u32* __restrict__ Nl, u32 np, u32* io, int iters) {
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

template <int TPI>
void run(int blocks, int iters) {
  constexpr int NL = LL * TPI;
  u32 hN[NL];
  srand(1);
  for (int j = 0; j < NL; ++j) hN[j] = ((u32)rand() ^ ((u32)rand() << 16)) & MASK;
  hN[0] |= 1;
  hN[NL - 1] &= MASK >> 3;  // N < R/4
  // n' = -N^-1 mod 2^27
  u32 inv = 1;
  for (int i = 0; i < 5; ++i) inv *= 2 - hN[0] * inv;
  const u32 np = (0u - inv) & MASK;
  u32 *dN, *io;
  const size_t n = (size_t)blocks * 256 * LL;
  (void)hipMalloc(&dN, NL * 4);
  (void)hipMalloc(&io, n * 4);
  (void)hipMemcpy(dN, hN, NL * 4, hipMemcpyHostToDevice);
  (void)hipMemset(io, 0, n * 4);
  const size_t lds = 4 * NL * (64 / TPI) * 4;
  hipLaunchKernelGGL(k_sq<TPI>, dim3(blocks), dim3(256), lds, 0, dN, np, io, 2);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  (void)hipEventRecord(a);
  hipLaunchKernelGGL(k_sq<TPI>, dim3(blocks), dim3(256), lds, 0, dN, np, io, iters);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  const double prods = (double)blocks * 256 / TPI * iters;
  const double mac32 = prods * (2.0 * (NL * 27 / 32.0) * (NL * 27 / 32.0));
  printf("TPI=%d NL=%d blocks=%d: %.3f ms, %.3e prod/s, %.2f TMAC32-equiv/s (2L^2 of %d-bit)\n", TPI, NL, blocks, ms,
         prods / (ms * 1e-3), mac32 / (ms * 1e-3) / 1e12, NL * 27);
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 2000;
  for (int bpc : {1, 2, 3, 4}) run<4>(256 * bpc, iters);
  for (int bpc : {1, 2, 3, 4}) run<2>(256 * bpc, iters);
  for (int bpc : {1, 2, 3, 4}) run<1>(256 * bpc, iters);
  return 0;
}
