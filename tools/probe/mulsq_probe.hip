// Throughput probe of the 28-bit engine at TPI 4 (2048-bit keys' n^2, 148 limbs; -DPROBE_TPI=2:
// p^2 / q^2 of 2048-bit keys, 74 limbs, the sq and mul modes only): what a wave
// sustains per element for
//   sq      : sqr() chains (the encrypt kernel's bulk)
//   mul     : mont_mul() with a fixed operand already in the LDS slot
//   mulslot : to_slot(B) from registers + mont_mul() each iteration
//   fold    : the fold kernel's term: 34 words gathered from an element-major row (random
//             index), load_chunk, to_slot, mont_mul (prefetched one product ahead)
// at 2 and 3 waves per SIMD (grid = CUs x 4 SIMDs x waves / 4 waves per block).
// Output: ns per element-product and the issued-mad rate against the half-rate peak.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probe/mulsq_probe.hip -o tools/probe/mulsq_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include "../../fate_amd/csrc/mont27_dev.h"
using namespace fphe;
using namespace fphe::r28;

#ifndef PROBE_TPI
#define PROBE_TPI 4
#endif
constexpr int TPI = PROBE_TPI;
using G = Geo<TPI>;
constexpr int E = G::E, NL = G::NL;

template <int MODE>
__device__ __forceinline__ void body(L27& A, L27& B, u32* bcol, u32 qoff, const Mod<TPI>& N, u32 np, int q,
                                     const u32* rows, size_t nrows, int iters, u32 seed) {
  constexpr int NW = kChunkWords<TPI>;
  const bool top = q == TPI - 1;
  auto fetch = [&](size_t idx, u32 (&W)[NW]) {
    const u32* base = rows + idx * 128 + 32u * q;
    const uint4* b4 = reinterpret_cast<const uint4*>(base);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint4 v = b4[k];
      W[4 * k] = v.x; W[4 * k + 1] = v.y; W[4 * k + 2] = v.z; W[4 * k + 3] = v.w;
    }
    const u32* tail = top ? base : base + 32;
    const uint2 t = *reinterpret_cast<const uint2*>(tail);
    W[32] = top ? 0u : t.x;
    W[33] = top ? 0u : t.y;
    if constexpr (NW > 34) {
      const u32 t2 = tail[2];
      W[34] = top ? 0u : t2;
    }
  };
  if constexpr (MODE == 0) {
#pragma unroll 1
    for (int it = 0; it < iters; ++it) sqr<TPI>(A, bcol, qoff, N, np, q);
  } else if constexpr (MODE == 1) {
    to_slot<TPI>(bcol, qoff, B);
#pragma unroll 1
    for (int it = 0; it < iters; ++it) mont_mul<TPI>(A, bcol, N, np, q);
  } else if constexpr (MODE == 2) {
#pragma unroll 1
    for (int it = 0; it < iters; ++it) {
      to_slot<TPI>(bcol, qoff, B);
      mont_mul<TPI>(A, bcol, N, np, q);
    }
  } else {
    // MODE 3: a wave's 16 elements read 16 consecutive rows (one random block per step);
    // MODE 4: every element reads its own random row (the fold's real gather pattern)
    u32 W[NW];
    u32 h = seed * 2654435761u + (MODE == 4 ? (u32)((threadIdx.x & 63) / TPI) * 40503u : 0u);
    auto nxt = [&]() -> size_t {
      h = h * 1664525u + 1013904223u;
      if constexpr (MODE == 4) return (size_t)((h >> 8) % (u32)nrows);
      return (size_t)(__builtin_amdgcn_readfirstlane(h) % (u32)(nrows / E)) * E + (threadIdx.x & 63) / TPI;
    };
    fetch(nxt(), W);
#pragma unroll 1
    for (int it = 0; it < iters; ++it) {
      load_chunk<TPI>(B, CSH * q, [&](int k) { return W[k]; });
      to_slot<TPI>(bcol, qoff, B);
      fetch(nxt(), W);
      mont_mul<TPI>(A, bcol, N, np, q);
    }
  }
}

template <int MODE, int OCC>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OCC))) void k_probe(const u32* __restrict__ Nl,
                                                                                        u32 np, u32* io,
                                                                                        const u32* rows, size_t nrows,
                                                                                        int iters) {
  extern __shared__ u32 lds[];
  G g;
  const u32 wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  u32* bcol = lds + wib * NL * E + g.e;
  const u32 qoff = lds_qoff<TPI>(g.q);
  Mod<TPI> N;
  N.init(Nl, g.q);
  const size_t base = ((size_t)blockIdx.x * 256 + threadIdx.x) * LL;
  L27 A, B;
#pragma unroll
  for (int j = 0; j < LL; ++j) {
    A.set(j, io[base + j] & MASK);
    B.set(j, (io[base + j] * 7u + 3u) & MASK);
  }
  body<MODE>(A, B, bcol, qoff, N, np, g.q, rows, nrows, iters, blockIdx.x * 4 + wib);
  finalize<TPI>(A, N, g.q);
#pragma unroll
  for (int j = 0; j < LL; ++j) io[base + j] = A[j];
}

// random 28-bit-safe words (a hash of the index): data-dependent power is part of what a real
// operand stream costs, so the probe does not run on a constant pattern
__global__ void k_fill(u32* p, size_t n, u32 salt) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    u32 h = (u32)i * 2654435761u ^ salt;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13; h *= 3266489917u; h ^= h >> 16;
    p[i] = h;
  }
}

template <int MODE, int OCC>
void run(const char* name, const u32* dN, u32 np, u32* io, const u32* rows, size_t nrows, int cus, int iters) {
  const int blocks = cus * OCC;  // 4 waves per block, OCC blocks per CU = OCC waves per SIMD
  const size_t lds = 4 * NL * E * 4;
  auto k = k_probe<MODE, OCC>;
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), lds, 0, dN, np, io, rows, nrows, 4);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  (void)hipEventRecord(a);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), lds, 0, dN, np, io, rows, nrows, iters);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  const double prods = (double)blocks * 256 / TPI * iters;
  // issued mads per element-product: general NL rows x 2 NL; squaring NL rows x TPI x (LL/2 + 1 + LL)
  const double mads = MODE == 0 ? (double)NL * TPI * (LL / 2 + 1 + LL) : 2.0 * NL * NL;
  const double peak = 256.0 * 128 * 2.4e9 / 2;  // half-rate v_mad_u64_u32 lane-ops/s
  printf("%-8s occ=%d blocks=%5d: %8.3f ms  %7.2f ns/elem-product  mad issue %.3f of peak\n", name, OCC, blocks, ms,
         ms * 1e6 / prods, prods * mads / (ms * 1e-3) / peak);
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 400;
  int dev = 0, cus = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  u32 hN[NL];
  srand(1);
  for (int j = 0; j < NL; ++j) hN[j] = ((u32)rand() ^ ((u32)rand() << 16)) & MASK;
  hN[0] |= 1;
  hN[NL - 1] &= MASK >> 3;
  u32 inv = 1;
  for (int i = 0; i < 5; ++i) inv *= 2 - hN[0] * inv;
  const u32 np = (0u - inv) & MASK;
  u32 *dN, *io, *rows;
  const size_t n = (size_t)cus * 4 * 256 * LL;
  const size_t nrows = (size_t)1 << 21;  // 1 GiB of element-major 4096-bit rows
  (void)hipMalloc(&dN, NL * 4);
  (void)hipMalloc(&io, n * 4);
  (void)hipMalloc(&rows, nrows * 128 * 4);
  (void)hipMemcpy(dN, hN, NL * 4, hipMemcpyHostToDevice);
  const bool rnd = argc > 2 && atoi(argv[2]) != 0;
  if (rnd) {
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, io, n, 0x1234u);
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, rows, nrows * 128, 0x9876u);
    (void)hipDeviceSynchronize();
  } else {
    (void)hipMemset(io, 0x5a, n * 4);
    (void)hipMemset(rows, 0x33, nrows * 128 * 4);
  }
  printf("operands: %s\n", rnd ? "random" : "constant pattern");
  run<0, 2>("sq", dN, np, io, rows, nrows, cus, iters);
  run<0, 3>("sq", dN, np, io, rows, nrows, cus, iters);
  run<1, 2>("mul", dN, np, io, rows, nrows, cus, iters);
  run<1, 3>("mul", dN, np, io, rows, nrows, cus, iters);
  run<2, 2>("mulslot", dN, np, io, rows, nrows, cus, iters);
  run<2, 3>("mulslot", dN, np, io, rows, nrows, cus, iters);
  if (TPI != 4) return 0;  // the fold modes gather 128-word rows
  run<3, 2>("fold", dN, np, io, rows, nrows, cus, iters);
  run<3, 3>("fold", dN, np, io, rows, nrows, cus, iters);
  run<4, 2>("foldrnd", dN, np, io, rows, nrows, cus, iters);
  run<4, 3>("foldrnd", dN, np, io, rows, nrows, cus, iters);
  return 0;
}
