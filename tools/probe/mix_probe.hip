// Marginal cost of non-mad instructions inside a v_mad_u64_u32 stream at 2 waves/SIMD
// (the Montgomery row's situation): per loop iteration 58 independent mads + 8 of OP.
// Output: ns per iteration per wave and the extra clock cycles OP adds versus mads alone.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef uint64_t u64;
typedef uint32_t u32;
#define ITERS 2048
#define M58(X) X X X X X X X X X X X X X X X X X X X X X X X X X X X X X X X X X X X X X X X X X X X X X X X X X X X X X X X X
#define MAD_BLOCK \
  asm volatile( \
      "v_mad_u64_u32 %0, vcc, %8, %9, %0\n\t" "v_mad_u64_u32 %1, vcc, %8, %9, %1\n\t" \
      "v_mad_u64_u32 %2, vcc, %8, %9, %2\n\t" "v_mad_u64_u32 %3, vcc, %8, %9, %3\n\t" \
      "v_mad_u64_u32 %4, vcc, %8, %9, %4\n\t" "v_mad_u64_u32 %5, vcc, %8, %9, %5\n\t" \
      "v_mad_u64_u32 %6, vcc, %8, %9, %6\n\t" "v_mad_u64_u32 %7, vcc, %8, %9, %7\n\t" \
      : "+v"(t[0]), "+v"(t[1]), "+v"(t[2]), "+v"(t[3]), "+v"(t[4]), "+v"(t[5]), "+v"(t[6]), "+v"(t[7]) \
      : "v"(a), "v"(b) : "vcc");

template <int OP>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_mix(u64* out, u32 a0) {
  u64 t[8];
  u32 a = a0 + threadIdx.x, b = a0 ^ (threadIdx.x * 7);
  u64 x = a * 3ull, y = b;
  u32 z0 = a, z1 = b, z2 = a ^ b, z3 = a + b;
  u32 d[8];
  u64 dd[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) { d[c] = c; dd[c] = c; }
#pragma unroll
  for (int c = 0; c < 8; ++c) t[c] = c + threadIdx.x;
  for (int i = 0; i < ITERS; ++i) {
    // 56 mads in 7 blocks of 8, + 2 -> 58 total with 8 OPs interleaved after blocks
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      MAD_BLOCK
      if constexpr (OP == 1) asm volatile("v_add_u32 %0, %0, %1" : "+v"(d[k]) : "v"(z1));
      if constexpr (OP == 2) asm volatile("v_lshrrev_b64 %0, 27, %1" : "=v"(dd[k]) : "v"(x));
      if constexpr (OP == 3) asm volatile("v_lshl_add_u64 %0, %1, 0, %0" : "+v"(dd[k]) : "v"(y));
      if constexpr (OP == 4) asm volatile("v_bfe_u32 %0, %1, %2, %3" : "=v"(d[k]) : "v"(z1), "v"(z2), "v"(z3));
      if constexpr (OP == 5) asm volatile("s_nop 1\n\tv_mov_b32_dpp %0, %1 quad_perm:[0,0,0,0] row_mask:0xf bank_mask:0xf" : "=v"(d[k]) : "v"(z1));
      if constexpr (OP == 6) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(d[k]) : "v"(z1));
      if constexpr (OP == 7) asm volatile("v_alignbit_b32 %0, %1, %2, 27" : "=v"(d[k]) : "v"(z1), "v"(z2));
      if constexpr (OP == 8) asm volatile("v_cndmask_b32 %0, %1, %2, vcc" : "=v"(d[k]) : "v"(z1), "v"(z2));
      if constexpr (OP == 9) asm volatile("s_nop 1\n\tv_and_b32_dpp %0, %1, %2 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "=v"(d[k]) : "v"(z1), "v"(z2));
      if constexpr (OP == 10) asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(d[k]) : "v"(z1) : "vcc");
      if constexpr (OP == 11) asm volatile("v_mov_b32 %0, 0" : "=v"(d[k]));
    }
    asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0\n\tv_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(t[0]) : "v"(a), "v"(b) : "vcc");
    if constexpr (OP != 0) {
      if constexpr (OP == 1) asm volatile("v_add_u32 %0, %0, %1" : "+v"(d[7]) : "v"(z1));
      if constexpr (OP == 2) asm volatile("v_lshrrev_b64 %0, 27, %1" : "=v"(dd[7]) : "v"(x));
      if constexpr (OP == 3) asm volatile("v_lshl_add_u64 %0, %1, 0, %0" : "+v"(dd[7]) : "v"(y));
      if constexpr (OP == 4) asm volatile("v_bfe_u32 %0, %1, %2, %3" : "=v"(d[7]) : "v"(z1), "v"(z2), "v"(z3));
      if constexpr (OP == 5) asm volatile("s_nop 1\n\tv_mov_b32_dpp %0, %1 quad_perm:[0,0,0,0] row_mask:0xf bank_mask:0xf" : "=v"(d[7]) : "v"(z1));
      if constexpr (OP == 6) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(d[7]) : "v"(z1));
      if constexpr (OP == 7) asm volatile("v_alignbit_b32 %0, %1, %2, 27" : "=v"(d[7]) : "v"(z1), "v"(z2));
      if constexpr (OP == 8) asm volatile("v_cndmask_b32 %0, %1, %2, vcc" : "=v"(d[7]) : "v"(z1), "v"(z2));
      if constexpr (OP == 9) asm volatile("s_nop 1\n\tv_and_b32_dpp %0, %1, %2 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "=v"(d[7]) : "v"(z1), "v"(z2));
      if constexpr (OP == 10) asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(d[7]) : "v"(z1) : "vcc");
      if constexpr (OP == 11) asm volatile("v_mov_b32 %0, 0" : "=v"(d[7]));
    }
  }
  u64 s = x + y + z0 + z1 + z2 + z3;
#pragma unroll
  for (int c = 0; c < 8; ++c) s += d[c] + dd[c];
#pragma unroll
  for (int c = 0; c < 8; ++c) s += t[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int OP>
float run(const char* name, int blocks, u64* buf, float base) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(k_mix<OP>, dim3(blocks), dim3(256), 0, 0, buf, 3u);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k_mix<OP>, dim3(blocks), dim3(256), 0, 0, buf, 3u);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  ms /= 5;
  // per SIMD: 2 waves, ITERS iterations each
  const double ns_iter = ms * 1e6 / ITERS / 2.0;
  printf("%-18s %8.3f ms  %.2f ns/iter/wave", name, ms, ns_iter);
  if (base > 0) printf("  +%.2f ns per OP ", (ns_iter - base) / 8);
  printf("\n");
  return (float)ns_iter;
}

int main() {
  hipDeviceProp_t prop;
  hipGetDeviceProperties(&prop, 0);
  const int blocks = prop.multiProcessorCount * 2;  // 2 waves/SIMD
  u64* buf;
  hipMalloc(&buf, (size_t)blocks * 256 * 8);
  printf("device %s CUs=%d; 58 mads/iter, 2 waves/SIMD\n", prop.gcnArchName, prop.multiProcessorCount);
  float base = run<0>("mads only", blocks, buf, 0);
  run<1>("v_add_u32", blocks, buf, base);
  run<2>("v_lshrrev_b64", blocks, buf, base);
  run<3>("v_lshl_add_u64", blocks, buf, base);
  run<4>("v_bfe_u32", blocks, buf, base);
  run<5>("v_mov_dpp(+nop1)", blocks, buf, base);
  run<6>("v_mul_lo_u32", blocks, buf, base);
  run<7>("v_alignbit_b32", blocks, buf, base);
  run<8>("v_cndmask_b32", blocks, buf, base);
  run<9>("v_and_dpp(+nop1)", blocks, buf, base);
  run<10>("v_add_co_u32", blocks, buf, base);
  run<11>("v_mov_b32 0", blocks, buf, base);
  return 0;
}
