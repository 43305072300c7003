// Probe: issue rates of the non-MAC instructions of a fused CIOS row (mont_gen_ll37.h) at the
// engines' 3 waves/SIMD and at 8, each as 8 independent chains per wave.  Not product code.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define ITERS 8192
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

#define K32(NAME, INSTR)                                                                     \
  __global__ void NAME(uint32_t* out, uint32_t a0) {                                         \
    uint32_t c0 = threadIdx.x, c1 = c0 + 1, c2 = c0 + 2, c3 = c0 + 3, c4 = c0 + 4, c5 = c0 + 5, c6 = c0 + 6, \
             c7 = c0 + 7;                                                                    \
    uint32_t a = a0 ^ threadIdx.x;                                                           \
    for (int i = 0; i < ITERS; ++i) {                                                        \
      asm volatile(INSTR(0) INSTR(1) INSTR(2) INSTR(3) INSTR(4) INSTR(5) INSTR(6) INSTR(7)   \
                   : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(c4), "+v"(c5), "+v"(c6), "+v"(c7) \
                   : "v"(a));                                                                \
    }                                                                                        \
    out[blockIdx.x * blockDim.x + threadIdx.x] = c0 + c1 + c2 + c3 + c4 + c5 + c6 + c7;      \
  }
#define K64(NAME, INSTR)                                                                     \
  __global__ void NAME(uint32_t* out, uint32_t a0) {                                         \
    uint64_t c0 = threadIdx.x, c1 = c0 + 1, c2 = c0 + 2, c3 = c0 + 3, c4 = c0 + 4, c5 = c0 + 5, c6 = c0 + 6, \
             c7 = c0 + 7;                                                                    \
    uint64_t a = a0 ^ threadIdx.x;                                                           \
    for (int i = 0; i < ITERS; ++i) {                                                        \
      asm volatile(INSTR(0) INSTR(1) INSTR(2) INSTR(3) INSTR(4) INSTR(5) INSTR(6) INSTR(7)   \
                   : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(c4), "+v"(c5), "+v"(c6), "+v"(c7) \
                   : "v"(a));                                                                \
    }                                                                                        \
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(c0 + c1 + c2 + c3 + c4 + c5 + c6 + c7); \
  }

#define I_ALIGN(k) "v_alignbit_b32 %" #k ", %8, %" #k ", 28\n\t"
#define I_LSHR(k) "v_lshrrev_b32 %" #k ", 28, %" #k "\n\t"
#define I_BFE(k) "v_bfe_u32 %" #k ", %" #k ", 1, 30\n\t"
#define I_MULLO(k) "v_mul_lo_u32 %" #k ", %" #k ", %8\n\t"
#define I_ANDDPP(k) "v_and_b32_dpp %" #k ", %" #k ", %8 row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
#define I_MOV0(k) "v_mov_b32 %" #k ", 0\n\t"
#define I_LSHR64(k) "v_lshrrev_b64 %" #k ", 28, %" #k "\n\t"
#define I_LSHLADD64(k) "v_lshl_add_u64 %" #k ", %8, 0, %" #k "\n\t"
#define I_MAD64(k) "v_mad_u64_u32 %" #k ", vcc, %8, %8, %" #k "\n\t"

K32(k_align, I_ALIGN)
K32(k_lshr, I_LSHR)
K32(k_bfe, I_BFE)
K32(k_mullo, I_MULLO)
K32(k_anddpp, I_ANDDPP)
K32(k_mov0, I_MOV0)
K64(k_lshr64, I_LSHR64)
K64(k_lshladd64, I_LSHLADD64)

__global__ void k_mad64(uint32_t* out, uint32_t a0) {
  uint64_t c0 = threadIdx.x, c1 = c0 + 1, c2 = c0 + 2, c3 = c0 + 3, c4 = c0 + 4, c5 = c0 + 5, c6 = c0 + 6, c7 = c0 + 7;
  uint32_t a = a0 ^ threadIdx.x;
  for (int i = 0; i < ITERS; ++i) {
    asm volatile(I_MAD64(0) I_MAD64(1) I_MAD64(2) I_MAD64(3) I_MAD64(4) I_MAD64(5) I_MAD64(6) I_MAD64(7)
                 : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(c4), "+v"(c5), "+v"(c6), "+v"(c7)
                 : "v"(a) : "vcc");
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(c0 + c1 + c2 + c3 + c4 + c5 + c6 + c7);
}

template <typename F>
static float time_it(F launch) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  launch();
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(a);
  for (int r = 0; r < 10; ++r) launch();
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms / 10;
}

int main() {
  hipDeviceProp_t prop;
  CHK(hipGetDeviceProperties(&prop, 0));
  const int threads = 256;
  void* buf;
  CHK(hipMalloc(&buf, (size_t)prop.multiProcessorCount * 8 * threads * 8));
  printf("lane-op/clk/CU at the nominal clock, 8 independent chains per wave\n");
  for (int bpc : {3, 8}) {
    const int blocks = prop.multiProcessorCount * bpc;
    const double ops = (double)blocks * threads * ITERS * 8;
#define RUN(NAME, KER)                                                                              \
  {                                                                                                 \
    float ms = time_it([&] { hipLaunchKernelGGL(KER, dim3(blocks), dim3(threads), 0, 0, (uint32_t*)buf, 5u); }); \
    printf("%d waves/SIMD %-18s %7.3f ms %6.1f\n", bpc, NAME, ms,                                   \
           ops / (ms * 1e-3) / prop.multiProcessorCount / (prop.clockRate * 1e3));                  \
  }
    RUN("v_mad_u64_u32", k_mad64)
    RUN("v_alignbit_b32", k_align)
    RUN("v_lshrrev_b32", k_lshr)
    RUN("v_bfe_u32", k_bfe)
    RUN("v_mul_lo_u32", k_mullo)
    RUN("v_and_b32_dpp", k_anddpp)
    RUN("v_mov_b32 0", k_mov0)
    RUN("v_lshrrev_b64", k_lshr64)
    RUN("v_lshl_add_u64", k_lshladd64)
  }
  CHK(hipFree(buf));
  return 0;
}
