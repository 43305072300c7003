// Calibrates rocprofv3 FETCH_SIZE / WRITE_SIZE (gfx950) for the access pattern of the
// modexp kernels' window table: one buffer_load_dword / buffer_store_dword per lane, a
// wave touching one 256-byte row per instruction.  Reads and writes exactly BYTES bytes
// (2 GiB, past the 256 MiB Infinity Cache) so the counters can be compared with a known
// byte count.  Run under `rocprofv3 --pmc FETCH_SIZE` and, separately, `--pmc WRITE_SIZE`.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

constexpr size_t BYTES = 2ull << 30;

__global__ __launch_bounds__(256) void k_read_rows(const uint32_t* buf, size_t nrows, uint32_t* sink) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(buf), 0, 0x7fffffff, 0x00020000);
  const uint32_t lane = threadIdx.x & 63;
  const size_t wave = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6), nwaves = (size_t)gridDim.x * 4;
  uint32_t acc = 0;
  for (size_t row = wave; row < nrows; row += nwaves) {
    // rows are 256 B; address via a per-row base (the descriptor range covers 2 GiB - 1)
    const uint32_t off = (uint32_t)(row * 256) + lane * 4;
    acc += __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0);
  }
  if (acc == 0x12345678u) sink[0] = acc;  // keep the loads alive
}

__global__ __launch_bounds__(256) void k_write_rows(uint32_t* buf, size_t nrows) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(buf, 0, 0x7fffffff, 0x00020000);
  const uint32_t lane = threadIdx.x & 63;
  const size_t wave = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6), nwaves = (size_t)gridDim.x * 4;
  for (size_t row = wave; row < nrows; row += nwaves)
    __builtin_amdgcn_raw_buffer_store_b32((uint32_t)row, r, (uint32_t)(row * 256) + lane * 4, 0, 0);
}

// The ct-add kernel's pattern (k_add27, 2048-bit key: L = 128 words, TPI = 4): ciphertexts in
// [tiles][128 words][64 elements] u32 tiles, a wave holding 16 consecutive elements x 4 lanes
// each, lane q of an element owning word rows 32q .. 32q + 31.  One buffer_load_dword per lane
// then touches four 64-byte segments, 8 KiB apart; the four waves of a block cover a tile's
// four 16-element quarters.
__device__ inline uint32_t quarter_off(size_t wt, uint32_t lane, uint32_t k) {
  const size_t tile = wt >> 2;
  const uint32_t quarter = (uint32_t)(wt & 3), q = lane >> 4, e = lane & 15;
  return (uint32_t)(((tile * 128 + 32 * q + k) * 64 + quarter * 16 + e) * 4);
}

__global__ __launch_bounds__(256) void k_read_quarters(const uint32_t* buf, size_t nwt, uint32_t* sink) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(buf), 0, 0x7fffffff, 0x00020000);
  const uint32_t lane = threadIdx.x & 63;
  const size_t wave = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6), nwaves = (size_t)gridDim.x * 4;
  uint32_t acc = 0;
  for (size_t wt = wave; wt < nwt; wt += nwaves)
    for (uint32_t k = 0; k < 32; ++k) acc += __builtin_amdgcn_raw_buffer_load_b32(r, quarter_off(wt, lane, k), 0, 0);
  if (acc == 0x12345678u) sink[0] = acc;
}

__global__ __launch_bounds__(256) void k_write_quarters(uint32_t* buf, size_t nwt) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(buf, 0, 0x7fffffff, 0x00020000);
  const uint32_t lane = threadIdx.x & 63;
  const size_t wave = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6), nwaves = (size_t)gridDim.x * 4;
  for (size_t wt = wave; wt < nwt; wt += nwaves)
    for (uint32_t k = 0; k < 32; ++k) __builtin_amdgcn_raw_buffer_store_b32((uint32_t)wt, r, quarter_off(wt, lane, k), 0, 0);
}

int main() {
  uint32_t *buf = nullptr, *sink = nullptr;
  const size_t bytes = BYTES - 256;  // stay inside the 2^31-1 descriptor range
  if (hipMalloc(&buf, BYTES) != hipSuccess || hipMalloc(&sink, 4) != hipSuccess) { printf("alloc failed\n"); return 1; }
  const size_t nrows = bytes / 256;
  hipLaunchKernelGGL(k_write_rows, dim3(2048), dim3(256), 0, 0, buf, nrows);   // dispatch 1: writes `bytes`
  hipLaunchKernelGGL(k_read_rows, dim3(2048), dim3(256), 0, 0, buf, nrows, sink);  // dispatch 2: reads `bytes`
  const size_t nwt = (bytes / (128 * 256)) * 4;  // whole 32-KiB tiles, 4 wave quarters each
  hipLaunchKernelGGL(k_write_quarters, dim3(2048), dim3(256), 0, 0, buf, nwt);        // dispatch 3
  hipLaunchKernelGGL(k_read_quarters, dim3(2048), dim3(256), 0, 0, buf, nwt, sink);   // dispatch 4
  if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 1; }
  printf("calibration: k_write_rows wrote %zu bytes, k_read_rows read %zu bytes (%.3f KiB each)\n", bytes, bytes,
         bytes / 1024.0);
  printf("calibration: k_write_quarters / k_read_quarters %zu bytes each (%.3f KiB)\n", nwt * 8192, nwt * 8.0);
  (void)hipFree(buf);
  (void)hipFree(sink);
  return 0;
}
