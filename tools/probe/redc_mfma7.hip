// Probe (round 2 research spike, not part of libfatephe): batched Montgomery reduction of
// 8192-bit products mod a 4096-bit N on the i8 matrix cores, base-128 variant.
//
// As tools/probe/redc_mfma.hip, but with balanced base-128 digits (|d| <= 64) held in int8:
// the column sums of q = T_low * N' are brought back into int8 range by THREE PARALLEL
// carry-save steps (each position keeps its balanced 7-bit digit and adds the carry of the
// position below; |digit| <= 67 afterwards, which int8 holds), instead of a 544-step
// sequential carry chain.  q is then a valid (non-canonical) representative of T N' mod R,
// R = 128^608: U = (T + qN)/R + N stays in (0, 2N).  Cost: 380 MFMAs per 32 elements
// (19 x 32-digit tiles) against 306, in exchange for no serial dependency.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

constexpr int QT = 19;      // q tiles: D = 608 digits
constexpr int TT = 38;      // T tiles (1216 digits)
constexpr int NA1 = 19;     // product-1 A tiles (offset 0..18)
constexpr int NA2 = 20;     // product-2 A tiles (offset 0..19)

__device__ __forceinline__ int swap_halves(int x, int h) {
  auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
  return h ? (int)r[0] : (int)r[1];
}

// one carry-save step over a C-layout tile (positions p = (r&3) + 8(r>>2) + 4h): every
// position keeps its balanced 7-bit digit and adds the carry of position p-1.  prev: the
// carry of the previous tile's position 31 (valid in half 0), updated to this tile's.
__device__ __forceinline__ void cs_step(int (&v)[16], int& prev, int h) {
  int c[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int d = __builtin_amdgcn_sbfe(v[r], 0, 7);
    c[r] = (v[r] - d) >> 7;
    v[r] = d;
  }
  int xs[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) xs[g] = swap_halves(c[4 * g + 3], h);  // the other half's c[4g+3]
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    int cp;
    if (r & 3) cp = c[r - 1];
    else {
      const int g = r >> 2;
      const int lo = g == 0 ? prev : xs[g - 1];  // half 0: position 8g-1 lives in half 1
      cp = h ? xs[g] : lo;                        // half 1: position 8g+3 lives in half 0
    }
    v[r] += cp;
  }
  prev = xs[3];  // half 0 now holds half 1's c[15] = carry out of position 31
}

extern "C" __global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void k_redc7(
    const v4i* __restrict__ Afrag, const int8_t* __restrict__ T, int* __restrict__ U, int nelem, int reps,
    int* __restrict__ dbg, int shared_t) {
  __shared__ v4i sA[(NA1 + NA2) * 64];
  for (int i = threadIdx.x; i < (NA1 + NA2) * 64; i += blockDim.x) sA[i] = Afrag[i];
  __syncthreads();
  const int lane = threadIdx.x & 63, e = lane & 31, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane((int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6));
  const int nwaves = (gridDim.x * blockDim.x) >> 6;
  const int nbatch = nelem / 32;
  for (int b = wave; b < nbatch; b += nwaves) {
    const int elem = b * 32 + e;
    // shared_t: every wave reads batch 0's T (compute-bound timing: T stays in L1/L2)
    const int tb = shared_t ? 0 : b;
    const v4i* Tb = reinterpret_cast<const v4i*>(T) + (size_t)tb * TT * 64;
    const int8_t* Tb8 = T + (size_t)tb * TT * 64 * 16;
    int* Ub = U + (size_t)b * QT * 16 * 64;
    for (int rep = 0; rep < reps; ++rep) {
      const v4i* Tr = Tb;
      asm volatile("" : "+s"(Tr));
      int al = lane;
      asm volatile("" : "+v"(al));
      int* Ur = Ub;
      asm volatile("" : "+s"(Ur));
      const int8_t* Tr8 = Tb8;
      asm volatile("" : "+s"(Tr8));
      v4i q[QT];
      int p1 = 0, p2 = 0, p3 = 0;  // carries of the previous tile, per carry-save step
#pragma unroll
      for (int m = 0; m < QT; ++m) {
        __builtin_amdgcn_sched_barrier(0);
        v16i acc = {0};
#pragma unroll
        for (int kt = 0; kt <= m; ++kt) {
          v4i a = sA[(m - kt) * 64 + al];
          v4i bf = Tr[kt * 64 + lane];
          acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, bf, acc, 0, 0, 0);
        }
        int v[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = acc[r];
        cs_step(v, p1, h);
        cs_step(v, p2, h);
        cs_step(v, p3, h);
        v4i qq;
#pragma unroll
        for (int w = 0; w < 4; ++w)
          qq[w] = (v[4 * w] & 255) | ((v[4 * w + 1] & 255) << 8) | ((v[4 * w + 2] & 255) << 16) |
                  ((unsigned)(v[4 * w + 3] & 255) << 24);
        q[m] = qq;
        if (dbg && rep == 0) {
#pragma unroll
          for (int r = 0; r < 16; ++r) dbg[(size_t)elem * 608 + 32 * m + (r & 3) + 8 * (r >> 2) + 4 * h] = v[r];
        }
      }
      int cU = 0;
#pragma unroll
      for (int t = 18; t < TT; ++t) {
        __builtin_amdgcn_sched_barrier(0);
        v16i acc = {0};
#pragma unroll
        for (int i = 0; i < QT; ++i) {
          const int d = t - i;
          if (d < 0 || d >= NA2) continue;
          v4i a = sA[(NA1 + d) * 64 + al];
          acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, q[i], acc, 0, 0, 0);
        }
        if (t == 18) {
          // positions 600..607 = rows 24..31 of tile 18
          double s = 0.0;
#pragma unroll
          for (int r4 = 0; r4 < 4; ++r4) {
            const int row = 24 + 4 * h + r4;
            const int v = acc[12 + r4] + (int)Tr8[((size_t)18 * 64 + 32 * (row >> 4) + e) * 16 + (row & 15)];
            s += (double)v * __builtin_ldexp(1.0, 7 * (row - 32));
          }
          const unsigned long long bits = __builtin_bit_cast(unsigned long long, s);
          const unsigned lo = (unsigned)swap_halves((int)(unsigned)bits, h);
          const unsigned hi = (unsigned)swap_halves((int)(unsigned)(bits >> 32), h);
          const double other = __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
          cU = (int)__builtin_rint(s + other);
        } else if (rep == reps - 1) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            int v = acc[r];
            if (t == 19 && r == 0 && h == 0) v += cU;
            Ur[((t - 19) * 16 + r) * 64 + lane] = v;
          }
        } else {
          int x = 0;
#pragma unroll
          for (int r = 0; r < 16; ++r) x ^= acc[r];
          asm volatile("" : : "v"(x));
        }
      }
    }
  }
}

extern "C" int redc7_launch(const void* Afrag, const void* T, void* U, int nelem, int reps, int grid, void* dbg,
                            int shared_t, void* stream) {
  hipLaunchKernelGGL(k_redc7, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const v4i*)Afrag, (const int8_t*)T,
                     (int*)U, nelem, reps, (int*)dbg, shared_t);
  return (int)hipGetLastError();
}
