// Probe (round 2 research spike, not part of libfatephe): batched Montgomery reduction of
// 8192-bit products modulo a 4096-bit N on the i8 matrix cores (v_mfma_i32_32x32x32_i8).
//
// Numbers are balanced base-256 digits (int8 in [-128, 127]).  R = 256^544.  For a wave of
// 32 elements (MFMA column = element, lane l: element l&31, half h = l>>5):
//   product 1: s = T_low * N' (lower-triangular Toeplitz of N' = -N^-1 mod R, A operand,
//              17 x 17 / 2 tiles), column sums in i32, normalised to balanced digits
//              mod R with a carry chain in the C layout  -> q (17 tiles, packed bytes)
//   product 2: P = N * q for the output tiles 16..33 (Toeplitz of N as the A operand, its K
//              order permuted to the C layout q is produced in, so q feeds the MFMA as
//              the B operand without moving lanes)
//   U = (T + qN)/R + N: the carry out of the low half is round(sum over positions
//       536..543 of (t_k + p_k) 256^(k-544)) (the lower positions weigh < 2^-48), the
//       high positions are t_k + p_k (i32 digit sums, written out unnormalised).
// Host (tools/probe/redc_mfma.py) builds T, N, N', the A fragments, checks U against
// Python integers, and times `reps` reductions per element.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

constexpr int QT = 17;      // q tiles: 544 digits
constexpr int TD = 1088;    // T digits per element (34 tiles)
constexpr int NA1 = 17;     // product-1 A tiles (offset d = 0..16)
constexpr int NA2 = 18;     // product-2 A tiles (offset d = 0..17)

__device__ __forceinline__ int swap_halves(int x, int h) {
  // value of lane l ^ 32
  auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
  return h ? (int)r[0] : (int)r[1];
}

// balanced digit of v and the exact carry
__device__ __forceinline__ int bal(int v, int& carry) {
  const int d = ((v + 128) & 255) - 128;
  carry = (v - d) >> 8;
  return d;
}

extern "C" __global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void k_redc(const v4i* __restrict__ Afrag, const int8_t* __restrict__ T,
                                                         int* __restrict__ U, int nelem, int reps,
                                                         int* __restrict__ dbg) {
  __shared__ v4i sA[(NA1 + NA2) * 64];
  for (int i = threadIdx.x; i < (NA1 + NA2) * 64; i += blockDim.x) sA[i] = Afrag[i];
  __syncthreads();
  const int lane = threadIdx.x & 63, e = lane & 31, h = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane((int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6));
  const int nwaves = (gridDim.x * blockDim.x) >> 6;
  const int nbatch = nelem / 32;
  for (int b = wave; b < nbatch; b += nwaves) {
    const int elem = b * 32 + e;
    // T in MFMA fragment order: [batch][tile 0..33][lane][16 B]; U: [batch][tile 0..16][reg][lane]
    const v4i* Tb = reinterpret_cast<const v4i*>(T) + (size_t)b * 34 * 64;
    const int8_t* Tb8 = T + (size_t)b * 34 * 64 * 16;
    int* Ub = U + (size_t)b * 17 * 16 * 64;
    for (int rep = 0; rep < reps; ++rep) {
      const v4i* Tr = Tb;
      asm volatile("" : "+s"(Tr));  // opaque per rep: no hoisting of the T fragment loads
      int al = lane;
      asm volatile("" : "+v"(al));  // likewise for the LDS A fragments (35 tiles x 4 VGPRs)
      int* Ur = Ub;
      asm volatile("" : "+s"(Ur));  // and the U store addresses (272 of them)
      const int8_t* Tr8 = Tb8;
      asm volatile("" : "+s"(Tr8));
      v4i q[QT];
      int carry = 0;  // valid in half 0
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
        // normalise positions 32m + p, p = 0..31: p -> half (p>>2)&1, register (p&3) + 4(p>>3)
        int dg[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) dg[r] = 0;
        int cin = carry;
#pragma unroll
        for (int g = 0; g < 8; ++g) {
          const int hh = g & 1, base = 4 * (g >> 1);
          int cc = cin;
#pragma unroll
          for (int r4 = 0; r4 < 4; ++r4) {
            int c2;
            const int d = bal(acc[base + r4] + cc, c2);
            cc = c2;
            dg[base + r4] = (h == hh) ? d : dg[base + r4];  // register base+r4 of THIS half
          }
          const int mine = (h == hh) ? cc : cin;
          cin = swap_halves(mine, h);  // the other half now holds this group's carry-out
        }
        carry = cin;  // after g = 7 (half 1) the carry sits in half 0
        // pack the 16 digits (register order) into the B fragment bytes
        v4i qq;
#pragma unroll
        for (int w = 0; w < 4; ++w)
          qq[w] = (dg[4 * w] & 255) | ((dg[4 * w + 1] & 255) << 8) | ((dg[4 * w + 2] & 255) << 16) |
                  ((unsigned)(dg[4 * w + 3] & 255) << 24);
        q[m] = qq;
        if (dbg && rep == 0) {
#pragma unroll
          for (int r = 0; r < 16; ++r) dbg[(size_t)elem * 544 + 32 * m + (r & 3) + 8 * (r >> 2) + 4 * h] = dg[r];
        }
      }
      // product 2: output tiles 16..33 (positions 512..1087)
      double csum = 0.0;
      int cU = 0;
#pragma unroll
      for (int t = 16; t < 34; ++t) {
        __builtin_amdgcn_sched_barrier(0);  // one output tile at a time (register pressure)
        v16i acc = {0};
#pragma unroll
        for (int i = 0; i < QT; ++i) {
          const int d = t - i;
          if (d < 0 || d >= NA2) continue;
          v4i a = sA[(NA1 + d) * 64 + al];
          acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, q[i], acc, 0, 0, 0);
        }
        if (t == 16) {
          // positions 536..543 = rows 24..31: half h holds rows 24+4h .. 27+4h in regs 12..15
          double s = 0.0;
#pragma unroll
          for (int r4 = 0; r4 < 4; ++r4) {
            const int row = 24 + 4 * h + r4;
            // T digit at position 512 + row of element e: fragment byte (lane 32*(row>>4) + e, j = row & 15)
            const int v = acc[12 + r4] + (int)Tr8[((size_t)16 * 64 + 32 * (row >> 4) + e) * 16 + (row & 15)];
            s += (double)v * __builtin_ldexp(1.0, 8 * (row - 32));
          }
          // total over both halves
          const double other = __builtin_bit_cast(double, (long long)(((unsigned long long)(unsigned)swap_halves(
                                   (int)(__builtin_bit_cast(unsigned long long, s) >> 32), h) << 32) |
                                   (unsigned)swap_halves((int)__builtin_bit_cast(unsigned long long, s), h)));
          csum = s + other;
          cU = (int)__builtin_rint(csum);
        } else if (rep == reps - 1) {
          // P_high (+ the low half's carry at position 0); the host adds T_high
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            int v = acc[r];
            if (t == 17 && r == 0 && h == 0) v += cU;
            Ur[((t - 17) * 16 + r) * 64 + lane] = v;
          }
        } else {
          // keep the tile live without a store
          int x = 0;
#pragma unroll
          for (int r = 0; r < 16; ++r) x ^= acc[r];
          asm volatile("" : : "v"(x));
        }
      }
    }
  }
}

extern "C" int redc_launch(const void* Afrag, const void* T, void* U, int nelem, int reps, int grid, void* dbg,
                           void* stream) {
  hipLaunchKernelGGL(k_redc, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const v4i*)Afrag, (const int8_t*)T,
                     (int*)U, nelem, reps, (int*)dbg);
  return (int)hipGetLastError();
}
