// Two-lanes-per-element ("TPI=2") Montgomery arithmetic for 4096-bit moduli (n^2 of a
// 2048-bit Paillier key) on gfx950.
//
// One element occupies lanes e and e+32 of a wave (e = lane & 31).  The lane in half h
// (h = lane >> 5) holds limbs [h*LL, h*LL+LL) of the running value A, the CIOS
// accumulator T and the modulus N (N in VGPRs: the two halves need different limbs, so
// it cannot be a scalar operand).  Per CIOS row the halves exchange two words with
// v_permlane32_swap_b32 (no LDS traffic; on gfx950 it exchanges vdst[32..63] with
// vsrc[0..31], verified by tools/probe/permlane_probe.hip): m (low -> high) and the high half's first
// reduction word (high -> low).  The carry that crosses limb 64 is kept pending in the
// low half (e0) and folded into the high half once per product.
//
// Why: with one lane per element a 4096-bit product needs A[128] + T[129] VGPRs, which
// caps the kernel at one wave per SIMD -- and a lone wave issues v_mad_u64_u32 at half
// the rate two waves reach (profiles/r01_probe_alu.txt).  Two lanes per element halve
// the per-lane footprint (~210 VGPRs) so two waves share each SIMD.
#pragma once
#include "../../fate_amd/csrc/mont_dev.h"

namespace fphe {

constexpr int kHalf = 32;  // elements per wave with TPI=2

// B operand column of this lane's element in the wave's LDS tile [2*LL][32].
// Lane half h stores/loads limbs [h*LL, h*LL+LL) at word offset hoff + j*32, where
// hoff = h*LL*32 is made opaque (half_off) so every access is base VGPR + immediate
// offset instead of one materialised address per limb.
template <int LL>
__device__ __forceinline__ u32 half_off(int h) {
  u32 o = (u32)h * LL * kHalf;
  asm volatile("" : "+v"(o));
  return o;
}

template <int LL>
__device__ __forceinline__ void slot2_store(u32* bcol, const u32 (&A)[LL], u32 hoff) {
#pragma unroll
  for (int j = 0; j < LL; ++j) bcol[hoff + j * kHalf] = A[j];
}

template <int LL>
__device__ __forceinline__ void slot2_store_uniform(u32* bcol, const u32* __restrict__ src, u32 hoff, int h) {
  const u32* s = src + h * LL;  // two values per limb (one per half): vector loads
#pragma unroll
  for (int j = 0; j < LL; ++j) bcol[hoff + j * kHalf] = s[j];
}

template <int LL>
__device__ __forceinline__ void slot2_store_small(u32* bcol, u32 v, u32 hoff, int h) {
#pragma unroll
  for (int j = 0; j < LL; ++j) bcol[hoff + j * kHalf] = (j == 0 && h == 0) ? v : 0u;
}

template <int LL>
__device__ __forceinline__ void tile2_to_slot(u32* bcol, const Tile& t, u32 soff, u32 hoff) {
#pragma unroll
  for (int j = 0; j < LL; ++j) bcol[hoff + j * kHalf] = t.ld(soff + j * 256u);
}

template <int LL>
__device__ __forceinline__ void slot2_to_tile(const Tile& t, u32 soff, const u32* bcol, u32 hoff) {
#pragma unroll
  for (int j = 0; j < LL; ++j) t.st(bcol[hoff + j * kHalf], soff + j * 256u);
}

// ---- A <- A * B * 2^(-64 LL) mod N ----------------------------------------------------
template <int LL>
__device__ __forceinline__ void mont_mul2(u32 (&A)[LL], const u32* bcol, const u32 (&NV)[LL], const u32 n0inv) {
  static_assert(LL % FPHE_MAC_G == 0, "limbs per lane must be a multiple of the asm group");
  constexpr int L = 2 * LL;
  u32 T[LL];
#pragma unroll
  for (int j = 0; j < LL; ++j) T[j] = 0;
  u32 e0 = 0;
  u32 b = bcol[0];
#pragma unroll 1
  for (int i = 0; i < L; ++i) {
    const u32 bn = bcol[((i + 1) & (L - 1)) * kHalf];
    u32 m, c1, c2, x;
    u64 k2;
    asm volatile(FPHE_ASM_FIRST_GROUP_TPI2
                 : FPHE_FIRST2_OUTS(T, c1, c2, m, x, k2)
                 : FPHE_FIRST2_INS(A, NV, b, n0inv)
                 : FPHE_MAC_CLOBBERS);
#pragma unroll
    for (int g = 1; g < LL / FPHE_MAC_G; ++g) {
      asm volatile(FPHE_ASM_STD_GROUP
                   : FPHE_STD_OUTS(T, g * FPHE_MAC_G, c1, c2, k2)
                   : FPHE_STD2_INS(A, NV, g * FPHE_MAC_G, b, m)
                   : FPHE_MAC_CLOBBERS);
    }
    asm volatile(FPHE_ASM_TAIL_TPI2
                 : FPHE_TAIL2_OUTS(T[LL - 1], e0)
                 : FPHE_TAIL2_INS(x, c1, c2)
                 : "v2", "v3", "vcc");
    b = bn;
  }
  // Fold the low half's pending carry (global limb LL) into the high half.
  u32 z;
  asm volatile(
      "v_mov_b32 %[z], 0\n\t"
      "v_mov_b32 v2, %[e0]\n\t"
      "s_nop 1\n\t"
      "v_permlane32_swap_b32 %[z], v2\n\t"  // z[32..63] <- e0[0..31]; z[0..31] stays 0
      "s_nop 1"
      : [z] "=&v"(z)
      : [e0] "v"(e0)
      : "v2");
  {
    u32 cw = 0;
    asm volatile(FPHE_ASM_ADDSMALL_FIRST : FPHE_ADDSMALL_OUTS(T, 0, cw) : [z] "v"(z) : "vcc");
#pragma unroll
    for (int g = 1; g < LL / FPHE_MAC_G; ++g)
      asm volatile(FPHE_ASM_ADDSMALL_STD : FPHE_ADDSMALL_OUTS(T, g * FPHE_MAC_G, cw) : : "vcc");
    e0 += cw;  // high half: limb 2LL (T < 2N keeps it <= 1); low half: becomes its carry (0)
  }
  const u32 hi_half = (__lane_id() >> 5);
  const u32 top = hi_half ? e0 : 0u;  // global limb 2LL lives in the high half
  // Conditional subtraction: D = T - N across both halves (borrow handed low -> high).
  u32 bw = 0;
#pragma unroll
  for (int g = 0; g < LL / FPHE_MAC_G; ++g)
    asm volatile(FPHE_ASM_SUBV : FPHE_SUB_OUTS(A, g * FPHE_MAC_G, bw) : FPHE_SUBV_INS(T, NV, g * FPHE_MAC_G) : "vcc");
  u32 bin;
  asm volatile(
      "v_mov_b32 %[bin], 0\n\t"
      "v_mov_b32 v2, %[bw]\n\t"
      "s_nop 1\n\t"
      "v_permlane32_swap_b32 %[bin], v2\n\t"  // bin[32..63] <- bw[0..31]
      "s_nop 1"
      : [bin] "=&v"(bin)
      : [bw] "v"(bw)
      : "v2");
  bw = bin;
#pragma unroll
  for (int g = 0; g < LL / FPHE_MAC_G; ++g)
    asm volatile(FPHE_ASM_SUBV : FPHE_SUB_OUTS(A, g * FPHE_MAC_G, bw) : FPHE_SUBV_INS(T, NV, g * FPHE_MAC_G) : "vcc");
  // keep T iff T < N: decided in the high half (final borrow and top limb), sent low.
  u32 keep_h = (top == 0u && bw != 0u) ? 1u : 0u;
  u32 keep;
  asm volatile(
      "v_mov_b32 %[k], %[kh]\n\t"
      "v_mov_b32 v2, %[kh]\n\t"
      "s_nop 1\n\t"
      "v_permlane32_swap_b32 v2, %[k]\n\t"  // k[0..31] <- kh[32..63]; k[32..63] = kh
      "s_nop 1"
      : [k] "=&v"(keep)
      : [kh] "v"(keep_h)
      : "v2");
#pragma unroll
  for (int j = 0; j < LL; ++j) A[j] = keep ? T[j] : A[j];
}

template <int LL>
__device__ __forceinline__ void mont_sqr2(u32 (&A)[LL], u32* bcol, const u32 (&NV)[LL], u32 n0inv, u32 hoff) {
  slot2_store<LL>(bcol, A, hoff);
  mont_mul2<LL>(A, bcol, NV, n0inv);
}

// Fixed-window modexp with a wave-uniform exponent; A in/out in Montgomery form.
// tb: the wave's global table, entry k at byte k*LL*256 (64 lanes x LL limbs).
template <int LL, int W>
__device__ __forceinline__ void powm_uniform2(u32 (&A)[LL], u32* bcol, const Tile& tb, const u32 (&NV)[LL],
                                              const u32 n0inv, const u32* __restrict__ E, const int ebits, u32 hoff) {
  constexpr u32 TE = LL * 256u;
  slot2_store<LL>(bcol, A, hoff);
  tile_store<LL>(tb, 1 * TE, A);
#pragma unroll 1
  for (int k = 2; k < (1 << W); ++k) {
    mont_mul2<LL>(A, bcol, NV, n0inv);
    tile_store<LL>(tb, (u32)k * TE, A);
  }
  const int nwin = (ebits + W - 1) / W;
  auto digit = [&](int w) -> int {
    const int b0 = w * W;
    const int limb = b0 >> 5, off = b0 & 31;
    u32 v = E[limb] >> off;
    if (off + W > 32) v |= E[limb + 1] << (32 - off);
    return (int)(v & ((1u << W) - 1));
  };
  int d = digit(nwin - 1);
  tile_load<LL>(A, tb, (u32)d * TE);
#pragma unroll 1
  for (int w = nwin - 2; w >= 0; --w) {
#pragma unroll 1
    for (int s = 0; s < W; ++s) mont_sqr2<LL>(A, bcol, NV, n0inv, hoff);
    d = digit(w);
    if (d != 0) {
      tile2_to_slot<LL>(bcol, tb, (u32)d * TE, hoff);
      mont_mul2<LL>(A, bcol, NV, n0inv);
    }
  }
}

}  // namespace fphe
