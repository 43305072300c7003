// Shared device helpers for gfx950 (CDNA4): buffer-descriptor tiles, the wave-uniform
// 32-bit CIOS product the decrypt CRT tail uses for its one-off products mod p and q
// (fate_phe.hip crt_tail / crt_combine), and small wave reductions.  The ciphertext
// engine itself is the reduced-radix one (mont27_dev.h).
//
// 32-bit CIOS layout: one element per lane; its L limbs live in VGPRs (A[L]) with the
// accumulator T[L+1]; the runtime-indexed operand b_i is staged in an LDS [limb][lane]
// slot (64 consecutive dwords per wave, conflict-free); the modulus is wave-uniform and
// read through scalar loads.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "mont_asm_gen.h"

#define FPHE_WAVE 64

namespace fphe {

typedef uint32_t u32;
typedef uint64_t u64;
typedef uint8_t u8;

// ---- global tiles through buffer descriptors -------------------------------------------
// Device vectors are tile-major: element e of a vector with L limbs per element lives in
// tile e/64, lane e%64: word ((e/64)*L + j)*64 + e%64.  A wave owns one tile per step, so
// limb j of all its 64 elements is one contiguous 256-byte row.  Addressing is a
// wave-uniform buffer descriptor + scalar byte offset (j*256 + ...) + lane*4, which keeps
// per-limb addresses out of VGPRs entirely.
struct Tile {
  __amdgpu_buffer_rsrc_t r;
  u32 vo;  // lane * 4
  __device__ __forceinline__ u32 ld(u32 soff) const { return __builtin_amdgcn_raw_buffer_load_b32(r, vo, soff, 0); }
  __device__ __forceinline__ void st(u32 v, u32 soff) const { __builtin_amdgcn_raw_buffer_store_b32(v, r, vo, soff, 0); }
};

__device__ __forceinline__ Tile make_tile(const void* base, u32 bytes, int lane) {
  Tile t;
  t.r = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
  t.vo = (u32)lane * 4u;
  return t;
}

// ---- LDS slot / tile helpers ----------------------------------------------------------
// `slot` points at this lane's column of a [limb][64] LDS tile.
template <int L>
__device__ __forceinline__ void slot_store_uniform(u32* slot, const u32* __restrict__ src) {
#pragma unroll
  for (int j = 0; j < L; ++j) slot[j * FPHE_WAVE] = src[j];
}

// entry-relative scalar byte offsets: limb j of entry k of an L-limb tile table
template <int L>
__device__ __forceinline__ void tile_load(u32 (&A)[L], const Tile& t, u32 soff) {
#pragma unroll
  for (int j = 0; j < L; ++j) A[j] = t.ld(soff + j * 256u);
}

// ---- Montgomery multiplication (CIOS) ------------------------------------------------
// A <- A * B * 2^(-32L) mod N, with B = slot[i*64], i < L.  Requires A < 2^(32L),
// B < N; output fully reduced to [0, N).  Each row i runs the operand chain
// T += A*b_i and the reduction chain T = (T + m*N) / 2^32 interleaved, 16 limbs per asm
// block (mont_asm_gen.h), 3 VALU ops per MAC.
template <int L>
__device__ __forceinline__ void mont_mul(u32 (&A)[L], const u32* slot,
                                         const u32* __restrict__ N, const u32 n0inv) {
  static_assert(L % FPHE_MAC_G == 0, "limb count must be a multiple of the asm group");
  u32 T[L + 1];
#pragma unroll
  for (int j = 0; j <= L; ++j) T[j] = 0;
  u32 b = slot[0];
#pragma unroll 1
  for (int i = 0; i < L; ++i) {
    // N through the constant address space (-> s_load), with an opaque zero offset so the
    // loads are re-issued per row instead of LICM pinning L SGPRs for the whole loop.
    u32 zoff = 0;
    asm volatile("" : "+s"(zoff));
    const __attribute__((address_space(4))) u32* NR =
        (const __attribute__((address_space(4))) u32*)(N) + zoff;
    const u32 bn = slot[((i + 1) & (L - 1)) * FPHE_WAVE];
    u32 m, c1, c2;
    u64 k2;
    asm volatile(FPHE_ASM_FIRST_GROUP
                 : FPHE_FIRST_OUTS(T, c1, c2, m, k2)
                 : FPHE_FIRST_INS(A, NR, b, n0inv)
                 : FPHE_MAC_CLOBBERS);
#pragma unroll
    for (int g = 1; g < L / FPHE_MAC_G; ++g) {
      asm volatile(FPHE_ASM_STD_GROUP
                   : FPHE_STD_OUTS(T, g * FPHE_MAC_G, c1, c2, k2)
                   : FPHE_STD_INS(A, NR, g * FPHE_MAC_G, b, m)
                   : FPHE_MAC_CLOBBERS);
    }
    u32 t1;
    asm volatile(
        "v_add_co_u32 %[tl], vcc, %[tl], %[c1]\n\t"
        "v_addc_co_u32 %[t1], vcc, 0, 0, vcc\n\t"
        "v_add_co_u32 %[tlm], %[k2], %[tl], %[c2]\n\t"
        "v_addc_co_u32 %[tl], %[k2], %[t1], 0, %[k2]"
        : [tl] "+v"(T[L]), [tlm] "+v"(T[L - 1]), [t1] "=&v"(t1), [k2] "=&s"(k2)
        : [c1] "v"(c1), [c2] "v"(c2)
        : "vcc");
    b = bn;
  }
  // T < 2N: conditional subtraction, A = T - N with a VALU borrow chain
  {
    u32 zoff = 0;
    asm volatile("" : "+s"(zoff));
    const __attribute__((address_space(4))) u32* NR =
        (const __attribute__((address_space(4))) u32*)(N) + zoff;
    u32 bw = 0;
    asm volatile(FPHE_ASM_SUB_FIRST : FPHE_SUB_OUTS(A, 0, bw) : FPHE_SUB_INS(T, NR, 0) : "v0", "vcc");
#pragma unroll
    for (int g = 1; g < L / FPHE_MAC_G; ++g) {
      asm volatile(FPHE_ASM_SUB_STD : FPHE_SUB_OUTS(A, g * FPHE_MAC_G, bw) : FPHE_SUB_INS(T, NR, g * FPHE_MAC_G)
                   : "v0", "vcc");
    }
    const bool keep = (T[L] == 0) & (bw != 0);  // T < N
#pragma unroll
    for (int j = 0; j < L; ++j) A[j] = keep ? T[j] : A[j];
  }
}

// ---- small helpers ------------------------------------------------------------------
__device__ __forceinline__ int wave_max_int(int v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const int o = __shfl_xor(v, off, FPHE_WAVE);
    v = o > v ? o : v;
  }
  return v;
}

}  // namespace fphe
