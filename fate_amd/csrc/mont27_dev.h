// Reduced-radix Montgomery arithmetic for gfx950: 27-bit limbs, 64-bit lazy accumulators.
//
// Why (measured): on gfx950 v_mad_u64_u32, v_add_co_u32 and v_addc_co_u32
// all issue at half rate, so a 32-bit-limb CIOS MAC (mad + add_co + addc) costs three
// half-rate issues.  With 27-bit limbs a product is < 2^54 and a 64-bit accumulator
// absorbs every product a column ever receives (<= 2*152 products < 2^62.3), so a MAC
// is ONE v_mad_u64_u32 (D64 = a*b + acc64) with no carry handling inside the product.
// 152 limbs cover 4096-bit moduli (4104 bits): 1.41x the MACs of 128 x 32-bit limbs at
// one third of the instructions.
//
// Layout: an element's NL = 38*TPI limbs are spread over TPI in {1,2,4} ADJACENT lanes
// (lane = TPI*e + q); lane q holds limbs [38q, 38q+38) of A (u32) and T (u64), and of the
// modulus N (u32 VGPRs when TPI > 1; wave-uniform scalar loads when TPI == 1).  Per CIOS
// row the lanes of an element exchange two values with DPP (full-rate VALU, no LDS):
//   m      : quad_perm broadcast from the element's lane 0        (lane i <- lane i&~(TPI-1))
//   X      : the reduction word leaving lane q's bottom limb goes to lane q-1's top limb
//            (row_shl:1: lane i <- lane i+1)
// DPP semantics verified on MI355X by tools/probe/dpp_probe.hip.
//
// Lazy Montgomery: R = 2^(27*NL) >= 4N for every modulus used here, so a product of two
// operands < 2N is < 2N again ((4N^2 + RN)/R <= 2N) and no conditional subtraction is
// needed between products; an operand >= 2N is allowed only against a second operand
// < N with the first < R (then (RN + RN)/R = 2N).  finalize() maps a final value < 2N
// to its canonical residue with one subtraction.
#pragma once
#include "mont_dev.h"
#include "mont27_asm_gen.h"

#ifndef FPHE_TAB_BATCH
#define FPHE_TAB_BATCH 1
#endif
#ifndef FPHE_PIN_BNEXT
#define FPHE_PIN_BNEXT 1
#endif

namespace fphe {
namespace r27 {

constexpr int LB = 27;
constexpr u32 MASK = (1u << LB) - 1u;
constexpr int LL = 38;  // limbs per lane: 38*27 = 1026 bits

// An operand's LL limbs of one lane, packed two per u64: the register allocator then
// places them as aligned VGPR pairs next to the u64 accumulators instead of fragmenting
// the file with 32-bit values in even slots (measured: 234 -> ~160 VGPRs at TPI=4).
struct L27 {
  u64 p[LL / 2];
  __device__ __forceinline__ u32 operator[](int j) const { return (u32)(p[j >> 1] >> ((j & 1) * 32)); }
  __device__ __forceinline__ void set(int j, u32 v) {
    if (j & 1) p[j >> 1] = (p[j >> 1] & 0xffffffffull) | ((u64)v << 32);
    else p[j >> 1] = (p[j >> 1] & 0xffffffff00000000ull) | v;
  }
  __device__ __forceinline__ void set2(int k, u32 lo, u32 hi) { p[k] = ((u64)hi << 32) | lo; }
};

#include "mont27_sq_gen.h"

template <int TPI>
struct Geo {
  static constexpr int E = FPHE_WAVE / TPI;  // elements per wave
  static constexpr int NL = LL * TPI;        // limbs per element
  int lane, q, e;
  __device__ __forceinline__ Geo() {
    lane = (int)(threadIdx.x & 63);
    q = lane & (TPI - 1);
    e = lane / TPI;
  }
};

// D64 = a * b + c in one v_mad_u64_u32.  As inline asm so the 32-bit operands stay 32-bit
// values: the C form (u64)a*b+c makes the compiler hoist zero-extended 64-bit copies of
// loop-invariant limbs (N) out of the row loop, doubling their register cost.
__device__ __forceinline__ u64 mad64(u32 a, u32 b, u64 c) {
  u64 d;
  asm("v_mad_u64_u32 %0, vcc, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c) : "vcc");
  return d;
}
__device__ __forceinline__ u64 mad64s(u32 a, u32 b_uniform, u64 c) {  // b in an SGPR
  u64 d;
  asm("v_mad_u64_u32 %0, vcc, %1, %2, %3" : "=v"(d) : "v"(a), "s"(b_uniform), "v"(c) : "vcc");
  return d;
}

// ---- DPP helpers (wave64, rows of 16 lanes) -------------------------------------------
__device__ __forceinline__ u32 dpp_from_next(u32 x) {  // lane i <- lane i+1 (row_shl:1), row end -> 0
  return (u32)__builtin_amdgcn_update_dpp(0, (int)x, 0x101, 0xf, 0xf, true);
}
__device__ __forceinline__ u32 dpp_from_prev(u32 x) {  // lane i <- lane i-1 (row_shr:1), row start -> 0
  return (u32)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, true);
}
template <int TPI>
__device__ __forceinline__ u32 dpp_bcast(u32 x) {  // lane i <- lane i & ~(TPI-1)
  if constexpr (TPI == 4) return (u32)__builtin_amdgcn_update_dpp(0, (int)x, 0x00, 0xf, 0xf, false);
  else if constexpr (TPI == 2) return (u32)__builtin_amdgcn_update_dpp(0, (int)x, 0xA0, 0xf, 0xf, false);
  else return x;
}
__device__ __forceinline__ u64 dpp_from_next64(u64 x) {
  return ((u64)dpp_from_next((u32)(x >> 32)) << 32) | dpp_from_next((u32)x);
}
__device__ __forceinline__ u64 dpp_from_prev64(u64 x) {
  return ((u64)dpp_from_prev((u32)(x >> 32)) << 32) | dpp_from_prev((u32)x);
}
template <int TPI>
__device__ __forceinline__ u32 dpp_from_top(u32 x) {  // lane i <- lane i | (TPI-1)
  if constexpr (TPI == 4) return (u32)__builtin_amdgcn_update_dpp(0, (int)x, 0xFF, 0xf, 0xf, false);  // [3,3,3,3]
  else if constexpr (TPI == 2) return (u32)__builtin_amdgcn_update_dpp(0, (int)x, 0xF5, 0xf, 0xf, false);  // [1,1,3,3]
  else return x;
}
// OR over the TPI lanes of an element (result in every lane of the element)
template <int TPI>
__device__ __forceinline__ u32 elem_or(u32 x) {
  if constexpr (TPI >= 2) x |= (u32)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xf, 0xf, false);  // [1,0,3,2]
  if constexpr (TPI >= 4) x |= (u32)__builtin_amdgcn_update_dpp(0, (int)x, 0x4E, 0xf, 0xf, false);  // [2,3,0,1]
  return x;
}

// ---- modulus operand: VGPR limbs (TPI > 1) or wave-uniform scalar loads (TPI == 1) -----
template <int TPI>
struct Mod {
  u64 v[TPI > 1 ? LL / 2 : 1];  // per-lane limbs, packed (TPI > 1)
  u32 s[TPI > 1 ? 1 : LL];      // wave-uniform limbs in SGPRs (TPI == 1)
  __device__ __forceinline__ void init(const u32* __restrict__ N, int q) {
    if constexpr (TPI > 1) {
      const u64* n2 = reinterpret_cast<const u64*>(N + q * LL);  // 8-byte aligned (LL even)
#pragma unroll
      for (int k = 0; k < LL / 2; ++k) v[k] = n2[k];
    } else {
#pragma unroll
      for (int j = 0; j < LL; ++j) s[j] = N[j];
    }
  }
  __device__ __forceinline__ u32 operator()(int j) const {
    if constexpr (TPI > 1) return (u32)(v[j >> 1] >> ((j & 1) * 32));
    else return s[j];
  }
  // m * N_j + c
  __device__ __forceinline__ u64 mad(u32 m, int j, u64 c) const {
    if constexpr (TPI > 1) return mad64(m, (*this)(j), c);
    else return mad64s(m, s[j], c);
  }
};

#ifndef FPHE_FUSED
#define FPHE_FUSED 1
#endif
#include "mont27_fused_gen.h"

// ---- A <- A * B * R^-1 (mod N), lazy ---------------------------------------------------
// bcol: this element's column of the wave's LDS operand tile [NL][E] (b_i at bcol[i*E]).
// In: A limbs < 2^27 + 2^12 (almost normalised), B likewise; values < 2N (see header).
// Out: A almost normalised, value < 2N.
template <int TPI>
__device__ __forceinline__ void normalize_almost(const u64 (&T)[LL], L27& A, int q) {
  u64 c = 0;
  u32 lo = 0;
#pragma unroll
  for (int j = 0; j < LL; ++j) {
    const u64 v = T[j] + c;
    const u32 a = (u32)v & MASK;
    c = v >> LB;
    if (j & 1) A.set2(j >> 1, lo, a);
    else lo = a;
  }
  if constexpr (TPI > 1) {
    u64 cin = dpp_from_prev64(c);  // carry leaving the lane below
    if (q == 0) cin = 0;
    const u64 v = (u64)A[0] + cin;
    A.set2(0, (u32)v & MASK, A[1] + (u32)(v >> LB));  // limb 1 < 2^27 + 2^11
  }
}

// One reduction row: m = T_0 n' mod 2^27 (broadcast from the element's lane 0), then
// T = (T + m N) / 2^27.  The word X leaving a lane's bottom limb (old position 38q) lands
// at new position 38q - 1, i.e. X 2^(27(38q-1)) = (X >> 27) 2^(27 38q) + (X mod 2^27)
// 2^(27(38q-1)): its high part stays in the lane's own new bottom limb and only the low 27
// bits move to the top limb of the lane below.  Lane 0's X is 0 mod 2^27 (the point of m),
// so what the previous element's top lane receives from it is 0, as required: no lane
// selects at all.
template <int TPI>
__device__ __forceinline__ void red_row(u64 (&T)[LL], const Mod<TPI>& N, const u32 nprime, int q) {
  (void)q;
  const u32 m = dpp_bcast<TPI>(((u32)T[0] * nprime) & MASK);
  // X = m N_0 + T_0 ; T_{j-1} = m N_j + T_j  (the shift by one limb)
  u64 X;
  if constexpr (TPI > 1) {
    asm volatile(R27_ASM_REDROW : [x] "=&v"(X), R27_T_OPS(T) : [m] "v"(m), R27_N_INS(N, "v") : "vcc", "memory");
    T[0] += X >> LB;
    T[LL - 1] = dpp_from_next64(X & (u64)MASK);  // row end (lane 15): 0, a top lane anyway
  } else {
    asm volatile(R27_ASM_REDROW : [x] "=&v"(X), R27_T_OPS(T) : [m] "v"(m), R27_N_INS(N, "s") : "vcc", "memory");
    T[0] += X >> LB;
    T[LL - 1] = 0;
  }
}

template <int TPI>
__device__ __forceinline__ void mont_mul(L27& A, const u32* bcol, const Mod<TPI>& N, const u32 nprime, int q) {
  constexpr int E = Geo<TPI>::E, NL = Geo<TPI>::NL;
  u64 T[LL];
#pragma unroll
  for (int j = 0; j < LL; ++j) T[j] = 0;
  u32 b = bcol[0];
  if constexpr (FPHE_FUSED && TPI > 1) {
    // one asm block per row (mont27_fused_gen.h); the LDS read of b_{i+1} is issued before
    // the row and waited for after it
    const u32 mk = MASK;
#pragma unroll 1
    for (int i = 0; i < NL; ++i) {
      u32 bn = bcol[(i + 1 < NL ? i + 1 : 0) * E];
      r27f_row<TPI>(T, A, b, N, nprime, mk);
      asm volatile("" : "+v"(bn));
      b = bn;
    }
    normalize_almost<TPI>(T, A, q);
    return;
  }
#pragma unroll 1
  for (int i = 0; i < NL; ++i) {
    // T += A * b_i  (LL MACs, mont27_asm_gen.h).  The memory clobbers pin the LDS read of
    // b_{i+1} between the two row blocks so its latency hides under the reduction row.
    asm volatile(R27_ASM_OPROW : R27_T_OPS(T) : R27_A_INS(A), [b] "v"(b) : "vcc", "memory");
    u32 bn = bcol[(i + 1 < NL ? i + 1 : 0) * E];
    red_row<TPI>(T, N, nprime, q);
#if FPHE_PIN_BNEXT
    asm volatile("" : "+v"(bn));
#endif
    b = bn;
  }
  normalize_almost<TPI>(T, A, q);
}

// ---- A <- A^2 R^-1 (mod N), lazy: half the operand MACs ----------------------------------
// The square needs each unordered limb pair {i, k} once (doubled) and each diagonal a_i^2
// once.  In the shifted CIOS frame, row i adds a_i a_k at position k, and the same pair can
// equally be added by row k at position i.  Positions are fixed to lanes (lane q holds
// [38q, 38q + 38)), and a SIMD row costs the MOST MACs any lane does, so the pairs are
// split to give every lane the same 20-position window per row: row i = 38 s + a (slice s,
// local index a) touches the lane-local positions (a + t) mod 38, t = 0..19, with multiplier
//   t = 0     : 2 a_i if q > s,  a_i if q == s (the diagonal),  0 if q < s
//   t = 1..18 : 2 a_i
//   t = 19    : 2 a_i if q < s,  2 a_i if q == s and a < 19,     0 otherwise.
// Pair (x in slice X, y in slice Y, X < Y, local xa, yb) is then added by row x iff
// (yb - xa) mod 38 in [0, 19) and by row y iff it is in [19, 38); a diagonal-block pair
// a < b by row a iff b - a <= 19, else by row b.  Exactly once either way.  Rows are
// unrolled by 38 so the window's register indices are compile-time; 20 + 38 MACs per row
// against 38 + 38.  Bounds: 2 a_i a_k < 2^55.01 and an absolute column receives <= 77
// operand and <= NL reduction products, < 2^62.3 (the mont_mul bound).
template <int TPI, int a>
__device__ __forceinline__ void sq_rows(u64 (&T)[LL], const L27& A, u32& b, const u32* bs, const u32* bnext,
                                        u32 shf, u32 mkf, u32 mkl0, u32 mkl1, const Mod<TPI>& N, u32 nprime,
                                        int q) {
  constexpr int E = Geo<TPI>::E;
  if constexpr (FPHE_FUSED && TPI > 1) {
    // fused path: the slot holds 2A (sqr), so b is already the doubled limb; shf/mkf are
    // the bit-field offset/width that give 2b (q > s), b (q == s) or 0 (q < s) in one op
    const u32 bf = __builtin_amdgcn_ubfe(b, shf, mkf);
    const u32 bl = b & (a < LL / 2 ? mkl0 : mkl1);
    u32 bn;
    if constexpr (a + 1 < LL) bn = bs[(a + 1) * E];
    else bn = bnext[0];
    r27f_sqrow<TPI, a>(T, A, bf, b, bl, N, nprime, MASK);
    asm volatile("" : "+v"(bn));
    b = bn;
    if constexpr (a + 1 < LL) sq_rows<TPI, a + 1>(T, A, b, bs, bnext, shf, mkf, mkl0, mkl1, N, nprime, q);
    return;
  }
  const u32 b2 = b << 1;
  const u32 bf = (b << shf) & mkf;
  const u32 bl = b2 & (a < LL / 2 ? mkl0 : mkl1);
  r27_sqrow<a>(T, A, bf, b2, bl);
  u32 bn;
  if constexpr (a + 1 < LL) bn = bs[(a + 1) * E];
  else bn = bnext[0];
  red_row<TPI>(T, N, nprime, q);
#if FPHE_PIN_BNEXT
  asm volatile("" : "+v"(bn));  // keep the LDS wait for b_{i+1} after this row's MACs
#endif
  b = bn;
  if constexpr (a + 1 < LL) sq_rows<TPI, a + 1>(T, A, b, bs, bnext, shf, mkf, mkl0, mkl1, N, nprime, q);
}

// bcol must hold A (2A on the fused path) -- sqr() below does that.
template <int TPI>
__device__ __forceinline__ void mont_sqr(L27& A, const u32* bcol, const Mod<TPI>& N, const u32 nprime, int q) {
  constexpr int E = Geo<TPI>::E;
  u64 T[LL];
#pragma unroll
  for (int j = 0; j < LL; ++j) T[j] = 0;
  u32 b = bcol[0];
#pragma unroll 1
  for (int s = 0; s < TPI; ++s) {
    constexpr bool kFused = FPHE_FUSED && TPI > 1;
    // fused: bit-field (offset, width) of the doubled limb; else shift and mask of b
    const u32 shf = kFused ? (q == s ? 1u : 0u) : (q > s ? 1u : 0u);
    const u32 mkf = kFused ? (q > s ? 31u : (q == s ? 30u : 0u)) : (q >= s ? ~0u : 0u);
    const u32 mkl0 = q <= s ? ~0u : 0u;
    const u32 mkl1 = q < s ? ~0u : 0u;
    const u32* bs = bcol + s * LL * E;
    const u32* bnext = s + 1 < TPI ? bs + LL * E : bcol;
    sq_rows<TPI, 0>(T, A, b, bs, bnext, shf, mkf, mkl0, mkl1, N, nprime, q);
  }
  normalize_almost<TPI>(T, A, q);
}

// ---- LDS operand tile helpers ------------------------------------------------------------
// hoff = 38*q*E made opaque so each limb access is base VGPR + immediate offset.
template <int TPI>
__device__ __forceinline__ u32 lds_qoff(int q) {
  u32 o = (u32)q * LL * Geo<TPI>::E;
  asm volatile("" : "+v"(o));
  return o;
}

template <int TPI>
__device__ __forceinline__ void to_slot(u32* bcol, u32 qoff, const L27& A) {
#pragma unroll
  for (int j = 0; j < LL; ++j) bcol[qoff + j * Geo<TPI>::E] = A[j];
}

// uniform NL-limb constant (27-bit limbs) -> slot
template <int TPI>
__device__ __forceinline__ void const_to_slot(u32* bcol, u32 qoff, const u32* __restrict__ C, int q) {
  const u32* c = C + q * LL;
#pragma unroll
  for (int j = 0; j < LL; ++j) bcol[qoff + j * Geo<TPI>::E] = c[j];
}

template <int TPI>
__device__ __forceinline__ void one_to_slot(u32* bcol, u32 qoff, int q) {
#pragma unroll
  for (int j = 0; j < LL; ++j) bcol[qoff + j * Geo<TPI>::E] = (j == 0 && q == 0) ? 1u : 0u;
}

template <int TPI>
__device__ __forceinline__ void sqr(L27& A, u32* bcol, u32 qoff, const Mod<TPI>& N, u32 np, int q) {
  if constexpr (FPHE_FUSED && TPI > 1) {
    // the fused squaring rows read doubled limbs (< 2^29): 2 a_i feeds the off-diagonal
    // MACs directly and the diagonal takes it back halved by the bit-field extract
#pragma unroll
    for (int j = 0; j < LL; ++j) bcol[qoff + j * Geo<TPI>::E] = A[j] << 1;
  } else {
    to_slot<TPI>(bcol, qoff, A);
  }
  mont_sqr<TPI>(A, bcol, N, np, q);
}

// per-lane table in global scratch: entry k, limb j at byte (k*LL + j)*256 (+ lane*4)
__device__ __forceinline__ void tab_store(const Tile& t, u32 k, const L27& A) {
#pragma unroll
  for (int j = 0; j < LL; ++j) t.st(A[j], (k * LL + j) * 256u);
}
__device__ __forceinline__ void tab_load(L27& A, const Tile& t, u32 k) {
#pragma unroll
  for (int j = 0; j < LL; j += 2) A.set2(j >> 1, t.ld((k * LL + j) * 256u), t.ld((k * LL + j + 1) * 256u));
}
// All LL loads are issued before the first LDS write (the scheduler otherwise pairs each
// load with its write, and the waitcnt pass then serialises LL/2 global-memory latencies).
template <int TPI>
__device__ __forceinline__ void tab_to_slot(u32* bcol, u32 qoff, const Tile& t, u32 k) {
  u32 w[LL];
#pragma unroll
  for (int j = 0; j < LL; ++j) w[j] = t.ld((k * LL + j) * 256u);
#if FPHE_TAB_BATCH
  __builtin_amdgcn_sched_barrier(0);
#endif
#pragma unroll
  for (int j = 0; j < LL; ++j) bcol[qoff + j * Geo<TPI>::E] = w[j];
}

// ---- exact normalisation + canonical finish -----------------------------------------------
// A almost normalised (value < 2^(27 NL)) -> exact 27-bit limbs.
template <int TPI>
__device__ __forceinline__ void normalize_exact(L27& A, int q) {
  u32 c = 0;
#pragma unroll
  for (int j = 0; j < LL; ++j) {
    const u32 v = A[j] + c;
    A.set(j, v & MASK);
    c = v >> LB;
  }
#pragma unroll
  for (int r = 1; r < TPI; ++r) {
    u32 cin = dpp_from_prev(c);
    if (q == 0) cin = 0;
    c = 0;
    u32 cc = cin;
#pragma unroll
    for (int j = 0; j < LL; ++j) {
      const u32 v = A[j] + cc;
      A.set(j, v & MASK);
      cc = v >> LB;
    }
    c = cc;
  }
}

// value < 2N (any product output) -> canonical residue mod N, exact limbs.
template <int TPI>
__device__ __forceinline__ void finalize(L27& A, const Mod<TPI>& N, int q) {
  normalize_exact<TPI>(A, q);
  // D = A - N with the borrow rippled through the element's lanes (TPI rounds)
  u32 D[LL];
  int c = 0, top = 0;
#pragma unroll
  for (int j = 0; j < LL; ++j) {
    const int v = (int)A[j] - (int)N(j) + c;
    D[j] = (u32)v & MASK;
    c = v >> LB;  // 0 or -1
  }
  top = c;
#pragma unroll
  for (int r = 1; r < TPI; ++r) {
    int cin = (int)dpp_from_prev((u32)c);
    if (q == 0) cin = 0;
#pragma unroll
    for (int j = 0; j < LL; ++j) {
      const int v = (int)D[j] + cin;
      D[j] = (u32)v & MASK;
      cin = v >> LB;
    }
    c = cin;
    top += c;
  }
  const bool lt = (int)dpp_from_top<TPI>((u32)top) < 0;  // A < N: keep A
#pragma unroll
  for (int j = 0; j < LL; ++j) A.set(j, lt ? A[j] : D[j]);
}

// ---- radix conversion 2^32 <-> 2^27 ----------------------------------------------------------
// A lane's 1026-bit chunk starts at bit 1026q = 32*(32q) + 2q of the element (bit offset sh
// of word w0 in general).  get(k) returns word w0 + k (k = 0..33), 0 past the end of the
// number: callers read through buffer descriptors sized to the number, whose hardware range
// check returns 0, so no per-lane guards (and no divergent branches) are needed.
template <class Get>
__device__ __forceinline__ void load_chunk(L27& A, u32 sh, Get get) {
  u32 W[34];
#pragma unroll
  for (int k = 0; k < 34; ++k) W[k] = get(k);
#pragma unroll
  for (int k = 0; k < 33; ++k) W[k] = __builtin_amdgcn_alignbit(W[k + 1], W[k], sh);
#pragma unroll
  for (int j = 0; j < LL; ++j) {
    const int bit = LB * j, w = bit >> 5, off = bit & 31;
    A.set(j, __builtin_amdgcn_alignbit(W[w + 1], W[w], off) & MASK);
  }
}

// Store this lane's chunk (exact limbs) as words [32q, 32q + 32) of the element, merging
// the two bits that overflow into the next lane's first word (TPI lanes adjacent).
// put(k, v) writes word 32q + k.
template <int TPI, class Put>
__device__ __forceinline__ void store_chunk(const L27& A, int q, Put put) {
  u32 W[33];
#pragma unroll
  for (int k = 0; k < 33; ++k) W[k] = 0;
#pragma unroll
  for (int j = 0; j < LL; ++j) {
    const int bit = LB * j, w = bit >> 5, off = bit & 31;
    W[w] |= A[j] << off;
    if (off > 32 - LB) W[w + 1] |= A[j] >> (32 - off);
  }
  const u32 sh = 2u * (u32)q;  // 1026*q = 32*(32q) + 2q
  u32 G[33];
#pragma unroll
  for (int k = 0; k < 33; ++k) {
    const u64 pair = ((u64)W[k] << 32) | (k ? W[k - 1] : 0u);
    G[k] = (u32)((pair << sh) >> 32);
  }
  if constexpr (TPI > 1) {
    u32 spill = dpp_from_prev(G[32]);  // top bits of the lane below
    if (q == 0) spill = 0;
    G[0] |= spill;
  }
#pragma unroll
  for (int k = 0; k < 32; ++k) put(k, G[k]);
}

}  // namespace r27
}  // namespace fphe
