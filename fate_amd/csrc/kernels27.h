// Reduced-radix (27-bit limb) modexp kernels: encrypt, decrypt (modexp phase), ct-add,
// ct x pt.  Included by fate_phe.hip after KeyArgs / nude_to_slot / helpers.
// Geometry: TPI adjacent lanes per element (r27::Geo), E = 64/TPI elements per wave; a
// wave's E elements always sit in one 64-element memory tile, so the memory tile index is
// wave-uniform and only the column (element % 64) is per lane.
#pragma once
#include "mont27_dev.h"
#include "inv27.h"

// Montgomery-engine kernels target 2 waves per SIMD (<= 256 VGPRs, no AGPR overflow): the
// v_mad_u64_u32 stream needs two waves to issue at full rate.  The encrypt
// kernel runs at 3 (<= 168 VGPRs; the compiler spills ~59 dwords, touched once per general
// row and 3 times per 38 squaring rows): +1.2-2.2% same-box; the half-size modexps of
// decrypt and key-holder encrypt likewise (+1.5%) (profiles/r01f_ab_occ3.txt).
#ifndef FPHE_ENC_OCC
#define FPHE_ENC_OCC 3
#endif
#define FPHE_OCC2 __attribute__((amdgpu_waves_per_eu(2)))
// ct-add / ct x pt / squeeze run at 3 waves too (same-box A/B, profiles/r02/
// r02f_ab_occ3_ops.txt: add +5%, ct x pt +1%); the segmented fold stays at 2 (-7% at 3).
// Round 1's 3-wave k_add27<64> memory fault was the register allocator reusing a
// per-lane buffer descriptor's VGPRs for a spill reload inside the readfirstlane loop
// the compiler builds around such a load; the kernels no longer pick a
// descriptor per lane, and tools/wfcheck.py checks every listing for such loops.
#ifndef FPHE_MISC_OCC
#define FPHE_MISC_OCC 3
#endif
#ifndef FPHE_FOLD_OCC
#define FPHE_FOLD_OCC 2
#endif
#define FPHE_OCC_MISC __attribute__((amdgpu_waves_per_eu(FPHE_MISC_OCC)))
#define FPHE_OCC_FOLD __attribute__((amdgpu_waves_per_eu(FPHE_FOLD_OCC)))
#define FPHE_OCC_ENC __attribute__((amdgpu_waves_per_eu(FPHE_ENC_OCC)))
// code-shape switches of the vector-op kernels (A/B and fault bisection):
// wave-uniform loop trip counts in SGPRs, and per-lane operand choice by loading both
// operands and selecting (never a per-lane buffer descriptor)
#ifndef FPHE_UNIFORM_LOOPS
#define FPHE_UNIFORM_LOOPS 1
#endif
#ifndef FPHE_SELECT_LOADS
#define FPHE_SELECT_LOADS 1
#endif
#ifndef FPHE_POW_OCC
#define FPHE_POW_OCC 3
#endif
#define FPHE_OCC_POW __attribute__((amdgpu_waves_per_eu(FPHE_POW_OCC)))

namespace {

using namespace fphe::r27;

// window-table entries per wave for powm27<., W>: entry 0 for the caller + 2^(W-1) odd powers
template <int W>
constexpr u32 kTabEntries = 1u + (1u << (W - 1));

// word w of element column `col` in a tile-major [.][rows][64] u32 tile: per-lane voffset
__device__ __forceinline__ u32 tld(const __amdgpu_buffer_rsrc_t& r, u32 col, u32 w) {
  return __builtin_amdgcn_raw_buffer_load_b32(r, (col + 64u * w) * 4u, 0, 0);
}
__device__ __forceinline__ void tst(const __amdgpu_buffer_rsrc_t& r, u32 col, u32 w, u32 v) {
  __builtin_amdgcn_raw_buffer_store_b32(v, r, (col + 64u * w) * 4u, 0, 0);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, u32 bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

// Words w0 + k of one element column of a tile-major [rows][64] u32 tile.  The descriptor
// covers exactly the tile, so reads past `rows` return 0 and writes past it are dropped
// (raw-buffer range check on voffset).  vb is opaque so the per-word addresses stay
// "vb + const" (folded into the instruction offset) instead of being hoisted as one VGPR
// per word.
struct ColIO {
  __amdgpu_buffer_rsrc_t r;
  u32 vb;
  __device__ __forceinline__ u32 ld(int k) const {
    return __builtin_amdgcn_raw_buffer_load_b32(r, vb + (u32)k * 256u, 0, 0);
  }
  __device__ __forceinline__ void st(int k, u32 v) const {
    __builtin_amdgcn_raw_buffer_store_b32(v, r, vb + (u32)k * 256u, 0, 0);
  }
};
__device__ __forceinline__ ColIO colio(const u32* tile_base, u32 rows, u32 col, u32 w0) {
  ColIO c;
  c.r = rsrc(tile_base, rows * 256u);
  u32 vb = (col + 64u * w0) * 4u;
  asm volatile("" : "+v"(vb));
  c.vb = vb;
  return c;
}

// Sliding-window modexp with a wave-uniform exponent (27-bit engine).  In: A = X in
// Montgomery form (< 2N).  Out: X^E in Montgomery form (< 2N).  Table entries
// [1, 1 + 2^(W-1)) hold the odd powers X^1, X^3, ..., X^(2^W - 1); entry 0 stays free for
// the caller.  The window schedule depends only on E, which is the same for every lane,
// so it is computed on the scalar unit and control flow never diverges.  For E = n
// (2048 bits, W = 6) this is ~2,373 products against 2,475 for the fixed w=5 window.
template <int TPI, int W>
__device__ __forceinline__ void powm27(L27& A, u32* bcol, u32 qoff, const Tile& tb, const Mod<TPI>& N,
                                       u32 np, const u32* __restrict__ Ex, int ebits, int q) {
  constexpr u32 kOdd = 1u << (W - 1);
  tab_store(tb, 1, A);                 // X
  to_slot<TPI>(bcol, qoff, A);
  mont_mul<TPI>(A, bcol, N, np, q);    // X^2 (general product: keeps one unrolled squaring body)
  to_slot<TPI>(bcol, qoff, A);         // slot = X^2 for the table build
  tab_load(A, tb, 1);
#pragma unroll 1
  for (u32 k = 1; k < kOdd; ++k) {
    mont_mul<TPI>(A, bcol, N, np, q);  // X^(2k+1)
    tab_store(tb, 1 + k, A);
  }
  auto bit = [&](int i) -> u32 { return (Ex[i >> 5] >> (i & 31)) & 1u; };
  // window [j, i]: the lowest set bit j >= i - W + 1, value odd
  auto window = [&](int i, int& j) -> u32 {
    j = i - W + 1 < 0 ? 0 : i - W + 1;
    while (!bit(j)) ++j;
    u32 v = 0;
    for (int t = i; t >= j; --t) v = (v << 1) | bit(t);
    return v;
  };
  int i = ebits - 1;
  int j;
  u32 v = window(i, j);
  tab_load(A, tb, 1 + (v >> 1));
  i = j - 1;
  // each step: the zero run, then the next window's squarings, then one table product.
  // One squaring call site: mont_sqr is a 38-row unrolled body, kept once in the I-cache.
#pragma unroll 1
  while (i >= 0) {
    int nsq = 0;
    while (i >= 0 && !bit(i)) {
      ++nsq;
      --i;
    }
    const bool mul = i >= 0;
    if (mul) {
      v = window(i, j);
      nsq += i - j + 1;
      i = j - 1;
    }
#pragma unroll 1
    for (int t = 0; t < nsq; ++t) sqr<TPI>(A, bcol, qoff, N, np, q);
    if (mul) {
      tab_to_slot<TPI>(bcol, qoff, tb, 1 + (v >> 1));
      mont_mul<TPI>(A, bcol, N, np, q);
    }
  }
}

// ======================================================================================
// encrypt (27-bit engine): TPI = 4 for 2048-bit keys (n^2: 152 limbs), 2 for 1024-bit.
// ======================================================================================
template <int L, int W>
__global__ __launch_bounds__(kBlock) FPHE_OCC_ENC void k_encrypt27(KeyArgs K, const u32* __restrict__ P, u32 lp,
                                                      const u8* __restrict__ neg, size_t count, int obf,
                                                      const u32* __restrict__ rin, u32* __restrict__ Cout,
                                                      u8* __restrict__ sout, u32* __restrict__ scratch, u32 ldsw) {
  constexpr int TPI = L / 32;  // 152 limbs for 4096-bit n^2, 76 for 2048-bit
  using G = Geo<TPI>;
  constexpr int E = G::E;
  constexpr u32 L32 = L, L1 = L / 2;
  extern __shared__ __attribute__((aligned(16))) u32 lds[];
  G g;
  const u32 wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const u32 gw = blockIdx.x * kWavesPerBlock + wib, nw = gridDim.x * kWavesPerBlock;
  u32* bcol = lds + wib * ldsw * E + g.e;
  const u32 qoff = lds_qoff<TPI>(g.q);
  const Tile tb = make_tile(scratch + (size_t)gw * ((size_t)kTabEntries<W> * LL * FPHE_WAVE),
                            kTabEntries<W> * LL * 256u, g.lane);
  Mod<TPI> N;
  N.init(K.N2_27, g.q);
  const u32 np = K.n2_np27;
  const u32 nwt = (u32)((count + E - 1) / E);
  for (u32 wt = gw; wt < nwt; wt += nw) {
    const size_t ebase = (size_t)wt * E;
    const u32 tile = (u32)(ebase >> 6);
    const u32 col = (u32)(ebase & 63) + (u32)g.e;
    const size_t elem = ebase + g.e;
    // 1. nude ciphertext 1 + m n (32-bit words) into the LDS tile, rows [0, L32)
    Tile Pt = make_tile(P + (size_t)tile * lp * FPHE_WAVE, lp * 256u, 0);
    Pt.vo = col * 4u;
    bool mneg = false;
    if (g.q == 0) {
      mneg = nude_to_slot<L, E>(bcol, K, Pt, lp, neg[elem] != 0);
      bcol[L * E] = 0;  // the top lane's chunk window reads two words past the number
      bcol[(L + 1) * E] = 0;
    }
    const ColIO Co = colio(Cout + (size_t)tile * L32 * FPHE_WAVE, L32, col, 32u * g.q);
    L27 A;
    {
      const u32* src = bcol + 32 * g.q * E;
      load_chunk(A, 2u * g.q, [&](int k) { return src[k * E]; });
    }
    if (!obf) {
      normalize_exact<TPI>(A, g.q);
      store_chunk<TPI>(A, g.q, [&](int k, u32 v) { Co.st(k, v); });
    } else {
      tab_store(tb, 0, A);  // C_nude, 27-bit
      const ColIO Ri = colio(rin + (size_t)tile * L1 * FPHE_WAVE, L1, col, 32u * g.q);
      load_chunk(A, 2u * g.q, [&](int k) { return Ri.ld(k); });
      const_to_slot<TPI>(bcol, qoff, K.N2R2_27, g.q);
      mont_mul<TPI>(A, bcol, N, np, g.q);                                 // r R
      powm27<TPI, W>(A, bcol, qoff, tb, N, np, K.n, K.nbits, g.q);        // r^n R
      tab_to_slot<TPI>(bcol, qoff, tb, 0);
      mont_mul<TPI>(A, bcol, N, np, g.q);                                 // r^n * C_nude (< 2N)
      finalize<TPI>(A, N, g.q);
      store_chunk<TPI>(A, g.q, [&](int k, u32 v) { Co.st(k, v); });
    }
    if (g.q == 0 && elem < count) sout[elem] = mneg ? 1 : 0;
  }
}

// ======================================================================================
// Half-size modexps mod p^2 and q^2 (TPI = 2 for 2048-bit keys), two uses:
//  decrypt (ENC = false): y_s = c^(s-1) mod s^2 for s in {p, q} (paillier/src/lib.rs:174-176,
//    the pow_mod of h_function); the CRT tail runs in k_decrypt_crt.
//  key-holder encrypt (ENC = true): x_s = r^n mod s^2 = r^(n mod s(s-1)) mod s^2 (the order
//    of (Z/s^2)^* is s(s-1)); k_encrypt_crt27 recombines x_p, x_q into r^n mod n^2 -- the
//    same integer paillier/src/lib.rs:94-98 computes with the public key alone.
// Output: 32-bit words to Y[tile][2*L1][64] (s = p rows [0,L1), s = q rows [L1, 2L1)).
// ======================================================================================
template <int TPI, int W, bool ENC>
__device__ __forceinline__ void pow_half27(const u32* intile, u32 col, u32 inrows, u32* bcol, u32 qoff,
                                           const Tile& tb, const u32* __restrict__ S2, u32 np,
                                           const u32* __restrict__ R1, const u32* __restrict__ R2,
                                           const u32* __restrict__ ex, int ex_bits, int q, L27& A) {
  constexpr int NL = Geo<TPI>::NL;
  // opaque modulus pointer: keeps LICM from hoisting both halves' limbs (p^2 and q^2) out
  // of the element loop, which would hold 2 x 38 VGPRs for the whole kernel
  const u32* S2o = S2;
  asm volatile("" : "+s"(S2o));
  Mod<TPI> N;
  N.init(S2o, q);
  if constexpr (ENC) {
    // r < n < 2^(27 NL) = R: one product with R^2 gives r R mod s^2 (< 2N)
    const ColIO Ri = colio(intile, inrows, col, 32u * q);
    load_chunk(A, 2u * q, [&](int k) { return Ri.ld(k); });
    const_to_slot<TPI>(bcol, qoff, R2, q);
    mont_mul<TPI>(A, bcol, N, np, q);
  } else {
    // c = c_lo + R c_hi (R = 2^(27 NL)):  X = mont(c_lo, R mod s^2) + mont(c_hi, R^2 mod s^2)
    // = c mod s^2 up to < 4N (c_lo < R against R1 < N, c_hi tiny); then X R via R^2.
    L27 B;
    {
      const u32 bit0 = 27u * NL + 1026u * q;
      const ColIO Ci = colio(intile, inrows, col, bit0 >> 5);
      load_chunk(B, bit0 & 31u, [&](int k) { return Ci.ld(k); });
    }
    const_to_slot<TPI>(bcol, qoff, R2, q);
    mont_mul<TPI>(B, bcol, N, np, q);
    tab_store(tb, 0, B);  // parked in the (otherwise unused) table entry 0, not in registers
    {
      const ColIO Ci = colio(intile, inrows, col, 32u * q);
      load_chunk(A, 2u * q, [&](int k) { return Ci.ld(k); });
    }
    const_to_slot<TPI>(bcol, qoff, R1, q);
    mont_mul<TPI>(A, bcol, N, np, q);
    tab_load(B, tb, 0);
#pragma unroll
    for (int j = 0; j < LL; ++j) A.set(j, A[j] + B[j]);
    normalize_exact<TPI>(A, q);  // < 4N, only ever multiplied by R^2 < N next
    const_to_slot<TPI>(bcol, qoff, R2, q);
    mont_mul<TPI>(A, bcol, N, np, q);  // c R, < 2N
  }
  powm27<TPI, W>(A, bcol, qoff, tb, N, np, ex, ex_bits, q);
  one_to_slot<TPI>(bcol, qoff, q);
  mont_mul<TPI>(A, bcol, N, np, q);  // leave Montgomery form (< 2N)
  finalize<TPI>(A, N, q);
}

// In: decrypt -- ciphertexts C [T][L][64]; encrypt -- nonces r [T][L/2][64].
template <int L, int W, bool ENC>
__global__ __launch_bounds__(kBlock) FPHE_OCC_POW void k_pow_half27(KeyArgs K, const u32* __restrict__ In, size_t count,
                                                       u32* __restrict__ Y, u32* __restrict__ scratch, u32 ldsw) {
  constexpr int TPI = L / 64;  // p^2, q^2: 76 limbs for 2048-bit keys, 38 for 1024-bit
  using G = Geo<TPI>;
  constexpr int E = G::E;
  constexpr u32 L1 = L / 2, IN = ENC ? L1 : L;
  extern __shared__ __attribute__((aligned(16))) u32 lds[];
  G g;
  const u32 wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const u32 gw = blockIdx.x * kWavesPerBlock + wib, nw = gridDim.x * kWavesPerBlock;
  u32* bcol = lds + wib * ldsw * E + g.e;
  const u32 qoff = lds_qoff<TPI>(g.q);
  const Tile tb = make_tile(scratch + (size_t)gw * ((size_t)kTabEntries<W> * LL * FPHE_WAVE),
                            kTabEntries<W> * LL * 256u, g.lane);
  const u32 nwt = (u32)((count + E - 1) / E);
  for (u32 wt = gw; wt < nwt; wt += nw) {
    const size_t ebase = (size_t)wt * E;
    const u32 tile = (u32)(ebase >> 6);
    const u32 col = (u32)(ebase & 63) + (u32)g.e;
    const u32* intile = In + (size_t)tile * IN * FPHE_WAVE;
    u32* ytile = Y + (size_t)tile * 2 * L1 * FPHE_WAVE;
    // the two halves in a rolled loop: one inlined copy of the modexp (I-cache)
#pragma unroll 1
    for (u32 h = 0; h < 2; ++h) {
      const bool hq = h != 0;
      const u32* ex;
      int exb;
      if constexpr (ENC) {
        ex = hq ? K.eq : K.ep;
        exb = hq ? K.eq_bits : K.ep_bits;
      } else {
        ex = hq ? K.qm1 : K.pm1;
        exb = hq ? K.qm1_bits : K.pm1_bits;
      }
      L27 A;
      pow_half27<TPI, W, ENC>(intile, col, IN, bcol, qoff, tb, hq ? K.Q2_27 : K.P2_27, hq ? K.q2_np27 : K.p2_np27,
                              hq ? K.Q2R1_27 : K.P2R1_27, hq ? K.Q2R2_27 : K.P2R2_27, ex, exb, g.q, A);
      const ColIO Yo = colio(ytile, 2 * L1, col, h * L1 + 32u * g.q);
      store_chunk<TPI>(A, g.q, [&](int k, u32 v) { Yo.st(k, v); });
    }
  }
}

// ======================================================================================
// key-holder encrypt, recombination: C = (1 + m n) (x_p Kp + x_q Kq) mod n^2, sign (m < 0)
// (paillier/src/lib.rs:104-121 with r^n from the CRT halves in Y; bit-identical to the
// public-key path for the same r).
// ======================================================================================
template <int L>
__global__ __launch_bounds__(kBlock) FPHE_OCC2 void k_encrypt_crt27(KeyArgs K, const u32* __restrict__ P, u32 lp,
                                                          const u8* __restrict__ neg, size_t count,
                                                          const u32* __restrict__ Y, u32* __restrict__ Cout,
                                                          u8* __restrict__ sout, u32 ldsw) {
  constexpr int TPI = L / 32;
  using G = Geo<TPI>;
  constexpr int E = G::E;
  constexpr u32 L32 = L, L1 = L / 2;
  extern __shared__ __attribute__((aligned(16))) u32 lds[];
  G g;
  const u32 wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const u32 gw = blockIdx.x * kWavesPerBlock + wib, nw = gridDim.x * kWavesPerBlock;
  u32* bcol = lds + wib * ldsw * E + g.e;
  const u32 qoff = lds_qoff<TPI>(g.q);
  Mod<TPI> N;
  N.init(K.N2_27, g.q);
  const u32 np = K.n2_np27;
  const u32 nwt = (u32)((count + E - 1) / E);
  for (u32 wt = gw; wt < nwt; wt += nw) {
    const size_t ebase = (size_t)wt * E;
    const u32 tile = (u32)(ebase >> 6);
    const u32 col = (u32)(ebase & 63) + (u32)g.e;
    const size_t elem = ebase + g.e;
    const u32* ytile = Y + (size_t)tile * 2 * L1 * FPHE_WAVE;
    L27 A, B;
    // x_p Kp + x_q Kq: descriptors of L1 rows each, so words past a half read as 0
    {
      const ColIO Xi = colio(ytile, L1, col, 32u * g.q);
      load_chunk(A, 2u * g.q, [&](int k) { return Xi.ld(k); });
    }
    const_to_slot<TPI>(bcol, qoff, K.KpR_27, g.q);
    mont_mul<TPI>(A, bcol, N, np, g.q);  // x_p Kp (< 2N)
#pragma unroll
    for (int k = 0; k < LL / 2; ++k) B.p[k] = A.p[k];
    {
      const ColIO Xi = colio(ytile + L1 * FPHE_WAVE, L1, col, 32u * g.q);
      load_chunk(A, 2u * g.q, [&](int k) { return Xi.ld(k); });
    }
    const_to_slot<TPI>(bcol, qoff, K.KqR_27, g.q);
    mont_mul<TPI>(A, bcol, N, np, g.q);  // x_q Kq (< 2N)
#pragma unroll
    for (int j = 0; j < LL; ++j) A.set(j, A[j] + B[j]);
    normalize_exact<TPI>(A, g.q);        // r^n + k n^2, < 4N, exact limbs
#pragma unroll
    for (int k = 0; k < LL / 2; ++k) B.p[k] = A.p[k];
    // nude ciphertext 1 + m n (32-bit words) into the LDS column, then to 27-bit limbs
    Tile Pt = make_tile(P + (size_t)tile * lp * FPHE_WAVE, lp * 256u, 0);
    Pt.vo = col * 4u;
    bool mneg = false;
    if (g.q == 0) {
      mneg = nude_to_slot<L, E>(bcol, K, Pt, lp, neg[elem] != 0);
      bcol[L * E] = 0;  // the top lane's chunk window reads two words past the number
      bcol[(L + 1) * E] = 0;
    }
    {
      const u32* src = bcol + 32 * g.q * E;
      load_chunk(A, 2u * g.q, [&](int k) { return src[k * E]; });
    }
    const_to_slot<TPI>(bcol, qoff, K.N2R2_27, g.q);
    mont_mul<TPI>(A, bcol, N, np, g.q);  // C_nude R (< 2N)
    to_slot<TPI>(bcol, qoff, A);
#pragma unroll
    for (int k = 0; k < LL / 2; ++k) A.p[k] = B.p[k];
    mont_mul<TPI>(A, bcol, N, np, g.q);  // r^n C_nude (4N x 2N operands: < 2N since R >= 256 N)
    finalize<TPI>(A, N, g.q);
    const ColIO Co = colio(Cout + (size_t)tile * L32 * FPHE_WAVE, L32, col, 32u * g.q);
    store_chunk<TPI>(A, g.q, [&](int k, u32 v) { Co.st(k, v); });
    if (g.q == 0 && elem < count) sout[elem] = mneg ? 1 : 0;
  }
}

// ======================================================================================
// ct-add (fixedpoint_paillier/src/lib.rs:301-333), 27-bit engine.
// Slot i of the launch computes element ord[i] (ord == nullptr: element i), so the host can
// hand the elements over in exponent-gap order -- a wave pays for its largest gap -- with
// no gather or scatter copies: operands and results are addressed through whole-vector
// buffer descriptors with a per-lane byte offset (the vector must be < 4 GiB, the host
// splits larger ones).  Lanes past `count` get the descriptor's size as offset: their
// loads return 0 and their stores are dropped by the hardware range check.
// ======================================================================================
template <int L>
__global__ __launch_bounds__(kBlock) FPHE_OCC_MISC void k_add27(KeyArgs K, const u32* __restrict__ Ca, const u8* __restrict__ sa,
                                                  const int32_t* __restrict__ ea, const u32* __restrict__ Cb,
                                                  const u8* __restrict__ sb, const int32_t* __restrict__ eb,
                                                  int bstride, size_t count, const int32_t* __restrict__ ord,
                                                  u32* __restrict__ Co, u8* __restrict__ so, int32_t* __restrict__ eo,
                                                  u32 ldsw) {
  constexpr int TPI = L / 32;
  using G = Geo<TPI>;
  constexpr int E = G::E;
  constexpr u32 L32 = L;
  extern __shared__ __attribute__((aligned(16))) u32 lds[];
  G g;
  const u32 wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const u32 gw = blockIdx.x * kWavesPerBlock + wib, nw = gridDim.x * kWavesPerBlock;
  u32* bcol = lds + wib * ldsw * E + g.e;
  const u32 qoff = lds_qoff<TPI>(g.q);
  Mod<TPI> N;
  N.init(K.N2_27, g.q);
  const u32 np = K.n2_np27;
  const u32 vbytes = (u32)((count + FPHE_WAVE - 1) / FPHE_WAVE) * L32 * 256u;
  const __amdgpu_buffer_rsrc_t ra = rsrc(Ca, vbytes), ro = rsrc(Co, vbytes);
  const __amdgpu_buffer_rsrc_t rb = rsrc(Cb, bstride ? vbytes : L32 * 256u);
  // byte offset of word 32q of element e (tile-major [tiles][L][64])
  auto voff = [&](size_t e) -> u32 { return (u32)(((e >> 6) * L32 + 32u * (u32)g.q) * FPHE_WAVE + (e & 63)) * 4u; };
  auto io = [&](const __amdgpu_buffer_rsrc_t& r, u32 vb) {
    asm volatile("" : "+v"(vb));  // opaque: word k stays "vb + k * 256" (instruction offset)
    ColIO c;
    c.r = r;
    c.vb = vb;
    return c;
  };
  // a lane's 1026-bit chunk spans words [32q, 32q + 34); the element's top lane must read
  // 0 past word L-1 (the descriptor spans the whole vector, so the range check no longer
  // does that: the next words belong to the next tile)
  const bool top = g.q == TPI - 1;
  auto ld = [&](const ColIO& c, int k) -> u32 {
    const u32 v = c.ld(k);
    return (k >= 32 && top) ? 0u : v;
  };
  const u32 nwt = (u32)((count + E - 1) / E);
  for (u32 wt = gw; wt < nwt; wt += nw) {
    const size_t slot = (size_t)wt * E + g.e;
    const bool live = slot < count;
    const size_t elem = !live ? 0 : (ord ? (size_t)(u32)ord[slot] : slot);
    const size_t be = bstride ? elem : 0;
    const u32 vo = live ? voff(elem) : vbytes;
    const ColIO Ai = io(ra, vo), Oo = io(ro, vo);
    const ColIO Bi = io(rb, live ? voff(be) : (bstride ? vbytes : L32 * 256u));
    const int xa = ea[elem], xb = eb[be];
    const u32 sav = sa[elem], sbv = sb[be];
    const bool x_is_a = xa > xb;
    L27 A, Bv;
    load_chunk(A, 2u * g.q, [&](int k) { return ld(Ai, k); });
    load_chunk(Bv, 2u * g.q, [&](int k) { return ld(Bi, k); });
    // literal-1 tests (:303-308) over the element's lanes
    u32 za = 0, zb = 0;
#pragma unroll
    for (int j = 0; j < LL; ++j) {
      const u32 one = (j == 0 && g.q == 0) ? 1u : 0u;
      za |= A[j] ^ one;
      zb |= Bv[j] ^ one;
    }
    za = elem_or<TPI>(za);
    zb = elem_or<TPI>(zb);
    const bool lit_a = za == 0 && sav == 0;
    const bool lit_b = zb == 0 && sbv == 0;
    const bool lit = lit_a || lit_b;
    int d = x_is_a ? xa - xb : xb - xa;
    if (lit || !live) d = 0;
    // x = higher-exp operand (stays in A); y is re-read at the end rather than held in
    // registers across the squarings
#pragma unroll
    for (int j = 0; j < LL; ++j) A.set(j, x_is_a ? A[j] : Bv[j]);
    const_to_slot<TPI>(bcol, qoff, K.N2R2_27, g.q);
    mont_mul<TPI>(A, bcol, N, np, g.q);  // x R
    // the squaring count is wave-uniform (an SGPR): the loop's control flow is scalar and
    // only the per-element `k < 4d` test masks lanes
    const int nsq = __builtin_amdgcn_readfirstlane(wave_max_int(4 * d));
#pragma unroll 1
    for (int k = 0; k < nsq; ++k) {
      if (k < 4 * d) sqr<TPI>(A, bcol, qoff, N, np, g.q);
    }
    // y: both operands' words are read and selected per lane -- wave-uniform descriptors
    // only (a per-lane descriptor becomes a readfirstlane loop around every load, which
    // the register allocator broke at 3 waves/SIMD: DESIGN.md §3)
    load_chunk(Bv, 2u * g.q, [&](int k) {
      const u32 wa = ld(Ai, k), wb = ld(Bi, k);
      return x_is_a ? wb : wa;
    });
    to_slot<TPI>(bcol, qoff, Bv);
    mont_mul<TPI>(A, bcol, N, np, g.q);  // x^(16^d) y mod n^2 (< 2N)
    finalize<TPI>(A, N, g.q);
    const u32 sy = x_is_a ? sbv : sav;
    u32 sign = d == 0 ? (sav ^ sbv) : sy;
    int exo = xa < xb ? xa : xb;
    if (lit) {
      // copy the other operand through untouched (words, not limbs: no re-encoding)
      sign = lit_a ? sbv : sav;
      exo = lit_a ? xb : xa;
    }
    if (__builtin_amdgcn_readfirstlane((u32)__any(lit))) {  // wave-uniform branch
      store_chunk<TPI>(A, g.q, [&](int k, u32 v) {
        const u32 wa = Ai.ld(k), wb = Bi.ld(k);
        Oo.st(k, lit ? (lit_a ? wb : wa) : v);
      });
    } else {
      store_chunk<TPI>(A, g.q, [&](int k, u32 v) { Oo.st(k, v); });
    }
    if (g.q == 0 && live) {
      so[elem] = (u8)sign;
      eo[elem] = exo;
    }
  }
}

// ======================================================================================
// ct x pt (fixedpoint_paillier/src/lib.rs:334-349), 27-bit engine, per-element exponents.
// k_mul_prep classifies each plaintext significand as the reference does:
//   pt >= n - max_int ("big", an encoded negative int): c^-1 ^ (n - pt)
//   pt <= max_int, negative float significand:           c^-1 ^ |pt|  (GMP powm, negative exp)
//   pt <= max_int otherwise:                              c ^ pt
//   else: panic "invalid plaintext"
// and writes need-inverse flags, the exponent magnitude E [T][L1][64] and its bit length.
// ======================================================================================
template <int L>
__global__ __launch_bounds__(256) void k_mul_prep(KeyArgs K, const u32* __restrict__ P, u32 lp,
                                                  const u8* __restrict__ pneg, int pstride, size_t count,
                                                  u8* __restrict__ need, u32* __restrict__ Eout,
                                                  int32_t* __restrict__ ebits_out, int32_t* __restrict__ err) {
  constexpr int L1 = L / 2;
  u32 ef = 0;
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < count; e += (size_t)gridDim.x * blockDim.x) {
    const size_t pe = pstride ? e : 0;
    u32 M[L1];
    u32 any = 0, br_max = 0, br_nmm = 0;
#pragma unroll
    for (int j = 0; j < L1; ++j) {
      M[j] = (u32)j < lp ? P[tiled(pe, lp, (u32)j)] : 0u;
      any |= M[j];
      const u64 d1 = (u64)K.max_int[j] - M[j] - br_max;
      br_max = (u32)(d1 >> 63);
      const u64 d2 = (u64)M[j] - K.n_mm[j] - br_nmm;
      br_nmm = (u32)(d2 >> 63);
    }
    u32 hi = 0;
    for (u32 j = L1; j < lp; ++j) hi |= P[tiled(pe, lp, j)];
    // negative significand: always powm(c^-1, |sig|) (a negative sig is <= max_int)
    const bool isneg = (pneg[pe] != 0) && (any != 0);
    bool big = !isneg && (br_nmm == 0) && hi == 0;  // P >= n - max_int
    bool invalid = hi != 0 || (!isneg && !big && br_max != 0);
    if (big) {  // exponent n - P
      u32 br = 0;
      u32 D[L1];
#pragma unroll
      for (int j = 0; j < L1; ++j) {
        const u64 d = (u64)K.n[j] - M[j] - br;
        D[j] = (u32)d;
        br = (u32)(d >> 63);
      }
      if (br) {
        // P > n: GMP powm(c^-1, n - P) with a negative exponent inverts the base again,
        // i.e. c^(P - n): no inverse, exponent P - n
        big = false;
        br = 0;
#pragma unroll
        for (int j = 0; j < L1; ++j) {
          const u64 d = (u64)M[j] - K.n[j] - br;
          M[j] = (u32)d;
          br = (u32)(d >> 63);
        }
      } else {
#pragma unroll
        for (int j = 0; j < L1; ++j) M[j] = D[j];
      }
    }
    int eb = 0;
#pragma unroll
    for (int j = 0; j < L1; ++j) {
      if (invalid) M[j] = 0;
      if (M[j]) eb = 32 * j + 32 - __clz(M[j]);
      Eout[tiled(e, L1, (u32)j)] = M[j];
    }
    if (invalid) ef |= FPHE_EF_MUL_INVALID_PT;
    need[e] = (isneg || big) && !invalid ? 1 : 0;
    ebits_out[e] = eb;
  }
  set_err(err, ef);
}

// ======================================================================================
template <int L, int W>
__global__ __launch_bounds__(kBlock) FPHE_OCC_MISC void k_mul27(KeyArgs K, const u32* __restrict__ Ca, const u32* __restrict__ Cinv,
                                                  const u8* __restrict__ need, const int32_t* __restrict__ ea,
                                                  const u32* __restrict__ Ex, const int32_t* __restrict__ ebits_in,
                                                  const int32_t* __restrict__ pexp, int pstride, size_t count,
                                                  u32* __restrict__ Co, u8* __restrict__ so, int32_t* __restrict__ eo,
                                                  u32* __restrict__ scratch, u32 ldsw) {
  constexpr int TPI = L / 32;
  using G = Geo<TPI>;
  constexpr int E = G::E;
  constexpr u32 L32 = L, L1 = L / 2;
  extern __shared__ __attribute__((aligned(16))) u32 lds[];
  G g;
  const u32 wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const u32 gw = blockIdx.x * kWavesPerBlock + wib, nw = gridDim.x * kWavesPerBlock;
  u32* bcol = lds + wib * ldsw * E + g.e;
  const u32 qoff = lds_qoff<TPI>(g.q);
  const Tile tb = make_tile(scratch + (size_t)gw * ((size_t)(1 << W) * LL * FPHE_WAVE), (1u << W) * LL * 256u, g.lane);
  Mod<TPI> N;
  N.init(K.N2_27, g.q);
  const u32 np = K.n2_np27;
  const u32 nwt = (u32)((count + E - 1) / E);
  for (u32 wt = gw; wt < nwt; wt += nw) {
    const size_t ebase = (size_t)wt * E;
    const u32 tile = (u32)(ebase >> 6);
    const u32 col = (u32)(ebase & 63) + (u32)g.e;
    const size_t elem = ebase + g.e;
    const bool inside = elem < count;
    const size_t pe = pstride ? elem : 0;
    const bool nd = inside && need[elem] != 0;
    const __amdgpu_buffer_rsrc_t Er = rsrc(Ex + (size_t)tile * L1 * FPHE_WAVE, L1 * 256u);
    const ColIO Ai = colio(Ca + (size_t)tile * L32 * FPHE_WAVE, L32, col, 32u * g.q);
    const ColIO Ii = colio(Cinv + (size_t)tile * L32 * FPHE_WAVE, L32, col, 32u * g.q);
    const ColIO Oo = colio(Co + (size_t)tile * L32 * FPHE_WAVE, L32, col, 32u * g.q);
    const int ebits = inside ? ebits_in[elem] : 0;
#if FPHE_UNIFORM_LOOPS
    const int maxbits = __builtin_amdgcn_readfirstlane(wave_max_int(ebits));  // SGPR: scalar loop control
#else
    const int maxbits = wave_max_int(ebits);
#endif
    L27 A;
#if FPHE_SELECT_LOADS
    load_chunk(A, 2u * g.q, [&](int k) {  // both loads, per-lane select: wave-uniform descriptors
      const u32 wi = Ii.ld(k), wa = Ai.ld(k);
      return nd ? wi : wa;
    });
#else
    load_chunk(A, 2u * g.q, [&](int k) { return nd ? Ii.ld(k) : Ai.ld(k); });
#endif
    const_to_slot<TPI>(bcol, qoff, K.N2R2_27, g.q);
    mont_mul<TPI>(A, bcol, N, np, g.q);  // X = base R
    if (maxbits > 0) {
      to_slot<TPI>(bcol, qoff, A);
      tab_store(tb, 1, A);
      {
        L27 one;
#pragma unroll
        for (int j = 0; j < LL; ++j) one.set(j, K.N2R1_27[g.q * LL + j]);
        tab_store(tb, 0, one);  // Montgomery 1
      }
#pragma unroll 1
      for (int k = 2; k < (1 << W); ++k) {
        mont_mul<TPI>(A, bcol, N, np, g.q);
        tab_store(tb, (u32)k, A);
      }
      const int nwin = (maxbits + W - 1) / W;
      auto digit = [&](int wi) -> u32 {
        const int b0 = wi * W;
        const u32 limb = (u32)(b0 >> 5);
        const int off = b0 & 31;
        u32 v = tld(Er, col, limb) >> off;
        if (off + W > 32 && limb + 1 < L1) v |= tld(Er, col, limb + 1) << (32 - off);
        return ebits == 0 ? 0u : (v & ((1u << W) - 1));
      };
      auto entry_tile = [&](u32 dgt) {  // per-element entry through the lane-varying voffset
        Tile t = tb;
        t.vo = tb.vo + dgt * LL * 256u;
        return t;
      };
      tab_load(A, entry_tile(digit(nwin - 1)), 0);
#pragma unroll 1
      for (int wi = nwin - 2; wi >= 0; --wi) {
#pragma unroll 1
        for (int s = 0; s < W; ++s) sqr<TPI>(A, bcol, qoff, N, np, g.q);
        tab_to_slot<TPI>(bcol, qoff, entry_tile(digit(wi)), 0);
        mont_mul<TPI>(A, bcol, N, np, g.q);
      }
    } else {
#pragma unroll
      for (int j = 0; j < LL; ++j) A.set(j, K.N2R1_27[g.q * LL + j]);
    }
    one_to_slot<TPI>(bcol, qoff, g.q);
    mont_mul<TPI>(A, bcol, N, np, g.q);  // leave Montgomery form (<= N)
    finalize<TPI>(A, N, g.q);
    store_chunk<TPI>(A, g.q, [&](int k, u32 v) { Oo.st(k, v); });
    if (g.q == 0 && inside) {
      so[elem] = 0;
      eo[elem] = ea[elem] + pexp[pe];
    }
  }
}

// ======================================================================================
// Segmented product fold: the ciphertext-add fold of same-exponent terms, one chunk of up
// to kFoldMax consecutive terms of a sorted index list per element, in one pass.
// For terms with equal exponents Ciphertext::add (fixedpoint_paillier/src/lib.rs:301-333)
// is the product mod n^2 with the signs XOR-ed (no alignment), and the literal-1 rule is
// the identity of that product, so a chunk is folded as
//   acc = t_0; acc = mont(acc, t_j) for j >= 1  (= prod t . R^-(len-1)); acc = mont(acc, R^len)
// -- one Montgomery product per term, terms read straight from the source vector by index
// (element-major source, no gather copies).  The callers (iupdate, intervals_sum, matmul folds) group terms by
// (segment, exponent) so every chunk is single-exponent; the few per-exponent partials of a
// segment are then merged with the aligning ct-add (k_add27).  Bit-exact by the order
// independence of the fold.
// ======================================================================================
constexpr int kFoldMax = 64;

template <int L>
__global__ __launch_bounds__(kBlock) FPHE_OCC_FOLD void k_fold27(KeyArgs K, const u32* __restrict__ Src,
                                                             const u8* __restrict__ ssign,
                                                             const int32_t* __restrict__ sexp,
                                                             const int64_t* __restrict__ ord,
                                                             const int64_t* __restrict__ cstart,
                                                             const int32_t* __restrict__ clen, size_t nchunks,
                                                             const u32* __restrict__ FR, u32* __restrict__ Co,
                                                             u8* __restrict__ so, int32_t* __restrict__ eo, u32 ldsw) {
  constexpr int TPI = L / 32;
  using G = Geo<TPI>;
  constexpr int E = G::E, NL = G::NL;
  constexpr u32 L32 = L;
  extern __shared__ __attribute__((aligned(16))) u32 lds[];
  G g;
  const u32 wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const u32 gw = blockIdx.x * kWavesPerBlock + wib, nw = gridDim.x * kWavesPerBlock;
  u32* bcol = lds + wib * ldsw * E + g.e;
  const u32 qoff = lds_qoff<TPI>(g.q);
  Mod<TPI> N;
  N.init(K.N2_27, g.q);
  const u32 np = K.n2_np27;
  // the 34 words of this lane's 1026-bit chunk of source element `idx` (0 past the number)
  // Src is element-major ([element][L] words): a lane's chunk is 136 contiguous bytes, so a
  // gathered term costs its own 512 B of lines instead of a 64-B line per 4-B word
  auto fetch = [&](int64_t idx, u32 (&W)[34]) {
    const uint4* b4 = reinterpret_cast<const uint4*>(Src + (size_t)idx * L32 + 32u * g.q);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint4 v = b4[k];
      W[4 * k] = v.x; W[4 * k + 1] = v.y; W[4 * k + 2] = v.z; W[4 * k + 3] = v.w;
    }
    const bool top = 32 * g.q + 32 >= (int)L32;  // the element's last lane: nothing past word L-1
    const uint2 t = top ? make_uint2(0u, 0u) : *reinterpret_cast<const uint2*>(Src + (size_t)idx * L32 + 32u * g.q + 32u);
    W[32] = t.x;
    W[33] = t.y;
  };
  const u32 nwt = (u32)((nchunks + E - 1) / E);
  for (u32 wt = gw; wt < nwt; wt += nw) {
    const size_t ebase = (size_t)wt * E;
    const u32 tile = (u32)(ebase >> 6);
    const u32 col = (u32)(ebase & 63) + (u32)g.e;
    const size_t ch = ebase + g.e;
    const bool inside = ch < nchunks;
    const int64_t st = inside ? cstart[ch] : 0;
    const int len = inside ? clen[ch] : 0;
#if FPHE_UNIFORM_LOOPS
    const int maxlen = __builtin_amdgcn_readfirstlane(wave_max_int(len));
#else
    const int maxlen = wave_max_int(len);
#endif
    L27 A, B;
    u32 W[34];
    u32 sg = 0;
    int ex = 0;
    if (inside) {
      const int64_t i0 = ord[st];
      fetch(i0, W);
      sg = ssign[i0];
      ex = sexp[i0];
    } else {
#pragma unroll
      for (int k = 0; k < 34; ++k) W[k] = 0;
    }
    load_chunk(A, 2u * g.q, [&](int k) { return W[k]; });
    // software pipeline: term j's words and sign are fetched during product j-1, and its
    // index (ord) during product j-2, so no load latency sits in front of a product
    u32 snext = 0;
    if (len > 1) {
      const int64_t i1 = ord[st + 1];
      fetch(i1, W);
      snext = ssign[i1];
    }
    int64_t inext2 = len > 2 ? ord[st + 2] : 0;
#pragma unroll 1
    for (int j = 1; j < maxlen; ++j) {
      if (j < len) {
        load_chunk(B, 2u * g.q, [&](int k) { return W[k]; });
        sg ^= snext;
        to_slot<TPI>(bcol, qoff, B);
        if (j + 1 < len) {
          fetch(inext2, W);
          snext = ssign[inext2];
        }
        inext2 = j + 2 < len ? ord[st + j + 2] : 0;
        mont_mul<TPI>(A, bcol, N, np, g.q);
      }
    }
    // undo the R^-(len-1): one product with R^len mod n^2 (FR row len)
    {
      const u32* f = FR + (size_t)(len > 0 ? len : 1) * NL + g.q * LL;
#pragma unroll
      for (int j = 0; j < LL; ++j) bcol[qoff + j * E] = f[j];
    }
    mont_mul<TPI>(A, bcol, N, np, g.q);
    finalize<TPI>(A, N, g.q);
    const ColIO Oo = colio(Co + (size_t)tile * L32 * FPHE_WAVE, L32, col, 32u * g.q);
    store_chunk<TPI>(A, g.q, [&](int k, u32 v) { Oo.st(k, v); });
    if (g.q == 0 && inside) {
      so[ch] = (u8)sg;
      eo[ch] = ex;
    }
  }
}

// ======================================================================================
// Co = Ca^(2^nsq) * Cb mod n^2, sign = sign(b): one step of pack_squeeze
// (fixedpoint_paillier/src/lib.rs:439-450: result.pow_mod_mut(2^shift) then
// result * y % ns; the powm result is canonical, so the product's sign is y's).
// ======================================================================================
template <int L>
__global__ __launch_bounds__(kBlock) FPHE_OCC_MISC void k_sqmul27(KeyArgs K, const u32* __restrict__ Ca, const u32* __restrict__ Cb,
                                                    const u8* __restrict__ sb, int nsq, size_t count,
                                                    u32* __restrict__ Co, u8* __restrict__ so, u32 ldsw) {
  constexpr int TPI = L / 32;
  using G = Geo<TPI>;
  constexpr int E = G::E;
  constexpr u32 L32 = L;
  extern __shared__ __attribute__((aligned(16))) u32 lds[];
  G g;
  const u32 wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const u32 gw = blockIdx.x * kWavesPerBlock + wib, nw = gridDim.x * kWavesPerBlock;
  u32* bcol = lds + wib * ldsw * E + g.e;
  const u32 qoff = lds_qoff<TPI>(g.q);
  Mod<TPI> N;
  N.init(K.N2_27, g.q);
  const u32 np = K.n2_np27;
  const u32 nwt = (u32)((count + E - 1) / E);
  for (u32 wt = gw; wt < nwt; wt += nw) {
    const size_t ebase = (size_t)wt * E;
    const u32 tile = (u32)(ebase >> 6);
    const u32 col = (u32)(ebase & 63) + (u32)g.e;
    const size_t elem = ebase + g.e;
    const ColIO Ai = colio(Ca + (size_t)tile * L32 * FPHE_WAVE, L32, col, 32u * g.q);
    const ColIO Bi = colio(Cb + (size_t)tile * L32 * FPHE_WAVE, L32, col, 32u * g.q);
    const ColIO Oo = colio(Co + (size_t)tile * L32 * FPHE_WAVE, L32, col, 32u * g.q);
    L27 A, B;
    load_chunk(A, 2u * g.q, [&](int k) { return Ai.ld(k); });
    const_to_slot<TPI>(bcol, qoff, K.N2R2_27, g.q);
    mont_mul<TPI>(A, bcol, N, np, g.q);  // a R
#pragma unroll 1
    for (int k = 0; k < nsq; ++k) sqr<TPI>(A, bcol, qoff, N, np, g.q);
    load_chunk(B, 2u * g.q, [&](int k) { return Bi.ld(k); });
    to_slot<TPI>(bcol, qoff, B);
    mont_mul<TPI>(A, bcol, N, np, g.q);  // a^(2^nsq) b  (< 2N)
    finalize<TPI>(A, N, g.q);
    store_chunk<TPI>(A, g.q, [&](int k, u32 v) { Oo.st(k, v); });
    if (g.q == 0 && elem < count) so[elem] = sb[elem];
  }
}

// ======================================================================================
// modular inverse of ciphertexts (GMP mpz_invert in math/src/rug/mod.rs:30-35; used by
// neg/sub/rsub, fixedpoint_paillier/src/lib.rs:259-285, and the invert branches of mul,
// :334-349).  Step 1: x0 = c^-1 mod n (safegcd, inv27.h) into X0 [tile][L1][64];
// step 2 (k_inv_lift27): c^-1 mod n^2 = x0 (2 - c x0).  need[e] == 0 skips an element
// (a wave with no such element skips the tile); need == nullptr means every element.
// ======================================================================================
template <int L>
__global__ __launch_bounds__(kBlock) void k_inv_n27(KeyArgs K, const u32* __restrict__ C, size_t count,
                                                    const u8* __restrict__ need, u32* __restrict__ X0,
                                                    int32_t* __restrict__ err, u32 ldsw) {
  constexpr int TPI = L / 64;  // n: 76 limbs for 2048-bit keys, 38 for 1024-bit
  using G = Geo<TPI>;
  constexpr int E = G::E, NL = G::NL;
  constexpr u32 L32 = L, L1 = L / 2;
  constexpr int kBatches = (49 * (L1 * 32) + 80) / 17 / LB + 2;  // Bernstein-Yang bound / 27, + margin
  extern __shared__ __attribute__((aligned(16))) u32 lds[];
  G g;
  const u32 wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const u32 gw = blockIdx.x * kWavesPerBlock + wib, nw = gridDim.x * kWavesPerBlock;
  u32* bcol = lds + wib * ldsw * E + g.e;
  const u32 qoff = lds_qoff<TPI>(g.q);
  Mod<TPI> N;
  N.init(K.Nn_27, g.q);
  const u32 np = K.nn_np27;
  const u32 nwt = (u32)((count + E - 1) / E);
  for (u32 wt = gw; wt < nwt; wt += nw) {
    const size_t ebase = (size_t)wt * E;
    const u32 tile = (u32)(ebase >> 6);
    const u32 col = (u32)(ebase & 63) + (u32)g.e;
    const size_t elem = ebase + g.e;
    const bool nd = elem < count && (need == nullptr || need[elem] != 0);
    if (!__any(nd)) continue;
    const u32* ctile = C + (size_t)tile * L32 * FPHE_WAVE;
    // x = c mod n: c = c_lo + R c_hi, R = 2^(27 NL); mont(c_lo, R mod n) + mont(c_hi, R^2 mod n)
    L27 A, B;
    {
      const u32 bit0 = 27u * NL + 1026u * g.q;
      const ColIO Ci = colio(ctile, L32, col, bit0 >> 5);
      load_chunk(B, bit0 & 31u, [&](int k) { return Ci.ld(k); });
    }
    const_to_slot<TPI>(bcol, qoff, K.NnR2_27, g.q);
    mont_mul<TPI>(B, bcol, N, np, g.q);
    {
      const ColIO Ci = colio(ctile, L32, col, 32u * g.q);
      load_chunk(A, 2u * g.q, [&](int k) { return Ci.ld(k); });
    }
    const_to_slot<TPI>(bcol, qoff, K.NnR1_27, g.q);
    mont_mul<TPI>(A, bcol, N, np, g.q);
#pragma unroll
    for (int j = 0; j < LL; ++j) A.set(j, A[j] + B[j]);
    normalize_exact<TPI>(A, g.q);  // < 4n
    finalize<TPI>(A, N, g.q);
    finalize<TPI>(A, N, g.q);
    finalize<TPI>(A, N, g.q);      // canonical c mod n
    const bool ok = inv_mod<TPI>(A, N, K.nn_inv27, kBatches, g.q);
    const ColIO Xo = colio(X0 + (size_t)tile * L1 * FPHE_WAVE, L1, col, 32u * g.q);
    store_chunk<TPI>(A, g.q, [&](int k, u32 v) { Xo.st(k, v); });
    if (g.q == 0 && nd && !ok) set_err(err, FPHE_EF_NOT_INVERTIBLE);
  }
}

template <int L>
__global__ __launch_bounds__(kBlock) FPHE_OCC2 void k_inv_lift27(KeyArgs K, const u32* __restrict__ C, size_t count,
                                                       const u8* __restrict__ need, const u32* __restrict__ X0,
                                                       u32* __restrict__ Co, u32 ldsw) {
  constexpr int TPI = L / 32;
  using G = Geo<TPI>;
  constexpr int E = G::E;
  constexpr u32 L32 = L, L1 = L / 2;
  extern __shared__ __attribute__((aligned(16))) u32 lds[];
  G g;
  const u32 wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const u32 gw = blockIdx.x * kWavesPerBlock + wib, nw = gridDim.x * kWavesPerBlock;
  u32* bcol = lds + wib * ldsw * E + g.e;
  const u32 qoff = lds_qoff<TPI>(g.q);
  Mod<TPI> N;
  N.init(K.N2_27, g.q);
  const u32 np = K.n2_np27;
  const u32 nwt = (u32)((count + E - 1) / E);
  for (u32 wt = gw; wt < nwt; wt += nw) {
    const size_t ebase = (size_t)wt * E;
    const u32 tile = (u32)(ebase >> 6);
    const u32 col = (u32)(ebase & 63) + (u32)g.e;
    const size_t elem = ebase + g.e;
    const bool nd = elem < count && (need == nullptr || need[elem] != 0);
    if (!__any(nd)) continue;
    L27 A;
    {
      const ColIO Xi = colio(X0 + (size_t)tile * L1 * FPHE_WAVE, L1, col, 32u * g.q);
      load_chunk(A, 2u * g.q, [&](int k) { return Xi.ld(k); });
    }
    const_to_slot<TPI>(bcol, qoff, K.N2R2_27, g.q);
    mont_mul<TPI>(A, bcol, N, np, g.q);  // x0 R
    to_slot<TPI>(bcol, qoff, A);         // the slot keeps x0 R for the rest of the element
    {
      const ColIO Ci = colio(C + (size_t)tile * L32 * FPHE_WAVE, L32, col, 32u * g.q);
      load_chunk(A, 2u * g.q, [&](int k) { return Ci.ld(k); });
    }
    mont_mul<TPI>(A, bcol, N, np, g.q);  // c x0 (plain form: c R^0 x0 R / R)
    // s = 2 - c x0  as  (2 + 2N - t) with t < 2N: positive, < 4N
    from_signed<TPI>(A, [&](int j) {
      return (int64_t)((j == 0 && g.q == 0) ? 2 : 0) + 2 * (int64_t)N(j) - (int64_t)A[j];
    }, g.q);
    mont_mul<TPI>(A, bcol, N, np, g.q);  // x0 (2 - c x0) R / R = x  (< 2N)
    finalize<TPI>(A, N, g.q);
    const ColIO Oo = colio(Co + (size_t)tile * L32 * FPHE_WAVE, L32, col, 32u * g.q);
    store_chunk<TPI>(A, g.q, [&](int k, u32 v) {
      if (nd) Oo.st(k, v);
    });
  }
}


// ======================================================================================
// Batch inversion mod n^2 (Montgomery's trick) for neg / sub / rsub (fixedpoint_paillier/
// src/lib.rs:259-285, invert via math/src/rug/mod.rs:30-35).  A wave owns 4 memory tiles
// (256 elements); its element group e (TPI lanes) owns KB = 256/E of them, {tile 4w + i /
// (64/E), column e + E (i mod 64/E)}, so every tile address stays wave-uniform.
//   k_binv_pre27:  Pbar_i = prod_{k<=i} a_k R (Montgomery form) into the per-wave table,
//                  and the group's total prod a_k (plain, canonical) into Tot.
//   (the totals are inverted with k_inv_n27 + k_inv_lift27: one inverse per KB elements)
//   k_binv_post27: walking back, a_i^-1 = I_i P_{i-1} and I_{i-1} = I_i a_i, I_i = inverse
//                  of the prefix product.
// 6 Montgomery products per element plus 1/KB of an inverse, against one safegcd inverse
// and a 3-product lift per element.  Positions past `count` (and whole tiles past the
// vector), and elements with need[e] == 0 when a mask is given (the invert branches of
// ct x pt), act as 1 and are not written.  A non-invertible element makes its group's total non-invertible:
// k_inv_n27 raises FPHE_EF_NOT_INVERTIBLE (the reference panics on unwrap()).
// ======================================================================================
template <int TPI>
__device__ __forceinline__ void set_one(L27& A, int q) {
#pragma unroll
  for (int k = 0; k < LL / 2; ++k) A.p[k] = 0;
  if (q == 0) A.set(0, 1u);
}

template <int L>
__global__ __launch_bounds__(kBlock) FPHE_OCC2 void k_binv_pre27(KeyArgs K, const u32* __restrict__ C, size_t count,
                                                       const u8* __restrict__ need, u32* __restrict__ Tab,
                                                       u32* __restrict__ Tot, u32 ldsw) {
  constexpr int TPI = L / 32;
  using G = Geo<TPI>;
  constexpr int E = G::E, PER = FPHE_WAVE / E, KB = 4 * PER;
  constexpr u32 L32 = L;
  extern __shared__ __attribute__((aligned(16))) u32 lds[];
  G g;
  const u32 wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const u32 gw = blockIdx.x * kWavesPerBlock + wib, nw = gridDim.x * kWavesPerBlock;
  u32* bcol = lds + wib * ldsw * E + g.e;
  const u32 qoff = lds_qoff<TPI>(g.q);
  Mod<TPI> N;
  N.init(K.N2_27, g.q);
  const u32 np = K.n2_np27;
  const u32 ntiles = (u32)((count + FPHE_WAVE - 1) / FPHE_WAVE);
  const u32 nwt = (ntiles + 3) / 4;
  for (u32 wt = gw; wt < nwt; wt += nw) {
    const Tile tb = make_tile(Tab + (size_t)wt * KB * LL * FPHE_WAVE, KB * LL * 256u, g.lane);
    L27 P;
#pragma unroll 1
    for (int i = 0; i < KB; ++i) {
      const u32 tile = wt * 4 + (u32)(i / PER);
      const u32 col = (u32)g.e + (u32)(E * (i % PER));
      L27 A;
      if (tile < ntiles) {  // wave-uniform
        const ColIO Ci = colio(C + (size_t)tile * L32 * FPHE_WAVE, L32, col, 32u * g.q);
        load_chunk(A, 2u * g.q, [&](int k) { return Ci.ld(k); });
      }
      const size_t elem = (size_t)tile * FPHE_WAVE + col;
      const bool live = tile < ntiles && elem < count && (need == nullptr || need[elem] != 0);
      if (!live) set_one<TPI>(A, g.q);
      const_to_slot<TPI>(bcol, qoff, K.N2R2_27, g.q);
      mont_mul<TPI>(A, bcol, N, np, g.q);  // a R
      if (i == 0) {
        P = A;
      } else {
        to_slot<TPI>(bcol, qoff, A);
        mont_mul<TPI>(P, bcol, N, np, g.q);  // Pbar_i = Pbar_{i-1} a_i R / R
      }
      tab_store(tb, (u32)i, P);
    }
    one_to_slot<TPI>(bcol, qoff, g.q);
    mont_mul<TPI>(P, bcol, N, np, g.q);  // plain prod a_k, < 2N
    finalize<TPI>(P, N, g.q);
    const size_t te = (size_t)wt * E + g.e;
    const ColIO To = colio(Tot + (te >> 6) * L32 * FPHE_WAVE, L32, (u32)(te & 63), 32u * g.q);
    store_chunk<TPI>(P, g.q, [&](int k, u32 v) { To.st(k, v); });
  }
}

template <int L>
__global__ __launch_bounds__(kBlock) FPHE_OCC2 void k_binv_post27(KeyArgs K, const u32* __restrict__ C, size_t count,
                                                        const u8* __restrict__ need, const u32* __restrict__ Tab,
                                                        const u32* __restrict__ Inv, u32* __restrict__ Co, u32 ldsw) {
  constexpr int TPI = L / 32;
  using G = Geo<TPI>;
  constexpr int E = G::E, PER = FPHE_WAVE / E, KB = 4 * PER;
  constexpr u32 L32 = L;
  extern __shared__ __attribute__((aligned(16))) u32 lds[];
  G g;
  const u32 wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const u32 gw = blockIdx.x * kWavesPerBlock + wib, nw = gridDim.x * kWavesPerBlock;
  u32* bcol = lds + wib * ldsw * E + g.e;
  const u32 qoff = lds_qoff<TPI>(g.q);
  Mod<TPI> N;
  N.init(K.N2_27, g.q);
  const u32 np = K.n2_np27;
  const u32 ntiles = (u32)((count + FPHE_WAVE - 1) / FPHE_WAVE);
  const u32 nwt = (ntiles + 3) / 4;
  for (u32 wt = gw; wt < nwt; wt += nw) {
    const Tile tb = make_tile(Tab + (size_t)wt * KB * LL * FPHE_WAVE, KB * LL * 256u, g.lane);
    L27 I;  // I_i R: Montgomery form of the inverse of a_0 ... a_i
    {
      const size_t te = (size_t)wt * E + g.e;
      const ColIO Ii = colio(Inv + (te >> 6) * L32 * FPHE_WAVE, L32, (u32)(te & 63), 32u * g.q);
      load_chunk(I, 2u * g.q, [&](int k) { return Ii.ld(k); });
    }
    const_to_slot<TPI>(bcol, qoff, K.N2R2_27, g.q);
    mont_mul<TPI>(I, bcol, N, np, g.q);
#pragma unroll 1
    for (int i = KB - 1; i >= 0; --i) {
      const u32 tile = wt * 4 + (u32)(i / PER);
      const u32 col = (u32)g.e + (u32)(E * (i % PER));
      const size_t elem = (size_t)tile * FPHE_WAVE + col;
      const bool live = tile < ntiles && elem < count && (need == nullptr || need[elem] != 0);
      // a_i^-1 = I_i P_{i-1} (I_0 for the first element)
      L27 X = I;
      if (i > 0) {
        tab_to_slot<TPI>(bcol, qoff, tb, (u32)(i - 1));
        mont_mul<TPI>(X, bcol, N, np, g.q);  // (I P) R
      }
      one_to_slot<TPI>(bcol, qoff, g.q);
      mont_mul<TPI>(X, bcol, N, np, g.q);    // plain, < 2N
      finalize<TPI>(X, N, g.q);
      if (tile < ntiles) {  // wave-uniform; columns past count are padding of the last tile
        const ColIO Xo = colio(Co + (size_t)tile * L32 * FPHE_WAVE, L32, col, 32u * g.q);
        if (live) store_chunk<TPI>(X, g.q, [&](int k, u32 v) { Xo.st(k, v); });
      }
      if (i == 0) break;
      // I_{i-1} = I_i a_i
      L27 A;
      if (tile < ntiles) {
        const ColIO Ci = colio(C + (size_t)tile * L32 * FPHE_WAVE, L32, col, 32u * g.q);
        load_chunk(A, 2u * g.q, [&](int k) { return Ci.ld(k); });
      }
      if (!live) set_one<TPI>(A, g.q);
      const_to_slot<TPI>(bcol, qoff, K.N2R2_27, g.q);
      mont_mul<TPI>(A, bcol, N, np, g.q);  // a_i R
      to_slot<TPI>(bcol, qoff, A);
      mont_mul<TPI>(I, bcol, N, np, g.q);
    }
  }
}

}  // namespace
