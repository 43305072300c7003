// Modular inverse on the device, in the 27-bit TPI layout of mont27_dev.h.
//
// The reference inverts with GMP mpz_invert (math/src/rug/mod.rs:30-35) for neg/sub/rsub
// (fixedpoint_paillier/src/lib.rs:259-285) and for ct x pt with a negative or "big"
// plaintext (:334-349).  Here c^-1 mod n^2 is computed in two steps:
//   1. x0 = c^-1 mod n by safegcd (Bernstein & Yang, "Fast constant-time gcd computation
//      and modular inversion", 2019): divsteps in batches of 27, each batch a 2x2
//      transition matrix computed from the low bits of f, g and applied to the
//      multi-limb f, g (exact division by 2^27) and d, e (mod n, made divisible by adding
//      a multiple of n).  The d/e range bookkeeping (d, e in (-2n, n)) follows the
//      published modinv design of libsecp256k1.
//   2. Hensel/Newton lift to n^2: x = x0 (2 - c x0) mod n^2 (c x0 = 1 + t n  =>
//      c x = 1 - t^2 n^2).
// Signed numbers are NL = 38*TPI limbs of 27 bits, limbs [0, NL-1) in [0, 2^27) and the top
// limb signed; lane q of an element holds limbs [38q, 38q+38).
#pragma once
#include "mont27_dev.h"

namespace fphe {
namespace r27 {

struct Trans {
  int u, v, q, r;
};

// 27 divsteps on the low bits of f (odd) and g; zeta = -(delta + 1/2).  Returns the
// transition matrix scaled by 2^27: [f', g'] * 2^27 = T [f, g].
__device__ __forceinline__ Trans divsteps27(int& zeta, u32 f, u32 g) {
  u32 u = 1, v = 0, q = 0, r = 1;
#pragma unroll
  for (int i = 0; i < LB; ++i) {
    u32 c1 = (u32)(zeta >> 31);  // zeta < 0
    const u32 c2 = 0u - (g & 1u);  // g odd
    const u32 x = (f ^ c1) - c1, y = (u ^ c1) - c1, z = (v ^ c1) - c1;
    g += x & c2;
    q += y & c2;
    r += z & c2;
    c1 &= c2;
    zeta = (int)(((u32)zeta ^ c1) - 1u);
    f += g & c1;
    u += q & c1;
    v += r & c1;
    g >>= 1;
    u <<= 1;
    v <<= 1;
  }
  return Trans{(int)u, (int)v, (int)q, (int)r};
}

__device__ __forceinline__ int64_t mad_i64(int a, int b, int64_t c) {  // a*b + c, one instruction
  int64_t d;
  asm("v_mad_i64_i32 %0, vcc, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c) : "vcc");
  return d;
}

template <int TPI>
__device__ __forceinline__ int bcast0(int x) {  // value of the element's lane 0
  return (int)dpp_bcast<TPI>((u32)x);
}

template <int TPI>
__device__ __forceinline__ int top_sign(const int (&X)[LL]) {  // -1 if X < 0 (exact limbs), else 0
  int s = X[LL - 1] >> 31;
  if constexpr (TPI == 4) return (int)__builtin_amdgcn_update_dpp(0, s, 0xFF, 0xf, 0xf, false);
  else if constexpr (TPI == 2) return (int)__builtin_amdgcn_update_dpp(0, s, 0xF5, 0xf, 0xf, false);
  else return s;
}

// [X, Y] <- ([[a, b], [c, d]] [X, Y] + N [mx, my]) / 2^27, in place, one pass over the
// columns (each column's old limbs die as its new limbs are written, so no second copy of
// the numbers is ever live).  Exact limbs out; the global limb 0 of each sum is divisible
// by 2^27 by construction (divsteps matrix for f, g; mx, my for d, e).
template <int TPI, bool WITH_N>
__device__ __forceinline__ void pair_update(int (&X)[LL], int (&Y)[LL], int a, int b, int c, int d, int mx, int my,
                                            const Mod<TPI>& N, int q) {
  int64_t cx = 0, cy = 0;
#pragma unroll
  for (int j = 0; j < LL; ++j) {
    const int xj = X[j], yj = Y[j];
    int64_t s = mad_i64(a, xj, mad_i64(b, yj, cx));
    int64_t t = mad_i64(c, xj, mad_i64(d, yj, cy));
    if constexpr (WITH_N) {
      s = mad_i64(mx, (int)N(j), s);
      t = mad_i64(my, (int)N(j), t);
    }
    X[j] = (int)(s & (int64_t)MASK);
    cx = s >> LB;
    Y[j] = (int)(t & (int64_t)MASK);
    cy = t >> LB;
  }
  int64_t tx = cx, ty = cy;  // what the lane carries upward in total (the top lane keeps it)
#pragma unroll
  for (int rr = 1; rr < TPI; ++rr) {
    int64_t ix = (int64_t)dpp_from_prev64((u64)cx), iy = (int64_t)dpp_from_prev64((u64)cy);
    if (q == 0) ix = iy = 0;
#pragma unroll
    for (int j = 0; j < LL; ++j) {
      const int64_t s = (int64_t)X[j] + ix, t = (int64_t)Y[j] + iy;
      X[j] = (int)(s & (int64_t)MASK);
      ix = s >> LB;
      Y[j] = (int)(t & (int64_t)MASK);
      iy = t >> LB;
    }
    cx = ix;
    cy = iy;
    tx += ix;
    ty += iy;
  }
  int ux = (int)dpp_from_next((u32)X[0]), uy = (int)dpp_from_next((u32)Y[0]);
  if (q == TPI - 1) {
    ux = (int)tx;
    uy = (int)ty;
  }
#pragma unroll
  for (int j = 0; j < LL - 1; ++j) {
    X[j] = X[j + 1];
    Y[j] = Y[j + 1];
  }
  X[LL - 1] = ux;
  Y[LL - 1] = uy;
}

// f, g <- T [f, g] / 2^27
template <int TPI>
__device__ __forceinline__ void update_fg(int (&F)[LL], int (&G)[LL], const Trans& t, const Mod<TPI>& N, int q) {
  pair_update<TPI, false>(F, G, t.u, t.v, t.q, t.r, 0, 0, N, q);
}

// d, e <- (T [d, e] + N [md, me]) / 2^27, md/me chosen for divisibility and so that d, e
// stay in (-2N, N) given they start there.
template <int TPI>
__device__ __forceinline__ void update_de(int (&D)[LL], int (&Ee)[LL], const Trans& t, const Mod<TPI>& N,
                                          u32 ninv, int q) {
  const int sd = top_sign<TPI>(D), se = top_sign<TPI>(Ee);
  int md = (t.u & sd) + (t.v & se);
  int me = (t.q & sd) + (t.r & se);
  const int d0 = bcast0<TPI>(D[0]), e0 = bcast0<TPI>(Ee[0]);
  const int64_t cd = (int64_t)t.u * d0 + (int64_t)t.v * e0;
  const int64_t ce = (int64_t)t.q * d0 + (int64_t)t.r * e0;
  md -= (int)((ninv * (u32)cd + (u32)md) & MASK);
  me -= (int)((ninv * (u32)ce + (u32)me) & MASK);
  pair_update<TPI, true>(D, Ee, t.u, t.v, t.q, t.r, md, me, N, q);
}

// Exact non-negative limbs of sum_j v(j) 2^(27 j) (v signed, |v| < 2^62, total >= 0).
template <int TPI, class Val>
__device__ __forceinline__ void from_signed(L27& A, Val val, int q) {
  int64_t c = 0;
  u32 l[LL];
#pragma unroll
  for (int j = 0; j < LL; ++j) {
    const int64_t t = val(j) + c;
    l[j] = (u32)(t & (int64_t)MASK);
    c = t >> LB;
  }
#pragma unroll
  for (int rr = 1; rr < TPI; ++rr) {
    int64_t cin = (int64_t)dpp_from_prev64((u64)c);
    if (q == 0) cin = 0;
    int64_t cc = cin;
#pragma unroll
    for (int j = 0; j < LL; ++j) {
      const int64_t t = (int64_t)l[j] + cc;
      l[j] = (u32)(t & (int64_t)MASK);
      cc = t >> LB;
    }
    c = cc;
  }
#pragma unroll
  for (int j = 0; j < LL; ++j) A.set(j, l[j]);
}

// x^-1 mod N for x in [0, N) (exact limbs) by safegcd; N odd, < 2^(27 NL - 2).
// Returns x^-1 mod N canonical in A, and ok = (gcd == 1).  `batches` >= the divstep
// bound / 27 for the modulus size; the loop also stops once g == 0 on every lane.
template <int TPI>
__device__ __forceinline__ bool inv_mod(L27& A, const Mod<TPI>& N, u32 ninv, int batches, int q) {
  int F[LL], G[LL], D[LL], Ee[LL];
#pragma unroll
  for (int j = 0; j < LL; ++j) {
    F[j] = (int)N(j);
    G[j] = (int)A[j];
    D[j] = 0;
    Ee[j] = (j == 0 && q == 0) ? 1 : 0;
  }
  int zeta = -1;
#pragma unroll 1
  for (int b = 0; b < batches; ++b) {
    const u32 f0 = (u32)bcast0<TPI>(F[0]), g0 = (u32)bcast0<TPI>(G[0]);
    const Trans t = divsteps27(zeta, f0, g0);
    update_de<TPI>(D, Ee, t, N, ninv, q);
    update_fg<TPI>(F, G, t, N, q);
    u32 gz = 0;
#pragma unroll
    for (int j = 0; j < LL; ++j) gz |= (u32)G[j];
    gz = elem_or<TPI>(gz);
    if (__all(gz == 0)) break;
  }
  // f = +-gcd (exact limbs).  +1 is limb 0 = 1 and the rest 0; -1 is all limbs 2^27-1
  // below a top limb of -1.
  const int sf = top_sign<TPI>(F);
  u32 bad = 0;
#pragma unroll
  for (int j = 0; j < LL; ++j) {
    const bool top = (q == TPI - 1) && (j == LL - 1);
    const int want_pos = (j == 0 && q == 0) ? 1 : 0;
    const int want_neg = top ? -1 : (int)MASK;
    bad |= (u32)(sf ? (F[j] != want_neg) : (F[j] != want_pos));
  }
  bad = elem_or<TPI>(bad);
  // v = d (f > 0) or -d (f < 0) is in (-2N, 2N); A = v + 2N in (0, 4N), then reduce mod N
  from_signed<TPI>(A, [&](int j) { return (sf ? -(int64_t)D[j] : (int64_t)D[j]) + 2 * (int64_t)N(j); }, q);
  finalize<TPI>(A, N, q);  // < 4N -> < 3N
  finalize<TPI>(A, N, q);  // -> < 2N
  finalize<TPI>(A, N, q);  // -> [0, N)
  if (bad) {
#pragma unroll
    for (int j = 0; j < LL; ++j) A.set(j, 0u);
  }
  return bad == 0;
}

}  // namespace r27
}  // namespace fphe
