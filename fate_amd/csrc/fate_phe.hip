// libfatephe: MI355X-native Paillier PHE kernels + C ABI (include/fate_phe.h).
//
// Reference semantics: rust/fate_utils/crates/paillier/src/lib.rs (L0) and
// rust/fate_utils/crates/fixedpoint_paillier/src/lib.rs (L1); SURVEY.md Appendix A.
// The modexp kernels (kernels27.h) spread an element over TPI adjacent lanes (27-bit limbs at
// TPI 4, 28-bit below: mont27_dev.h);
// the codec, CRT-tail, permutation and wire kernels take one element per lane.  All run
// grid-stride loops over 64-element tiles; see DESIGN.md for layouts and rooflines.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <stdlib.h>
#include <stdio.h>
#include <vector>
#include <mutex>

#include "../../include/fate_phe.h"
#include "mont_dev.h"
#include "chacha_dev.h"
#include "host_bn.h"

using namespace fphe;

namespace {

constexpr int kBlock = 256;      // 4 waves per workgroup
constexpr int kWavesPerBlock = kBlock / FPHE_WAVE;
// Path selection per context (fphe_ctx_set_option, include/fate_phe.h): calls of at most
// this many elements run the one-element-per-wave latency kernels (wide_dev.h).  Decrypt: the
// throughput kernel takes ~25 ms for anything up to ~32k elements (its waves run alone at their
// per-row latency), the latency kernel 4.3 ms for up to ~300 and 10.9 ms for 2,048
// (profiles/r05/r05g_latency_leg.txt).  Public-key encrypt: the throughput kernel takes ~52 ms
// up to ~16k elements.  Key-holder encrypt with drawn (z_p, z_q): the z^s mod s^2 halves on
// k_pow_half_enc_wide (decrypt's chain shape).  The env variables set a new context's
// defaults (0 turns a latency path off); tests switch them per context to run the parity
// fixtures through both kernels of each op.
inline int64_t env_i64(const char* name, int64_t dflt) {
  const char* e = getenv(name);
  return e ? (int64_t)strtoll(e, nullptr, 10) : dflt;
}
constexpr int kWinSlide = 6;     // sliding window of the 27-bit engine's shared-exponent modexps
// the decrypt halves of <= 1024-bit keys (TPI 1, exponents p-1 / q-1 of <= 512 bits): a 5-bit
// window builds 16 fewer table entries than it adds window products (~101 general products
// against ~105 at 6 bits), and halves the per-lane table
#ifndef FPHE_WIN_DEC1
#define FPHE_WIN_DEC1 5
#endif
#ifndef FPHE_WIN_DEC2
#define FPHE_WIN_DEC2 6
#endif
template <int TPI>
constexpr int kWinDec = TPI == 1 ? FPHE_WIN_DEC1 : (TPI == 2 ? FPHE_WIN_DEC2 : kWinSlide);
constexpr int kWinMul = 4;       // window of the per-lane-exponent modexp (ct x pt): table capacity
#ifndef FPHE_MUL_ADAPT
#define FPHE_MUL_ADAPT 1  // ct x pt: 3-bit window for short exponents, all-zero windows skipped
#endif
constexpr int kMulShortBits = 64;
constexpr u32 kAddRegions = 8;          // k_add27: one run of wave tiles per XCD (blocks b, b + 8, ...)
constexpr u32 kAddCounterStride = 32;   // the runs' tile counters, 128 B apart  // waves whose longest exponent fits this take a 3-bit window

// Uniform key material, passed by value (lands in the kernarg segment -> SGPRs).
struct KeyArgs {
  const u32* N2;       // n^2                     [L2]
  const u32* N2_R2;    // R^2 mod n^2, R=2^(32 L2) [L2]
  const u32* N2_R1;    // R mod n^2 (Montgomery 1) [L2]
  const u32* n;        // n, padded               [L1+1]
  const u32* nm1;      // n-1                     [L1]
  const u32* max_int;  // floor(n/2)              [L1]
  const u32* n_mm;     // n - max_int             [L1]
  u32 n2_n0inv;
  int nbits;
  // private half (valid iff has_sk)
  const u32* P2; const u32* P2_R3; const u32* pm1; const u32* p; const u32* pinv2; const u32* hpR;
  const u32* Q2; const u32* Q2_R3; const u32* qm1; const u32* q; const u32* qinv2; const u32* hqR;
  const u32* pinvqR;   // p^{-1} mod q, times R_q mod q
  u32 p2_n0inv, p_n0inv, q2_n0inv, q_n0inv;
  int pm1_bits, qm1_bits;
  // reduced-radix engine (kernels27.h): LB-bit limbs (27 for n^2 of 2048-bit keys, 28 for
  // every other modulus), R = 2^(LB NL); the _27 suffix names the engine, not the radix
  const u32* N2_27; const u32* N2R1_27; const u32* N2R2_27;  // n^2, R mod n^2, R^2 mod n^2 [NL2]
  const u32* P2_27; const u32* P2R1_27; const u32* P2R2_27;  // p^2 ...                      [NLh]
  const u32* Q2_27; const u32* Q2R1_27; const u32* Q2R2_27;
  u32 n2_np27, p2_np27, q2_np27;                             // -N^{-1} mod 2^LB
  const u32* Nn_27; const u32* NnR1_27; const u32* NnR2_27;  // n, R mod n, R^2 mod n    [NLh]
  u32 nn_np27, nn_inv27;                                     // -n^{-1}, n^{-1} mod 2^LB
  // key-holder (CRT) encryption, valid iff has_sk: r^n mod s^2 = r^(n mod s(s-1)) mod s^2,
  // recombined as x_p Kp + x_q Kq mod n^2 (Kp = q^2 (q^-2 mod p^2), Kq = p^2 (p^-2 mod q^2))
  const u32* ep; const u32* eq;          // n mod p(p-1), n mod q(q-1)           [L1]
  int ep_bits, eq_bits;
  const u32* KpR_27; const u32* KqR_27;  // Kp R, Kq R mod n^2 (R = 2^(LB NL2))         [NL2]
  // Montgomery-resident ciphertexts: vectors hold M(c) = c R mod n^2 with the
  // n^2 engine's R.  R^3 mod n^2 takes a plain value x to x R^2 in one product (inverses,
  // the key-holder nude factor); R_s^2 R^-1 mod s^2 takes M(c) mod s^2 to c R_s (decrypt).
  const u32* N2R3_27;                    // R^3 mod n^2                                  [NL2]
  const u32* P2RX_27; const u32* Q2RX_27;  // R_s^2 R^-1 mod s^2, s = p, q                [NLh]
  const u32* N2M1;                       // M(1) = R mod n^2 in 32-bit words (literal 1)  [L2]
  // key-holder encryption in two steps (FPHE_KH_SPLIT): z_s = r^(e_s)
  // mod s with e_p = q mod (p-1), e_q = p mod (q-1), on the engine of s (TPIs = L2/128 lanes,
  // at least 1), then x_s = z_s^s mod s^2 on the s^2 engine
  const u32* Ps_27; const u32* PsR2_27; const u32* PsR3_27;  // p, R_s^2, R_s^3 mod p      [NLs]
  const u32* Qs_27; const u32* QsR2_27; const u32* QsR3_27;
  u32 ps_np27, qs_np27;
  const u32* e1p; const u32* e1q;        // q mod (p-1), p mod (q-1)                   [LQ]
  int e1p_bits, e1q_bits, p_bits, q_bits;
};

__device__ __forceinline__ void set_err(int32_t* err, u32 f) {
  if (f) atomicOr(err, (int32_t)f);
}

// word index of limb j of element e in a tile-major [ntiles][lp][64] vector
__device__ __forceinline__ size_t tiled(size_t e, u32 lp, u32 j) {
  return ((e >> 6) * lp + j) * FPHE_WAVE + (e & 63);
}

// Per-kernel geometry: one 64-element tile per wave per grid-stride step.
struct WaveCtx {
  int lane;
  u32 gw, nw;  // global wave id, waves in grid (both wave-uniform)
};

__device__ __forceinline__ WaveCtx wave_ctx() {
  WaveCtx w;
  w.lane = (int)(threadIdx.x & 63);
  const u32 wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  w.gw = blockIdx.x * kWavesPerBlock + wib;
  w.nw = gridDim.x * kWavesPerBlock;
  return w;
}

template <int L>
__device__ __forceinline__ u32* lds_slot(u32* lds, int lane) {
  const u32 wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  return lds + wib * L * FPHE_WAVE + lane;
}

// ======================================================================================
// encrypt: C = (1 + m*n mod n^2) * r^n mod n^2, sign = (m < 0)
//   crates/paillier/src/lib.rs:104-121; both branches of :106-113 reduce to 1 + m*n
//   mod n^2 (the invert branch computes inv(1 - (n-m)n) = 1 + m n), and the sign of
//   the truncating product at :116 is the sign of m (r^n > 0).
// ======================================================================================
// C_nude = 1 + m*n (m >= 0) or n^2 - |m| n + 1 (m < 0) into an LDS column with limb
// stride S (64 for one lane per element, 32 for two).
template <int L, int S = FPHE_WAVE>
__device__ __forceinline__ bool nude_to_slot(u32* slot, const KeyArgs& K, const Tile& Pt, u32 lp, bool negflag) {
  constexpr int L1 = L / 2;
#pragma unroll
  for (int j = 0; j < L; ++j) slot[j * S] = 0u;
  u32 any = 0;
#pragma unroll 1
  for (u32 k = 0; k < lp; ++k) {
    const u32 pk = Pt.ld(k * 256u);
    any |= pk;
    u64 acc = 0;
#pragma unroll
    for (int j = 0; j < L1; ++j) {
      u32* s = slot + (k + j) * S;
      acc = (u64)pk * K.n[j] + *s + (acc >> 32);
      *s = (u32)acc;
    }
    slot[(k + L1) * S] = (u32)(acc >> 32);
  }
  const bool mneg = negflag && (any != 0);
  if (mneg) {  // n^2 - |m| n
    u32 br = 0;
#pragma unroll
    for (int j = 0; j < L; ++j) {
      u32* s = slot + j * S;
      const u64 d = (u64)K.N2[j] - *s - br;
      *s = (u32)d;
      br = (u32)(d >> 63);
    }
  }
  u32 c = 1;  // + 1
#pragma unroll
  for (int j = 0; j < L; ++j) {
    u32* s = slot + j * S;
    const u64 t = (u64)*s + c;
    *s = (u32)t;
    c = (u32)(t >> 32);
  }
  return mneg;
}

// r uniform in [1, n-1] (L1 = limbs of n) from this element's ChaCha20 stream.
template <int L1>
__device__ __forceinline__ void draw_r(u32 (&A)[L1], const KeyArgs& K, const ChaChaKey& ck, u64 nonce, size_t e) {
  constexpr int NB = (L1 + 15) / 16;
  // keep bits(n) random bits: words past the top of n (keys narrower than the L1-word
  // geometry) are 0, the top word is masked
  auto wmask = [&](int j) -> u32 {
    const int b = K.nbits - 32 * j;
    return b >= 32 ? 0xffffffffu : (b <= 0 ? 0u : ((1u << b) - 1u));
  };
  bool done = false;
  u32 attempt = 0;
  while (__any(!done)) {
    if (!done) {
      u32 x[L1];
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        u32 blk[16];
        // element index: low 32 bits in the first nonce word, bits 32..47 in the top half
        // of the block counter (attempt * NB + b stays far below 2^16)
        chacha20_block(ck, (attempt * NB + b) | ((u32)(e >> 32) << 16), (u32)e, (u32)(nonce >> 32), (u32)nonce,
                       blk);
#pragma unroll
        for (int i = 0; i < 16; ++i)
          if (b * 16 + i < L1) x[b * 16 + i] = blk[i];
      }
#pragma unroll
      for (int j = 0; j < L1; ++j) x[j] &= wmask(j);
      // accept iff x < n - 1, then r = x + 1 in [1, n-1]  (random.rs:22-25)
      u32 br = 0;
#pragma unroll
      for (int j = 0; j < L1; ++j) {
        const u64 d = (u64)x[j] - K.nm1[j] - br;
        br = (u32)(d >> 63);
      }
      if (br) {
        u32 c = 1;
#pragma unroll
        for (int j = 0; j < L1; ++j) {
          const u64 t = (u64)x[j] + c;
          A[j] = (u32)t;
          c = (u32)(t >> 32);
        }
        done = true;
      }
    }
    ++attempt;
  }
}

// r for every element into a tile-major [ntiles][L1][64] buffer (ChaCha20 per element,
// rejection sampling into [1, n-1]); kept out of the modexp kernel so its registers do
// not count against the modexp's occupancy.
__global__ __launch_bounds__(256) void k_chacha_blocks(ChaChaKey ck, u32 counter, u32 n0, u32 n1, u32 n2,
                                                       size_t nblocks, u32* __restrict__ out) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nblocks; i += (size_t)gridDim.x * blockDim.x) {
    u32 blk[16];
    chacha20_block(ck, counter + (u32)i, n0, n1, n2, blk);
#pragma unroll
    for (int k = 0; k < 16; ++k) out[i * 16 + k] = blk[k];
  }
}

// element e of the launch draws the stream of element ebase + e of the call (a call split
// into spans draws exactly what one launch over all its elements would)
template <int L1>
__global__ __launch_bounds__(256) void k_draw_r(KeyArgs K, size_t count, ChaChaKey ck, u64 nonce, size_t ebase,
                                                 u32* __restrict__ R) {
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < count; e += (size_t)gridDim.x * blockDim.x) {
    u32 r[L1];
    draw_r<L1>(r, K, ck, nonce, ebase + e);
#pragma unroll
    for (int j = 0; j < L1; ++j) R[tiled(e, L1, j)] = r[j];
  }
}

// Key-holder obfuscation drawn in its CRT coordinates.  The split modexp (k_pow_small27, then
// k_pow_half27<., ., true>) turns r into z_p = r^(q mod (p-1)) mod p and z_q likewise, then
// raises z_s to s mod s^2.  For r uniform in Z_n^*, (r mod p, r mod q) is uniform in
// Z_p^* x Z_q^*, and x -> x^q is a bijection of Z_p^* when gcd(q, p - 1) = 1 (x -> x^p of Z_q^*
// likewise): so (z_p, z_q) is uniform in Z_p^* x Z_q^*, and drawing it directly gives r^n mod
// n^2 with the distribution of the reference's random_rn (paillier/src/lib.rs:94-98;
// random.rs:22-25, r in [1, n-1]: the r sharing a factor with n, probability < 2^-1000, aside)
// for the cost of the second step only.  Injected r (parity mode) keeps the two-step path.
// z_s uniform in [1, s-1] from element e's ChaCha20 stream of half h.  The call's nonce is
// used as is; the streams are told apart in the block counter: bit 31 set for (z_p, z_q), clear
// for draw_r, bit 30 = h.  The low 16 bits count blocks (attempt NB + b, far below 2^14 in
// practice: each attempt succeeds with probability > 1/2) and bits 16..29 carry e >> 32 (0:
// a call has fewer than 2^32 elements), so no two draws of one call share a ChaCha20 block.
constexpr u32 kDrawZTag = 1u << 31, kDrawHalfTag = 1u << 30;
template <int LQ>
__device__ __forceinline__ void draw_below(u32 (&A)[LQ], const u32* __restrict__ sm1, int sbits, const ChaChaKey& ck,
                                           u64 nonce, size_t e, u32 tag) {
  constexpr int NB = (LQ + 15) / 16;
  auto wmask = [&](int j) -> u32 {
    const int b = sbits - 32 * j;
    return b >= 32 ? 0xffffffffu : (b <= 0 ? 0u : ((1u << b) - 1u));
  };
  bool done = false;
  u32 attempt = 0;
  while (__any(!done)) {
    if (!done) {
      u32 x[LQ];
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        u32 blk[16];
        chacha20_block(ck, (attempt * NB + b) | ((u32)(e >> 32) << 16) | tag, (u32)e, (u32)(nonce >> 32),
                       (u32)nonce, blk);
#pragma unroll
        for (int i = 0; i < 16; ++i)
          if (b * 16 + i < LQ) x[b * 16 + i] = blk[i];
      }
#pragma unroll
      for (int j = 0; j < LQ; ++j) x[j] &= wmask(j);
      u32 br = 0;  // accept iff x < s - 1, then z = x + 1 in [1, s - 1]
#pragma unroll
      for (int j = 0; j < LQ; ++j) {
        const u64 d = (u64)x[j] - sm1[j] - br;
        br = (u32)(d >> 63);
      }
      if (br) {
        u32 c = 1;
#pragma unroll
        for (int j = 0; j < LQ; ++j) {
          const u64 t = (u64)x[j] + c;
          A[j] = (u32)t;
          c = (u32)(t >> 32);
        }
        done = true;
      }
    }
    ++attempt;
  }
}

template <int L>
__global__ __launch_bounds__(256) void k_draw_z(KeyArgs K, size_t count, ChaChaKey ck, u64 nonce, size_t ebase,
                                                 u32* __restrict__ Z) {
  constexpr int LQ = L / 4;
  constexpr u32 ZW = 32u * (L >= 128 ? L / 128 : 1);  // kZWords<L> (kernels27.h): z_s words per half
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < count; e += (size_t)gridDim.x * blockDim.x) {
#pragma unroll 1
    for (u32 h = 0; h < 2; ++h) {
      u32 z[LQ];
      draw_below<LQ>(z, h ? K.qm1 : K.pm1, h ? K.q_bits : K.p_bits, ck, nonce, ebase + e,
                     kDrawZTag | (h ? kDrawHalfTag : 0u));
#pragma unroll
      for (u32 j = 0; j < ZW; ++j) Z[tiled(e, 2 * ZW, h * ZW + j)] = j < (u32)LQ ? z[j] : 0u;
    }
  }
}

// ======================================================================================
// decrypt (CRT): crates/paillier/src/lib.rs:163-176
// ======================================================================================
// d_s = L_s(y) * h_s mod s from y = c^(s-1) mod s^2 (LH words): paillier/src/lib.rs:174-176
template <int L>
__device__ __forceinline__ void crt_tail(u32 (&dout)[L / 4], const u32 (&A)[L / 2], u32* slot,
                                         const u32* __restrict__ S, u32 s_n0inv, const u32* __restrict__ sinv2,
                                         const u32* __restrict__ hsR) {
  constexpr int LH = L / 2, LQ = L / 4;
  // L(y) = (y - 1) / s, exact for units: (y-1) * s^{-1} mod 2^(32 LQ)
  u32 nz = 0;
#pragma unroll
  for (int j = 0; j < LH; ++j) nz |= A[j];
  u32 y1[LQ];
  {
    u32 br = 1;
#pragma unroll
    for (int j = 0; j < LQ; ++j) {
      const u64 d = (u64)A[j] - br;
      y1[j] = (u32)d;
      br = (u32)(d >> 63);
    }
  }
  u32 Ls[LQ];
#pragma unroll
  for (int j = 0; j < LQ; ++j) Ls[j] = 0;
#pragma unroll
  for (int i = 0; i < LQ; ++i) {
    u64 acc = 0;
#pragma unroll
    for (int j = 0; i + j < LQ; ++j) {
      acc = (u64)y1[i] * sinv2[j] + Ls[i + j] + (acc >> 32);
      Ls[i + j] = (u32)acc;
    }
  }
  if (nz == 0) {  // y == 0: reference computes (0-1)/s = 0 (truncating)
#pragma unroll
    for (int j = 0; j < LQ; ++j) Ls[j] = 0;
  }
  slot_store_uniform<LQ>(slot, hsR);
  mont_mul<LQ>(Ls, slot, S, s_n0inv);  // L * h_s mod s
#pragma unroll
  for (int j = 0; j < LQ; ++j) dout[j] = Ls[j];
}

// m = dp + p * ((dq - dp) p^{-1} mod q): paillier/src/lib.rs:163-172
template <int L>
__device__ __forceinline__ void crt_combine(const u32 (&dp)[L / 4], const u32 (&dq)[L / 4], const KeyArgs& K,
                                            u32* slot, const Tile& Pt) {
  constexpr int LQ = L / 4;
  // u = (dq - dp) mod q ; u = u * p^{-1} mod q  (paillier/src/lib.rs:166, canonical form; the
  // reference's `if o < 0 { o += n }` at :168-170 lands on the same value)
  u32 u[LQ];
  u32 br = 0;
#pragma unroll
  for (int j = 0; j < LQ; ++j) {
    const u64 d = (u64)dq[j] - dp[j] - br;
    u[j] = (u32)d;
    br = (u32)(d >> 63);
  }
  if (br) {
    u32 c = 0;
#pragma unroll
    for (int j = 0; j < LQ; ++j) {
      const u64 t = (u64)u[j] + K.q[j] + c;
      u[j] = (u32)t;
      c = (u32)(t >> 32);
    }
  }
  slot_store_uniform<LQ>(slot, K.pinvqR);
  mont_mul<LQ>(u, slot, K.q, K.q_n0inv);
  // m = u * p + dp  (p uniform outer operand, shifting accumulator; limb i final after step i)
  u32 T[LQ + 1];
#pragma unroll
  for (int j = 0; j < LQ; ++j) T[j] = dp[j];
  T[LQ] = 0;
#pragma unroll 1
  for (int i = 0; i < LQ; ++i) {
    const u32 pi = K.p[i];
    u64 acc = 0;
#pragma unroll
    for (int j = 0; j < LQ; ++j) {
      acc = (u64)u[j] * pi + T[j] + (acc >> 32);
      T[j] = (u32)acc;
    }
    T[LQ] += (u32)(acc >> 32);
    Pt.st(T[0], (u32)i * 256u);
#pragma unroll
    for (int j = 0; j < LQ; ++j) T[j] = T[j + 1];
    T[LQ] = 0;
  }
#pragma unroll
  for (int j = 0; j < LQ; ++j) Pt.st(T[j], (u32)(LQ + j) * 256u);
}

// decrypt, CRT phase for the reduced-radix path: y_p, y_q (k_pow_half27<., ., false>) -> m.
template <int L>
__global__ __launch_bounds__(kBlock) void k_decrypt_crt(KeyArgs K, const u32* __restrict__ Y, u32 ntiles,
                                                        u32* __restrict__ Pout) {
  constexpr int LH = L / 2, LQ = L / 4;
  extern __shared__ __attribute__((aligned(16))) u32 lds[];
  const WaveCtx w = wave_ctx();
  u32* slot = lds_slot<LQ>(lds, w.lane);
  for (u32 tile = w.gw; tile < ntiles; tile += w.nw) {
    const Tile Yt = make_tile(Y + (size_t)tile * 2 * LH * FPHE_WAVE, 2 * LH * 256u, w.lane);
    const Tile Pt = make_tile(Pout + (size_t)tile * LH * FPHE_WAVE, LH * 256u, w.lane);
    u32 dp[LQ], dq[LQ];
    {
      u32 A[LH];
      tile_load<LH>(A, Yt, 0u);
      crt_tail<L>(dp, A, slot, K.p, K.p_n0inv, K.pinv2, K.hpR);
    }
    {
      u32 A[LH];
      tile_load<LH>(A, Yt, LH * 256u);
      crt_tail<L>(dq, A, slot, K.q, K.q_n0inv, K.qinv2, K.hqR);
    }
    crt_combine<L>(dp, dq, K, slot, Pt);
  }
}

// ======================================================================================
// fixed-point encode / decode (fixedpoint_paillier/src/lib.rs:148-192)
// ======================================================================================
__device__ __forceinline__ u32 encode_core(double x, u64& mag, bool& ng, int& ex) {
  const u64 b = (u64)__double_as_longlong(x);
  const int E = (int)((b >> 52) & 0x7ff);
  const u64 frac = b & ((1ull << 52) - 1);
  ng = (b >> 63) != 0;
  if (E == 0x7ff) { mag = 0; ex = 0; ng = false; return FPHE_EF_ENCODE_NONFINITE; }
  if (E == 0 && frac == 0) { mag = 0; ex = -14; ng = false; return 0; }  // frexp(0).1 = 0 -> exp=-14
  int e;       // frexp exponent: x = f * 2^e, f in [0.5, 1)
  int lsb;     // x = m * 2^lsb
  u64 m;
  if (E != 0) { m = frac | (1ull << 52); e = E - 1022; lsb = E - 1075; }
  else { const int bl = 64 - __clzll(frac); m = frac; e = bl - 1074; lsb = -1074; }
  ex = (e - 53) >> 2;         // floor((e-53)/4), arithmetic shift
  mag = m << (lsb - 4 * ex);  // exact: x * 16^-ex  (round() is exact here)
  return 0;
}

__global__ __launch_bounds__(256) void k_encode_f32(const float* __restrict__ x, size_t count, u32* __restrict__ P,
                                                    u8* __restrict__ neg, int32_t* __restrict__ exp,
                                                    int32_t* __restrict__ err) {
  u32 ef = 0;
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < count; e += (size_t)gridDim.x * blockDim.x) {
    u64 mag; bool ng; int ex;
    ef |= encode_core((double)x[e], mag, ng, ex);
    P[tiled(e, 2, 0)] = (u32)mag; P[tiled(e, 2, 1)] = (u32)(mag >> 32);
    neg[e] = ng ? 1 : 0; exp[e] = ex;
  }
  set_err(err, ef);
}

__global__ __launch_bounds__(256) void k_encode_f64(const double* __restrict__ x, size_t count, u32* __restrict__ P,
                                                    u8* __restrict__ neg, int32_t* __restrict__ exp,
                                                    int32_t* __restrict__ err) {
  u32 ef = 0;
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < count; e += (size_t)gridDim.x * blockDim.x) {
    u64 mag; bool ng; int ex;
    ef |= encode_core(x[e], mag, ng, ex);
    P[tiled(e, 2, 0)] = (u32)mag; P[tiled(e, 2, 1)] = (u32)(mag >> 32);
    neg[e] = ng ? 1 : 0; exp[e] = ex;
  }
  set_err(err, ef);
}

// decode_f64 (:169-186).  exp >= 0: (M << 4exp).to_f64() truncates (mpz_get_d);
// exp < 0: M * Float(53)^exp is rounded to 53 bits (RNE) by MPFR, then to_f64 (RNE, a
// second rounding only in the subnormal range).
template <int L1>
__device__ __forceinline__ double decode_core(const u32* __restrict__ P, u32 lp, size_t e, int ex,
                                              const KeyArgs& K, u32& ef) {
  u32 M[L1];
  u32 br_n = 0, br_max = 0, br_nmm = 0;
#pragma unroll
  for (int j = 0; j < L1; ++j) {
    M[j] = (u32)j < lp ? P[tiled(e, lp, j)] : 0u;
    const u64 d0 = (u64)K.n[j] - M[j] - br_n; br_n = (u32)(d0 >> 63);        // n - P
    const u64 d1 = (u64)K.max_int[j] - M[j] - br_max; br_max = (u32)(d1 >> 63);
    const u64 d2 = (u64)M[j] - K.n_mm[j] - br_nmm; br_nmm = (u32)(d2 >> 63);
  }
  // limbs beyond L1 must be zero (P < 2^(32 L1)) else corrupted
  u32 hi = 0;
  for (u32 j = L1; j < lp; ++j) hi |= P[tiled(e, lp, j)];
  if (br_n || hi) { ef |= FPHE_EF_DECODE_CORRUPTED; return 0.0; }
  bool ng = false;
  if (br_max == 0) {
    // M <= max_int: mantissa = M
  } else if (br_nmm == 0) {
    ng = true;  // mantissa = M - n (negative): magnitude n - M
    u32 br = 0;
#pragma unroll
    for (int j = 0; j < L1; ++j) {
      const u64 d = (u64)K.n[j] - M[j] - br;
      M[j] = (u32)d; br = (u32)(d >> 63);
    }
  } else {
    ef |= FPHE_EF_DECODE_OVERFLOW; return 0.0;
  }
  // locate the top limb
  int h = -1;
#pragma unroll
  for (int j = 0; j < L1; ++j) if (M[j]) h = j;
  if (h < 0) return 0.0;
  u32 w0 = 0, w1 = 0, w2 = 0, sticky = 0;
#pragma unroll
  for (int j = 0; j < L1; ++j) {
    if (j == h) w0 = M[j];
    if (j == h - 1) w1 = M[j];
    if (j == h - 2) w2 = M[j];
    if (j < h - 2) sticky |= M[j];
  }
  const int lz = __clz(w0);
  const u64 top = ((u64)w0 << 32) | w1;
  const u64 t64 = lz ? ((top << lz) | ((u64)w2 >> (32 - lz))) : top;
  const u32 rest = lz ? (w2 << lz) : w2;
  sticky |= rest;
  int E2 = 32 * h + 31 - lz + 4 * ex;  // exponent of the leading bit
  u64 mant = t64 >> 11;
  if (ex < 0) {
    const u32 low = (u32)(t64 & 0x7ff);
    if (low > 0x400u || (low == 0x400u && (sticky || (mant & 1)))) ++mant;
    if (mant >> 53) { mant >>= 1; ++E2; }
  }
  u64 bits;
  if (E2 > 1023) {
    bits = 0x7ff0000000000000ull;
  } else if (E2 >= -1022) {
    bits = ((u64)(E2 + 1023) << 52) | (mant & ((1ull << 52) - 1));
  } else {
    const int sh = -1022 - E2;
    u64 q = 0;
    if (sh <= 53) {
      q = mant >> sh;
      const u64 rem = mant & ((1ull << sh) - 1);
      const u64 half = 1ull << (sh - 1);
      if (rem > half || (rem == half && (q & 1))) ++q;
    }
    bits = q;
  }
  if (ng) bits |= 0x8000000000000000ull;
  return __longlong_as_double((long long)bits);
}

template <int L1>
__global__ __launch_bounds__(256) void k_decode_f32(KeyArgs K, const u32* __restrict__ P, u32 lp,
                                                    const int32_t* __restrict__ exp, size_t count,
                                                    float* __restrict__ out, int32_t* __restrict__ err) {
  u32 ef = 0;
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < count; e += (size_t)gridDim.x * blockDim.x)
    out[e] = __double2float_rn(decode_core<L1>(P, lp, e, exp[e], K, ef));
  set_err(err, ef);
}

template <int L1>
__global__ __launch_bounds__(256) void k_decode_f64(KeyArgs K, const u32* __restrict__ P, u32 lp,
                                                    const int32_t* __restrict__ exp, size_t count,
                                                    double* __restrict__ out, int32_t* __restrict__ err) {
  u32 ef = 0;
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < count; e += (size_t)gridDim.x * blockDim.x)
    out[e] = decode_core<L1>(P, lp, e, exp[e], K, ef);
  set_err(err, ef);
}

}  // namespace

#include "codec_dev.h"
#include "kernels27.h"
namespace {
#include "group_dev.h"
#include "wide_dev.h"
}  // namespace

// ======================================================================================
// host side: context + C ABI
// ======================================================================================
struct fphe_ctx {
  int device = 0;
  uint32_t key_bits = 0;
  int L2 = 0, L1 = 0, LQ = 0;
  bool has_sk = false;
  int cus = 0;
  u32* blob = nullptr;
  KeyArgs K{};
  u32* scratch = nullptr;
  size_t scratch_bytes = 0;
  // the stream that last used `scratch`: a call on another stream first waits for it, so
  // two streams never share the window tables / intermediates at the same time
  hipStream_t scratch_stream = nullptr;
  bool scratch_used = false;
  // a non-blocking side stream and its fork/join events (created on first use):
  // fphe_fold_segments copies the source to element-major rows there while the call's
  // stream reads back the exponent range and sorts the terms
  hipStream_t side = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  // the key holder may draw its obfuscation as (z_p, z_q) directly (k_draw_z): set when
  // gcd(q, p - 1) = gcd(p, q - 1) = 1, which makes r -> (z_p, z_q) a bijection
  bool kh_direct = false;
  // path options (fphe_ctx_set_option): latency-kernel thresholds, and whether the key holder
  // draws (z_p, z_q) (effective only when kh_direct)
  int64_t wide_decrypt_max = 4096, wide_encrypt_max = 2048, wide_kh_encrypt_max = 4096;
  bool kh_direct_z = true;
  std::mutex mu;
};

namespace {

using hbn::Limbs;

fphe_status hip_ok(hipError_t e) { return e == hipSuccess ? FPHE_OK : FPHE_ERR_HIP; }

struct DevGuard {
  int prev = 0;
  explicit DevGuard(int d) { (void)hipGetDevice(&prev); (void)hipSetDevice(d); }
  ~DevGuard() { (void)hipSetDevice(prev); }
};

// context-less entry points launch on the device of the caller's stream (a non-null stream;
// on the null stream, on the current device, which the caller sets)
struct StreamDevGuard {
  int prev = -1;
  explicit StreamDevGuard(void* stream) {
    hipDevice_t d;
    if (stream && hipStreamGetDevice((hipStream_t)stream, &d) == hipSuccess && hipGetDevice(&prev) == hipSuccess)
      (void)hipSetDevice(d);
    else
      prev = -1;
  }
  ~StreamDevGuard() { if (prev >= 0) (void)hipSetDevice(prev); }
};

Limbs from_words(const uint32_t* w, size_t n) { return hbn::norm(Limbs(w, w + n)); }

// little-endian 32-bit words -> nl limbs of lb bits (the engine radix of the modulus)
Limbs to_radix(const Limbs& v, int nl, int lb) {
  Limbs o((size_t)nl, 0u);
  for (int i = 0; i < nl; ++i) {
    const size_t bit = (size_t)lb * i, w = bit >> 5;
    const unsigned off = (unsigned)(bit & 31);
    u64 x = w < v.size() ? v[w] : 0u;
    if (w + 1 < v.size()) x |= (u64)v[w + 1] << 32;
    o[(size_t)i] = (u32)(x >> off) & ((1u << lb) - 1u);
  }
  return o;
}

template <typename KernT>
unsigned occ_grid(const fphe_ctx* c, KernT k, size_t lds, size_t waves, const char* what = "") {
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k, kBlock, lds) != hipSuccess || nb < 1) nb = 1;
  size_t g = (size_t)c->cus * (size_t)nb;
  const size_t need = (waves + kWavesPerBlock - 1) / kWavesPerBlock;
  if (need < g) g = need;
  if (getenv("FPHE_DEBUG"))
    fprintf(stderr, "[fphe] %s: occupancy api %d blocks/CU, lds %zu B/block, grid %zu blocks for %zu waves\n", what, nb,
            lds, g, waves);
  return (unsigned)(g ? g : 1);
}

// Grid: `bpc` workgroups per CU (from LDS/VGPR budget), capped by the work.
u32 ntiles_of(size_t count) { return (u32)((count + FPHE_WAVE - 1) / FPHE_WAVE); }

unsigned grid_for(const fphe_ctx* c, size_t count, int bpc) {
  const size_t groups = (count + kBlock - 1) / kBlock;  // 4 tiles per workgroup
  size_t g = (size_t)c->cus * bpc;
  if (groups < g) g = groups;
  return (unsigned)(g ? g : 1);
}

fphe_status ensure_scratch(fphe_ctx* c, size_t bytes, hipStream_t s) {
  if (c->scratch_used && c->scratch_stream != s && hipStreamSynchronize(c->scratch_stream) != hipSuccess)
    return FPHE_ERR_HIP;
  c->scratch_stream = s;
  c->scratch_used = true;
  if (c->scratch_bytes >= bytes) return FPHE_OK;
  if (c->scratch) { (void)hipFree(c->scratch); c->scratch = nullptr; c->scratch_bytes = 0; }
  if (hipMalloc(&c->scratch, bytes) != hipSuccess) return FPHE_ERR_HIP;
  c->scratch_bytes = bytes;
  return FPHE_OK;
}

// Long calls run as spans of whole grid rounds, at least kSpanTarget elements each (a
// 2048-bit encrypt of 2^21 elements is ~6 s): no single launch of a 100M-element call runs
// for minutes, the per-span scratch (drawn nonces, CRT halves) stays ~1 GB instead of
// growing with the call, and every span but the last fills its grid's last round exactly.
// FPHE_SPAN_TARGET overrides the target (tests force several spans on small calls).
constexpr size_t kSpanTarget = (size_t)1 << 21;
template <typename KernT>
size_t span_elems(const fphe_ctx* c, KernT k, size_t lds, int E) {
  const char* env = getenv("FPHE_SPAN_TARGET");
  const size_t target = env ? (size_t)strtoull(env, nullptr, 10) : kSpanTarget;
  const size_t cap = (size_t)occ_grid(c, k, lds, (size_t)1 << 40) * kWavesPerBlock * (size_t)E;  // one round
  const size_t rounds = target / cap > 0 ? target / cap : 1;
  return cap * rounds;  // a multiple of 64: spans start on tile boundaries
}

template <typename KernT>
void set_lds(KernT k, size_t bytes) {
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

// workgroups per CU for a kernel whose per-wave LDS slot is `slot_limbs` limbs
int bpc_for_slot(int slot_limbs) {
  const size_t per_block = (size_t)kWavesPerBlock * slot_limbs * FPHE_WAVE * 4;
  int b = (int)((160 * 1024) / per_block);
  return b < 1 ? 1 : (b > 2 ? 2 : b);
}

}  // namespace

namespace {
// ---- reduced-radix engine launchers (kernels27.h) ---------------------------------------
template <int L>
fphe_status launch_mont_const27(fphe_ctx* c, const uint32_t* C, size_t count, const u32* X, uint32_t* Co,
                                hipStream_t s) {
  constexpr int TPI = L / 32, E = FPHE_WAVE / TPI, NL = rad_ll(TPI) * TPI;
  auto kern = KS<TPI>::template mont_const<L>();
  const size_t lds = (size_t)kWavesPerBlock * NL * E * 4;
  set_lds(kern, lds);
  const unsigned grid = occ_grid(c, kern, lds, (count + E - 1) / E, "mont_const27");
  hipLaunchKernelGGL(kern, dim3(grid), dim3(kBlock), lds, s, c->K, C, count, X, Co, (u32)NL);
  return hip_ok(hipGetLastError());
}

template <int L>
fphe_status launch_encrypt27(fphe_ctx* c, const uint32_t* P, uint32_t lp, const uint8_t* neg, size_t count, int obf,
                             const uint32_t* r, const uint32_t key[8], uint64_t nonce, uint32_t* C, uint8_t* sign,
                             hipStream_t s) {
  constexpr int TPI = L / 32, E = FPHE_WAVE / TPI, NL = rad_ll(TPI) * TPI, LDSW = NL > L + 3 ? NL : L + 3, L1 = L / 2;
  auto kern = KS<TPI>::template encrypt<L, kWinSlide>();
  const size_t lds = (size_t)kWavesPerBlock * LDSW * E * 4;
  set_lds(kern, lds);
  const size_t span = span_elems(c, kern, lds, E);
  const size_t m0 = count < span ? count : span;
  const unsigned grid = occ_grid(c, kern, lds, (m0 + E - 1) / E, "encrypt27");
  const size_t tbytes = (size_t)grid * kWavesPerBlock * kTabEntries<kWinSlide> * rad_ll(TPI) * FPHE_WAVE * 4;
  const size_t rbytes = (size_t)ntiles_of(m0) * L1 * FPHE_WAVE * 4;
  const bool draw = obf && !r;
  ChaChaKey ck;
  if (draw)
    for (int i = 0; i < 8; ++i) ck.k[i] = key[i];
  if (obf && (int64_t)count <= c->wide_encrypt_max) {
    // few elements: one wave per element on the latency kernel (wide_dev.h), M-form written
    // directly; r drawn as on the throughput path (element e's stream), so the integers agree
    const size_t rb = (size_t)ntiles_of(count) * L1 * FPHE_WAVE * 4;
    if (draw && ensure_scratch(c, rb, s) != FPHE_OK) return FPHE_ERR_HIP;
    const u32* rbuf = r;
    if (draw) {
      const unsigned rgrid = (unsigned)std::min<size_t>((count + 255) / 256, (size_t)c->cus * 4);
      hipLaunchKernelGGL(k_draw_r<L1>, dim3(rgrid), dim3(256), 0, s, c->K, count, ck, nonce, (size_t)0, c->scratch);
      rbuf = c->scratch;
    }
    hipLaunchKernelGGL((k_encrypt_wide<L, kWinSlide>), dim3((unsigned)count), dim3(64), 0, s, c->K, P, lp, neg, count,
                       rbuf, C, sign);
    return hip_ok(hipGetLastError());
  }
  if (ensure_scratch(c, tbytes + (draw ? rbytes : 0), s) != FPHE_OK) return FPHE_ERR_HIP;
  for (size_t e0 = 0; e0 < count; e0 += span) {  // spans run in stream order over one scratch
    const size_t m = count - e0 < span ? count - e0 : span, t0 = e0 / FPHE_WAVE;
    const u32* rbuf = r ? r + t0 * L1 * FPHE_WAVE : nullptr;
    if (draw) {
      u32* rdev = c->scratch + tbytes / 4;
      const unsigned rgrid = (unsigned)std::min<size_t>((m + 255) / 256, (size_t)c->cus * 4);
      hipLaunchKernelGGL(k_draw_r<L1>, dim3(rgrid), dim3(256), 0, s, c->K, m, ck, nonce, e0, rdev);
      rbuf = rdev;
    }
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kBlock), lds, s, c->K, P + t0 * lp * FPHE_WAVE, lp, neg + e0, m, obf,
                       rbuf, C + t0 * L * FPHE_WAVE, sign + e0, c->scratch, (u32)LDSW);
    // into the Montgomery-resident form, in place (one product per element)
    if (launch_mont_const27<L>(c, C + t0 * L * FPHE_WAVE, m, c->K.N2R2_27, C + t0 * L * FPHE_WAVE, s) != FPHE_OK)
      return FPHE_ERR_HIP;
  }
  return FPHE_OK;
}

template <int L>
fphe_status launch_decrypt27(fphe_ctx* c, const uint32_t* C, size_t count, uint32_t* P, hipStream_t s) {
  constexpr int TPI = L / 64, E = FPHE_WAVE / TPI, NL = rad_ll(TPI) * TPI, LH = L / 2, LQ = L / 4;
  if ((int64_t)count <= c->wide_decrypt_max) {
    // few elements: one wave per (element, half) on the latency kernel (wide_dev.h), which
    // writes the same y_s rows k_pow_half27 does; the CRT tail is the same kernel
    const size_t ybytes = (size_t)ntiles_of(count) * 2 * LH * FPHE_WAVE * 4;
    if (ensure_scratch(c, ybytes, s) != FPHE_OK) return FPHE_ERR_HIP;
    u32* Y = c->scratch;
    hipLaunchKernelGGL((k_pow_half_wide<L, kWinDec<TPI>>), dim3((unsigned)(2 * count)), dim3(64), 0, s, c->K, C, count, Y);
    auto kcrt = k_decrypt_crt<L>;
    const size_t lds2 = (size_t)kWavesPerBlock * LQ * FPHE_WAVE * 4;
    set_lds(kcrt, lds2);
    hipLaunchKernelGGL(kcrt, dim3(grid_for(c, count, bpc_for_slot(LQ))), dim3(kBlock), lds2, s, c->K, Y,
                       ntiles_of(count), P);
    return hip_ok(hipGetLastError());
  }
  auto kern = KS<TPI>::template pow_half<L, kWinDec<TPI>, false>();
  const size_t lds = (size_t)kWavesPerBlock * NL * E * 4;
  set_lds(kern, lds);
  const size_t span = span_elems(c, kern, lds, E);
  const size_t m0 = count < span ? count : span;
  const unsigned grid = occ_grid(c, kern, lds, (m0 + E - 1) / E, "decrypt_pow27");
  const size_t tbytes = (size_t)grid * kWavesPerBlock * kTabEntries<kWinDec<TPI>> * rad_ll(TPI) * FPHE_WAVE * 4;
  const size_t ybytes = (size_t)ntiles_of(m0) * 2 * LH * FPHE_WAVE * 4;
  if (ensure_scratch(c, tbytes + ybytes, s) != FPHE_OK) return FPHE_ERR_HIP;
  u32* Y = c->scratch + tbytes / 4;
  auto kcrt = k_decrypt_crt<L>;
  const size_t lds2 = (size_t)kWavesPerBlock * LQ * FPHE_WAVE * 4;
  set_lds(kcrt, lds2);
  for (size_t e0 = 0; e0 < count; e0 += span) {
    const size_t m = count - e0 < span ? count - e0 : span, t0 = e0 / FPHE_WAVE;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kBlock), lds, s, c->K, C + t0 * L * FPHE_WAVE, m, Y, c->scratch,
                       (u32)NL);
    const unsigned grid2 = grid_for(c, m, bpc_for_slot(LQ));
    hipLaunchKernelGGL(kcrt, dim3(grid2), dim3(kBlock), lds2, s, c->K, Y, ntiles_of(m), P + t0 * LH * FPHE_WAVE);
    if (hipGetLastError() != hipSuccess) return FPHE_ERR_HIP;
  }
  return FPHE_OK;
}

// key-holder encryption: r^n mod p^2 and mod q^2 (half-size modexps), then the CRT
// recombination times the nude ciphertext.  Same integers as launch_encrypt27.
template <int L>
fphe_status launch_encrypt_crt27(fphe_ctx* c, const uint32_t* P, uint32_t lp, const uint8_t* neg, size_t count,
                                 const uint32_t* r, const uint32_t key[8], uint64_t nonce, uint32_t* C,
                                 uint8_t* sign, hipStream_t s) {
  constexpr int TPIh = L / 64, Eh = FPHE_WAVE / TPIh, NLh = rad_ll(TPIh) * TPIh, L1 = L / 2;
  constexpr int TPI = L / 32, E = FPHE_WAVE / TPI, NL = rad_ll(TPI) * TPI, LDSW = NL > L + 3 ? NL : L + 3;
  constexpr int TPIs = L >= 128 ? L / 128 : 1, Es = FPHE_WAVE / TPIs, NLs = rad_ll(TPIs) * TPIs;
  auto k1 = KS<TPIh>::template pow_half<L, kWinSlide, true>();
  const size_t lds1 = (size_t)kWavesPerBlock * NLh * Eh * 4;
  set_lds(k1, lds1);
  const size_t span = span_elems(c, k1, lds1, Eh);
  const size_t m0 = count < span ? count : span;
  const unsigned g1 = occ_grid(c, k1, lds1, (m0 + Eh - 1) / Eh, "pow_half27<enc>");
  size_t tbytes = (size_t)g1 * kWavesPerBlock * kTabEntries<kWinSlide> * rad_ll(TPIh) * FPHE_WAVE * 4;
  // the split modexp's first step (FPHE_KH_SPLIT): z_s = r^(e_s) mod s into Z, then k1 raises
  // z_s to s mod s^2; both share the window-table region
  auto k0 = KS<TPIs>::template pow_small<L, kWinSlide>();
  const size_t lds0 = (size_t)kWavesPerBlock * NLs * Es * 4;
  unsigned g0 = 0;
  size_t zbytes = 0;
  const bool direct = !r && c->kh_direct && c->kh_direct_z;
  if (kKhSplit<L> && !direct) {  // the direct draw skips the first step (and its table)
    set_lds(k0, lds0);
    g0 = occ_grid(c, k0, lds0, (m0 + Es - 1) / Es, "pow_small27");
    tbytes = std::max(tbytes, (size_t)g0 * kWavesPerBlock * kTabEntries<kWinSlide> * rad_ll(TPIs) * FPHE_WAVE * 4);
  }
  if (kKhSplit<L> || direct) zbytes = (size_t)ntiles_of(m0) * 2 * kZWords<L> * FPHE_WAVE * 4;
  // the second step alone on drawn (z_p, z_q): k1 itself when the key splits its modexp,
  // otherwise (keys <= 1024 bits) the same kernel reading Z (|p|-bit exponent in place of |n|)
  auto k1z = KS<TPIh>::template pow_half_z<L, kWinSlide>();
  if (direct && !kKhSplit<L>) set_lds(k1z, lds1);
  const size_t ybytes = (size_t)ntiles_of(m0) * 2 * L1 * FPHE_WAVE * 4;
  const size_t rbytes = (size_t)ntiles_of(m0) * L1 * FPHE_WAVE * 4;
  if (ensure_scratch(c, tbytes + ybytes + zbytes + ((r || direct) ? 0 : rbytes), s) != FPHE_OK) return FPHE_ERR_HIP;
  u32* Y = c->scratch + tbytes / 4;
  u32* Z = Y + ybytes / 4;
  ChaChaKey ck;
  if (!r)
    for (int i = 0; i < 8; ++i) ck.k[i] = key[i];
  auto k2 = KS<TPI>::template encrypt_crt<L>();
  const size_t lds2 = (size_t)kWavesPerBlock * LDSW * E * 4;
  set_lds(k2, lds2);
  const unsigned g2 = occ_grid(c, k2, lds2, (m0 + E - 1) / E, "encrypt_crt27");
  for (size_t e0 = 0; e0 < count; e0 += span) {
    const size_t m = count - e0 < span ? count - e0 : span, t0 = e0 / FPHE_WAVE;
    const u32* rbuf = r ? r + t0 * L1 * FPHE_WAVE : nullptr;
    const unsigned rgrid = (unsigned)std::min<size_t>((m + 255) / 256, (size_t)c->cus * 4);
    if (direct) {  // (z_p, z_q) drawn in place of r and its first modexp step
      hipLaunchKernelGGL(k_draw_z<L>, dim3(rgrid), dim3(256), 0, s, c->K, m, ck, nonce, e0, Z);
      if ((int64_t)count <= c->wide_kh_encrypt_max)  // few elements: one per wave and half
        hipLaunchKernelGGL((k_pow_half_enc_wide<L, kWinDec<TPIh>>), dim3((unsigned)(2 * m)), dim3(64), 0, s, c->K,
                           (const u32*)Z, m, Y);
      else
        hipLaunchKernelGGL(k1z, dim3(g1), dim3(kBlock), lds1, s, c->K, (const u32*)Z, m, Y, c->scratch, (u32)NLh);
      hipLaunchKernelGGL(k2, dim3(g2), dim3(kBlock), lds2, s, c->K, P + t0 * lp * FPHE_WAVE, lp, neg + e0, m, Y,
                         C + t0 * L * FPHE_WAVE, sign + e0, (u32)LDSW);
      if (hipGetLastError() != hipSuccess) return FPHE_ERR_HIP;
      continue;
    }
    if (!r) {
      u32* rdev = Z + zbytes / 4;
      hipLaunchKernelGGL(k_draw_r<L1>, dim3(rgrid), dim3(256), 0, s, c->K, m, ck, nonce, e0, rdev);
      rbuf = rdev;
    }
    if (kKhSplit<L>) {
      hipLaunchKernelGGL(k0, dim3(g0), dim3(kBlock), lds0, s, c->K, rbuf, m, Z, c->scratch, (u32)NLs);
      hipLaunchKernelGGL(k1, dim3(g1), dim3(kBlock), lds1, s, c->K, (const u32*)Z, m, Y, c->scratch, (u32)NLh);
    } else {
      hipLaunchKernelGGL(k1, dim3(g1), dim3(kBlock), lds1, s, c->K, rbuf, m, Y, c->scratch, (u32)NLh);
    }
    hipLaunchKernelGGL(k2, dim3(g2), dim3(kBlock), lds2, s, c->K, P + t0 * lp * FPHE_WAVE, lp, neg + e0, m, Y,
                       C + t0 * L * FPHE_WAVE, sign + e0, (u32)LDSW);
    if (hipGetLastError() != hipSuccess) return FPHE_ERR_HIP;
  }
  return FPHE_OK;
}

template <int L>
fphe_status launch_fold27(fphe_ctx* c, const uint32_t* Src, const uint8_t* ssign, const int32_t* sexp,
                          const int64_t* ord, const int64_t* cstart, const int32_t* clen, size_t nchunks,
                          uint32_t* Co, uint8_t* so, int32_t* eo, hipStream_t s) {
  constexpr int TPI = L / 32, E = FPHE_WAVE / TPI, NL = rad_ll(TPI) * TPI;
  auto kern = KS<TPI>::template fold<L, int64_t, false, true>();
  const size_t lds = (size_t)kWavesPerBlock * NL * E * 4;
  set_lds(kern, lds);
  const unsigned grid = occ_grid(c, kern, lds, (nchunks + E - 1) / E, "fold27");
  hipLaunchKernelGGL(kern, dim3(grid), dim3(kBlock), lds, s, c->K, Src, ssign, sexp, ord, cstart, clen, nchunks,
                     (const int32_t*)nullptr, (const int32_t*)nullptr, (u32*)nullptr, Co, so, eo, (u32)NL);
  return hip_ok(hipGetLastError());
}

// ---- SecureBoost bin indexes -> fold terms (fphe_positions_terms) ---------------------------
// positions [ns][npos] (int32 or int64, sample-major as iupdate's Vec<Vec<usize>>): term
// (i, j, t) = pair p = i npos + j, then t < stride, at p stride + t: src = i stride + t, slot =
// pos stride + t, or -1 when pos is outside [0, lim) (fphe_fold_segments then reports the
// segment out of range).  One thread per pair; the range test runs on the position's own width.
template <typename PT>
__global__ __launch_bounds__(256) void k_positions_terms(const PT* __restrict__ pos, size_t npairs, uint32_t npos,
                                                          int32_t stride, int64_t lim, int32_t* __restrict__ src,
                                                          int32_t* __restrict__ slot) {
  for (size_t p = (size_t)blockIdx.x * blockDim.x + threadIdx.x; p < npairs; p += (size_t)gridDim.x * blockDim.x) {
    const int64_t v = (int64_t)pos[p];
    const bool ok = v >= 0 && v < lim;
    const int32_t i = (int32_t)(p / npos);
    for (int32_t t = 0; t < stride; ++t) {
      src[p * stride + t] = i * stride + t;
      slot[p * stride + t] = ok ? (int32_t)v * stride + t : -1;
    }
  }
}

// ---- segmented fold with device grouping (fphe_fold_segments) --------------------------------
// Stream-ordered scratch of one call: freed (hipFreeAsync) on the call's stream at the end.
// Small requests are carved from 64-MiB arenas (256-B aligned) and large ones get their own
// block: a call makes ~50 requests, and each stream-ordered free is a packet the stream
// processes after the call's kernels (~0.5 ms of idle stream per 1M-sample histogram when
// every request had its own block, profiles/r03/r03g_*).
struct CallBufs {
  static constexpr size_t kArena = (size_t)64 << 20;
  hipStream_t s;
  std::vector<void*> ptrs;
  char* cur = nullptr;
  size_t left = 0;
  bool ok = true;
  explicit CallBufs(hipStream_t st) : s(st) {}
  template <class T>
  T* get(size_t n) {
    const size_t bytes = (((n ? n : 1) * sizeof(T)) + 255) & ~(size_t)255;
    if (bytes <= left) {
      T* r = (T*)cur;
      cur += bytes;
      left -= bytes;
      return r;
    }
    const size_t sz = bytes > kArena / 4 ? bytes : kArena;
    void* p = nullptr;
    if (hipMallocAsync(&p, sz, s) != hipSuccess) {
      ok = false;
      return nullptr;
    }
    ptrs.push_back(p);
    if (sz == bytes) return (T*)p;  // a large request: its own block, the arena stays
    cur = (char*)p + bytes;
    left = sz - bytes;
    return (T*)p;
  }
  ~CallBufs() {
    for (void* p : ptrs) (void)hipFreeAsync(p, s);
  }
};

constexpr size_t kMaxFoldKeys = (size_t)1 << 25;  // (segment, exponent) buckets per call
// one squaring on a lone wave (~35 us) in products of chip-wide fold throughput
// (~1.6 ns each): the merge chain's price in k_gr_gapchoose
constexpr long long kLoneSquaringProducts = 20000;

fphe_status ensure_side(fphe_ctx* c) {
  if (c->side) return FPHE_OK;
  if (hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking) != hipSuccess) {
    c->side = nullptr;
    return FPHE_ERR_HIP;
  }
  if (hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming) != hipSuccess)
    return FPHE_ERR_HIP;
  return FPHE_OK;
}

// Joins work forked onto the context's side stream back into the call's stream when the
// call returns, on every path: declared after the call's CallBufs, it runs first, so the
// stream-ordered frees of the call's scratch come after the side work.
struct SideJoin {
  fphe_ctx* c;
  hipStream_t s;
  bool armed = false;
  ~SideJoin() {
    if (armed) (void)hipStreamWaitEvent(s, c->ev_join, 0);
  }
  fphe_status join() {
    if (!armed) return FPHE_OK;
    armed = false;
    return hip_ok(hipStreamWaitEvent(s, c->ev_join, 0));
  }
};

// exclusive scan of n int32 on the device (3 launches); the total lands in *total if given
fphe_status dev_scan(const fphe_ctx* c, const int32_t* in, size_t n, int32_t* out, int32_t* total, CallBufs& B) {
  const size_t nb = (n + kScanTile - 1) / kScanTile;
  int32_t* bsum = B.get<int32_t>(nb);
  if (!B.ok) return FPHE_ERR_HIP;
  hipLaunchKernelGGL(k_scan_tiles, dim3((unsigned)(nb ? nb : 1)), dim3(kGrBlock), 0, B.s, in, n, out, bsum);
  hipLaunchKernelGGL(k_scan_sums, dim3(1), dim3(kGrBlock), 0, B.s, bsum, nb, total);
  hipLaunchKernelGGL(k_scan_add, dim3((unsigned)(nb ? nb : 1)), dim3(kGrBlock), 0, B.s, out, n, bsum);
  (void)c;
  return hip_ok(hipGetLastError());
}

int32_t fold_klen(size_t n) {  // chunk length: fill ~32K wave slots, 8..64 terms (kFoldMax)
  size_t k = (n + 32767) / 32768;
  return (int32_t)(k < 8 ? 8 : (k > (size_t)kFoldMax ? (size_t)kFoldMax : k));
}

// A fold level's input: items (element-major rows + sign + exp), grouped by key in
// contiguous runs: key k's items at [off[k], off[k] + cnt[k]) of the item order (ord, or the
// items themselves when ord is null).  Sizes past the first level live on the device (n_dev);
// the host keeps upper bounds (n_ub items, maxcnt per key, nnz non-empty keys), so the levels
// run back to back without reading anything back.
struct FoldLevel {
  const u32* rows;
  const u8* sign;
  const int32_t* exp;
  const int32_t* ord;
  const int32_t* cnt;
  const int32_t* off;
  size_t nkeys;
  size_t n_ub;     // items (exact on the first level)
  int32_t maxcnt;  // largest run (bound)
  size_t nnz;      // non-empty keys (bound)
};
struct FoldOut {
  u32* rows;
  u8* sign;
  int32_t* exp;
  int32_t* key;    // key of each output partial (ascending)
  int32_t* cnt;    // per key: partials produced
  int32_t* off;    // per key: first partial
  int32_t* n_dev;  // partials (device)
  size_t n_ub;     // partials (bound)
  int32_t maxcnt;
};

// stats (may be null): the first level reads back {largest run, non-empty keys}
template <int L>
fphe_status fold_level(fphe_ctx* c, FoldLevel& in, FoldOut& out, CallBufs& B, bool read_stats) {
  constexpr int TPI = L / 32, E = FPHE_WAVE / TPI, NL = rad_ll(TPI) * TPI;
  hipStream_t s = B.s;
  const int32_t k = fold_klen(in.n_ub);
  int32_t* nch = B.get<int32_t>(in.nkeys);
  int32_t* choff = B.get<int32_t>(in.nkeys);
  int32_t* hdr = B.get<int32_t>(4);
  if (!B.ok) return FPHE_ERR_HIP;
  if (hipMemsetAsync(hdr, 0, 4 * sizeof(int32_t), s) != hipSuccess) return FPHE_ERR_HIP;
  hipLaunchKernelGGL(k_gr_nchunks, dim3(gr_grid(in.nkeys, c->cus)), dim3(kGrBlock), 0, s, in.cnt, in.nkeys, k, nch, hdr);
  if (dev_scan(c, nch, in.nkeys, choff, hdr + 2, B) != FPHE_OK) return FPHE_ERR_HIP;
  if (read_stats) {
    int32_t h[4];
    if (hipMemcpyAsync(h, hdr, sizeof(h), hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
      return FPHE_ERR_HIP;
    in.maxcnt = h[0];
    in.nnz = (size_t)h[1];
  }
  // chunks <= sum over non-empty keys of (cnt / k + 1)
  const size_t ub = in.n_ub / (size_t)k + in.nnz + 1;
  int32_t* cstart = B.get<int32_t>(ub);
  int32_t* clen = B.get<int32_t>(ub);
  out.key = B.get<int32_t>(ub);
  out.rows = B.get<u32>(ub * L);
  out.sign = B.get<u8>(ub);
  out.exp = B.get<int32_t>(ub);
  if (!B.ok) return FPHE_ERR_HIP;
  hipLaunchKernelGGL(k_gr_chunks, dim3(gr_grid(in.nkeys, c->cus)), dim3(kGrBlock), 0, s, in.cnt, in.off, choff, in.nkeys,
                     k, cstart, clen, out.key);
  // big levels: chunks handed to the waves longest first (a counting sort on the length) and
  // wave tiles from a device counter; the outputs stay in key order (row = chunk index)
  int32_t* cperm = nullptr;
  u32* ctr = nullptr;
  if (ub >= ((size_t)1 << 15)) {
    int32_t* nfull = B.get<int32_t>(in.nkeys);
    int32_t* fulloff = B.get<int32_t>(in.nkeys);
    int32_t* bc = B.get<int32_t>((size_t)k + 1);
    int32_t* boff = B.get<int32_t>((size_t)k + 1);
    int32_t* bfill = B.get<int32_t>((size_t)k + 1);
    int32_t* nf = B.get<int32_t>(1);
    cperm = B.get<int32_t>(ub);
    ctr = B.get<u32>(1);
    if (!B.ok) return FPHE_ERR_HIP;
    if (hipMemsetAsync(bc, 0, (k + 1) * 4, s) != hipSuccess || hipMemsetAsync(bfill, 0, (k + 1) * 4, s) != hipSuccess ||
        hipMemsetAsync(ctr, 0, 4, s) != hipSuccess)
      return FPHE_ERR_HIP;
    const unsigned gk = gr_grid(in.nkeys, c->cus);
    hipLaunchKernelGGL(k_gr_permcnt, dim3(gk), dim3(kGrBlock), 0, s, in.cnt, in.nkeys, k, nfull, bc);
    if (dev_scan(c, nfull, in.nkeys, fulloff, nf, B) != FPHE_OK) return FPHE_ERR_HIP;
    if (dev_scan(c, bc, (size_t)k + 1, boff, nullptr, B) != FPHE_OK) return FPHE_ERR_HIP;
    hipLaunchKernelGGL(k_gr_perm, dim3(gk), dim3(kGrBlock), 0, s, in.cnt, choff, nfull, fulloff, nf, boff, bfill,
                       in.nkeys, k, cperm);
  }
  auto kern = in.ord ? KS<TPI>::template fold<L, int32_t, true, true>()
                     : KS<TPI>::template fold<L, int32_t, true, false>();
  const size_t lds = (size_t)kWavesPerBlock * NL * E * 4;
  set_lds(kern, lds);
  const unsigned grid = occ_grid(c, kern, lds, (ub + E - 1) / E, "fold_segments");
  hipLaunchKernelGGL(kern, dim3(grid), dim3(kBlock), lds, s, c->K, in.rows, in.sign, in.exp, in.ord, cstart, clen,
                     ub, (const int32_t*)(hdr + 2), (const int32_t*)cperm, ctr, out.rows, out.sign, out.exp,
                     (u32)NL);
  out.cnt = nch;
  out.off = choff;
  out.n_dev = hdr + 2;
  out.n_ub = ub;
  out.maxcnt = (in.maxcnt + k - 1) / k;
  return hip_ok(hipGetLastError());
}

// every key's run of element-major items (contiguous, in.ord null) to one partial in one
// launch: k_keytree27, a wave per key (sequential slot folds, then a product tree over the
// wave's slots).  The outputs are compacted to the non-empty keys in key order (at most
// in.nnz of them, the exact count on the device).
template <int L>
fphe_status fold_keys_tree(fphe_ctx* c, const FoldLevel& in, FoldOut& out, CallBufs& B) {
  constexpr int TPI = L / 32, E = FPHE_WAVE / TPI, NL = rad_ll(TPI) * TPI;
  hipStream_t s = B.s;
  int32_t* flag = B.get<int32_t>(in.nkeys);
  int32_t* pos = B.get<int32_t>(in.nkeys);
  int32_t* hdr = B.get<int32_t>(4);
  const size_t ub = in.nnz ? in.nnz : 1;
  out.rows = B.get<u32>(ub * L);
  out.sign = B.get<u8>(ub);
  out.exp = B.get<int32_t>(ub);
  out.key = B.get<int32_t>(ub);
  if (!B.ok) return FPHE_ERR_HIP;
  if (hipMemsetAsync(hdr, 0, 4 * sizeof(int32_t), s) != hipSuccess) return FPHE_ERR_HIP;
  // flag[k] = (cnt[k] + 2^30 - 1) / 2^30 = 1 for a non-empty key (counts < 2^30), else 0
  hipLaunchKernelGGL(k_gr_nchunks, dim3(gr_grid(in.nkeys, c->cus)), dim3(kGrBlock), 0, s, in.cnt, in.nkeys,
                     (int32_t)1 << 30, flag, hdr);
  if (dev_scan(c, flag, in.nkeys, pos, hdr + 2, B) != FPHE_OK) return FPHE_ERR_HIP;
  int32_t* keyof = B.get<int32_t>(ub);
  if (!B.ok) return FPHE_ERR_HIP;
  hipLaunchKernelGGL(k_gr_keyof, dim3(gr_grid(in.nkeys, c->cus)), dim3(kGrBlock), 0, s, (const int32_t*)flag,
                     (const int32_t*)pos, in.nkeys, keyof);
  auto kern = KS<TPI>::template keytree<L>();
  const size_t lds = (size_t)kWavesPerBlock * NL * E * 4;
  set_lds(kern, lds);
  const unsigned grid = occ_grid(c, kern, lds, ub, "keytree");  // a wave per non-empty key (bound)
  hipLaunchKernelGGL(kern, dim3(grid), dim3(kBlock), lds, s, c->K, in.rows, in.sign, in.exp, in.cnt, in.off,
                     (const int32_t*)keyof, (const int32_t*)(hdr + 2), out.rows, out.sign, out.exp, out.key, (u32)NL);
  out.cnt = flag;
  out.off = pos;
  out.n_dev = hdr + 2;
  out.n_ub = ub;
  out.maxcnt = 1;
  return hip_ok(hipGetLastError());
}

// the largest per-key run the tree fold takes (FPHE_FOLD_TREE_MAX; 0: the chunk levels always)
int32_t fold_tree_max() {
  const char* e = getenv("FPHE_FOLD_TREE_MAX");
  return e ? (int32_t)strtol(e, nullptr, 10) : 256;
}

// fold every key's run down to one partial (levels of chunked products)
template <int L>
fphe_status fold_runs(fphe_ctx* c, FoldLevel lv, FoldOut& out, CallBufs& B, bool read_stats) {
  const int32_t tree_max = fold_tree_max();
  for (;;) {
    // short runs: the rest in one tree launch (chunk levels first while runs are long)
    if (!read_stats && !lv.ord && lv.maxcnt > 1 && lv.maxcnt <= tree_max) return fold_keys_tree<L>(c, lv, out, B);
    if (fold_level<L>(c, lv, out, B, read_stats) != FPHE_OK) return FPHE_ERR_HIP;
    read_stats = false;
    if (out.maxcnt <= 1) return FPHE_OK;
    lv = FoldLevel{out.rows, out.sign, out.exp, nullptr, out.cnt, out.off, lv.nkeys, out.n_ub, out.maxcnt, lv.nnz};
  }
}

template <int L>
fphe_status launch_fold_segments(fphe_ctx* c, const u32* Src, const u8* ssign, const int32_t* sexp, size_t nsrc,
                                 const int32_t* idx, const int32_t* seg, size_t T, size_t nseg, u32* Co, u8* so,
                                 int32_t* eo, u8* present, int32_t* err, hipStream_t s) {
  constexpr int TPI = L / 32, E = FPHE_WAVE / TPI, NL = rad_ll(TPI) * TPI;
  CallBufs B(s);
  const unsigned g0 = gr_grid(nseg * FPHE_WAVE, c->cus);
  hipLaunchKernelGGL(k_gr_init_out<L>, dim3(g0), dim3(kGrBlock), 0, s, nseg, c->K.N2M1, Co, so, eo, present);
  if (T == 0) return hip_ok(hipGetLastError());
  // 1. element-major copy of the source (the fold gathers whole rows), on the context's side
  // stream: it overlaps the counting sort below, and the stream joins it before the fold (or on
  // any early return, before the scratch is freed).  It is forked before the exponent-range
  // read-back, beside k_gr_minmax (which then shares HBM with it: ~0.3 ms).  Forking it after
  // the read-back instead (FPHE_FOLD_COPY_EARLY=0) measured the same call time, 16.59 against
  // 16.53 ms median over 12 alternating cold calls (profiles/r06/r06f_iupdate_ab_copy_late.txt)
  int32_t* mm = B.get<int32_t>(4);
  u32* rows = B.get<u32>(nsrc * L);
  if (!B.ok) return FPHE_ERR_HIP;
  SideJoin sj{c, s};
  auto fork_copy = [&]() -> fphe_status {
    if (ensure_side(c) != FPHE_OK || hipEventRecord(c->ev_fork, s) != hipSuccess ||
        hipStreamWaitEvent(c->side, c->ev_fork, 0) != hipSuccess)
      return FPHE_ERR_HIP;
    hipLaunchKernelGGL(k_tiles_to_rows<L>, dim3((unsigned)std::min<size_t>(ntiles_of(nsrc), (size_t)c->cus * 8)),
                       dim3(kGrBlock), 0, c->side, Src, nsrc, rows);
    if (hipEventRecord(c->ev_join, c->side) != hipSuccess) {
      (void)hipStreamSynchronize(c->side);
      return FPHE_ERR_HIP;
    }
    sj.armed = true;
    return FPHE_OK;
  };
  const char* ce = getenv("FPHE_FOLD_COPY_EARLY");
  const bool copy_early = !(ce && ce[0] == '0');
  if (copy_early && fork_copy() != FPHE_OK) return FPHE_ERR_HIP;
  // 2. exponent range (one small read back: it sizes the key space)
  const int32_t mm0[4] = {kI32Max, kI32Min, 0, 0};
  if (hipMemcpyAsync(mm, mm0, sizeof(mm0), hipMemcpyHostToDevice, s) != hipSuccess) return FPHE_ERR_HIP;
  hipLaunchKernelGGL(k_gr_minmax, dim3(gr_grid(T, c->cus)), dim3(kGrBlock), 0, s, idx, seg, sexp, T, nsrc, nseg, mm);
  int32_t h[4];
  if (hipMemcpyAsync(h, mm, sizeof(h), hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
    return FPHE_ERR_HIP;
  if (h[2]) return FPHE_ERR_ARG;  // an index or segment out of range
  if (!copy_early && fork_copy() != FPHE_OK) return FPHE_ERR_HIP;
  const int32_t emin = h[0];  // (h is reused for later read-backs)
  const int64_t NE = (int64_t)h[1] - h[0] + 1;
  if (NE < 1 || (size_t)NE * nseg > kMaxFoldKeys) return FPHE_ERR_RANGE;
  const size_t nkeys = (size_t)NE * nseg;
  // small key spaces: per-block LDS counts (k_gr_bkeys / k_gr_bscatter); larger ones: counter
  // copies against atomic contention on hot keys (k_gr_keys), while they stay small
  const bool lds_counts = nkeys <= kBcMaxKeys;
  const int32_t R = lds_counts ? 1 : (nkeys <= ((size_t)1 << 22) ? 8 : 1);
  int32_t* keys = B.get<int32_t>(T);
  int32_t* cntR = B.get<int32_t>(nkeys * R);
  int32_t* offR = B.get<int32_t>(nkeys * R);
  int32_t* fill = B.get<int32_t>(nkeys * R);
  int32_t* last = B.get<int32_t>(nseg);
  u8* litseg = B.get<u8>(nseg);
  int32_t* ord = B.get<int32_t>(T);
  int32_t* skey = B.get<int32_t>(T);
  if (!B.ok) return FPHE_ERR_HIP;
  // 3. keys, counts, counting sort
  if (hipMemsetAsync(cntR, 0, nkeys * R * 4, s) != hipSuccess || hipMemsetAsync(fill, 0, nkeys * R * 4, s) != hipSuccess ||
      hipMemsetAsync(last, 0xff, nseg * 4, s) != hipSuccess || hipMemsetAsync(litseg, 0, nseg, s) != hipSuccess)
    return FPHE_ERR_HIP;
  const unsigned nbc = (unsigned)((T + kBcTerms - 1) / kBcTerms);
  if (lds_counts) {
    set_lds(k_gr_bkeys, nkeys * 4);
    set_lds(k_gr_bscatter, nkeys * 4);
  }
  if (lds_counts)
    hipLaunchKernelGGL(k_gr_bkeys, dim3(nbc), dim3(kGrBlock), nkeys * 4, s, idx, seg, sexp, T, h[0], (int32_t)NE,
                       (int32_t)nkeys, keys, cntR);
  else
    hipLaunchKernelGGL(k_gr_keys, dim3(gr_grid(T, c->cus)), dim3(kGrBlock), 0, s, idx, seg, sexp, T, h[0], (int32_t)NE,
                       R, keys, cntR);
  if (dev_scan(c, cntR, nkeys * R, offR, nullptr, B) != FPHE_OK) return FPHE_ERR_HIP;
  if (lds_counts)
    hipLaunchKernelGGL(k_gr_bscatter, dim3(nbc), dim3(kGrBlock), nkeys * 4, s, keys, idx, ssign, T, (int32_t)nkeys,
                       offR, fill, ord, skey);
  else
    hipLaunchKernelGGL(k_gr_scatter, dim3(gr_grid(T, c->cus)), dim3(kGrBlock), 0, s, keys, idx, ssign, T, R, offR, fill,
                       ord, skey);
  // 4. fold every (segment, exponent) run to one partial.  First level: the sorted items in
  // equal ranges of r per wave slot, whatever the runs (k_segfold27: balanced, a whole number
  // of wave rounds); then chunk levels per key until one partial is left per key.
  auto ksf = KS<TPI>::template segfold<L, true>();
  const size_t lds = (size_t)kWavesPerBlock * NL * E * 4;
  set_lds(ksf, lds);
  const size_t round = (size_t)occ_grid(c, ksf, lds, (size_t)1 << 40, "segfold") * kWavesPerBlock * E;
  size_t r = (T + round - 1) / round;
  r = r < 8 ? 8 : (r > (size_t)kSegFoldMax ? (size_t)kSegFoldMax : r);
  size_t nslots = (T + r - 1) / r;
  // raised keys (group_dev.h k_gr_gapsel / k_gr_gapchoose / k_gr_plan): keys far enough above
  // their segment's least exponent that raising them inside the balanced level costs less than
  // their merge chain get slots of their own whose partials k_segfold27 raises in place.
  // FPHE_FOLD_RAISE=0 turns it off, =force raises every key above the least (tests).
  const char* rmode = getenv("FPHE_FOLD_RAISE");
  const bool rforce = rmode && !strcmp(rmode, "force");
  const bool raise = NE > 1 && lds_counts && !(rmode && !strcmp(rmode, "0"));
  int32_t* plan = nullptr;
  u8* raised = nullptr;
  if (raise) {
    const size_t smax = 2 * std::max(round, nslots) + 2 * (size_t)kRaiseMax + 2;
    if (smax < ((size_t)1 << 31)) {
      int32_t* ng = B.get<int32_t>(2);  // [0] keys recorded, [1] the chosen threshold
      int32_t* gk = B.get<int32_t>(5 * (size_t)kRaiseMax);
      unsigned long long* ghist = B.get<unsigned long long>(kGapHist);
      int32_t* gnum = B.get<int32_t>(kGapHist);
      plan = B.get<int32_t>(kPlanWords);
      raised = B.get<u8>(nkeys);
      if (!B.ok) return FPHE_ERR_HIP;
      if (hipMemsetAsync(ng, 0, 8, s) != hipSuccess || hipMemsetAsync(raised, 0, nkeys, s) != hipSuccess ||
          hipMemsetAsync(ghist, 0, kGapHist * 8, s) != hipSuccess || hipMemsetAsync(gnum, 0, kGapHist * 4, s) != hipSuccess)
        return FPHE_ERR_HIP;
      const int32_t gmin = rforce ? 1 : 4, xmax = rforce ? kI32Max : (int32_t)(r - 1);
      const unsigned gsg = gr_grid(nseg, c->cus);
      int32_t* gsel = nullptr;
      if (!rforce) {  // pass 1 and the threshold (group_dev.h); forced: every candidate
        hipLaunchKernelGGL(k_gr_gapsel<L>, dim3(gsg), dim3(kGrBlock), 0, s, cntR, offR, nseg, (int32_t)NE, h[0], gmin,
                           xmax, (int32_t)r, (const int32_t*)ord, Src, ssign, c->K.N2M1, ghist, gnum,
                           (const int32_t*)nullptr, ng, gk, gk + kRaiseMax, gk + 2 * kRaiseMax, gk + 3 * kRaiseMax,
                           gk + 4 * kRaiseMax);
        gsel = ng + 1;
        hipLaunchKernelGGL(k_gr_gapchoose, dim3(1), dim3(1), 0, s, ghist, gnum, gmin, kLoneSquaringProducts, gsel);
      }
      hipLaunchKernelGGL(k_gr_gapsel<L>, dim3(gsg), dim3(kGrBlock), 0, s, cntR, offR, nseg, (int32_t)NE, h[0], gmin,
                         xmax, (int32_t)r, (const int32_t*)ord, Src, ssign, c->K.N2M1, (unsigned long long*)nullptr,
                         (int32_t*)nullptr, (const int32_t*)gsel, ng, gk, gk + kRaiseMax, gk + 2 * kRaiseMax,
                         gk + 3 * kRaiseMax, gk + 4 * kRaiseMax);
      hipLaunchKernelGGL(k_gr_plan, dim3(1), dim3(kGrBlock), 0, s, ng, gk, gk + kRaiseMax, gk + 2 * kRaiseMax,
                         gk + 3 * kRaiseMax, gk + 4 * kRaiseMax, (int64_t)T, (int32_t)round, (int32_t)r,
                         (int32_t)kSegFoldMax, (int32_t)smax, plan, raised);
      if (getenv("FPHE_DEBUG")) {  // the plan's size (a read-back: debugging only)
        int32_t ph[2] = {0, 0}, nh = 0;
        if (hipMemcpyAsync(ph, plan, 8, hipMemcpyDeviceToHost, s) == hipSuccess &&
            hipMemcpyAsync(&nh, ng, 4, hipMemcpyDeviceToHost, s) == hipSuccess && hipStreamSynchronize(s) == hipSuccess)
          fprintf(stderr, "[fphe] fold plan: %d raise candidates, %d regions, %d slots (r0 %zu, round %zu, T %zu)\n", nh,
                  ph[0], ph[1], r, round, T);
      }
      nslots = smax;  // a bound: the plan's count is on the device (slots past it stay empty)
    }
  }
  int32_t* pcnt = B.get<int32_t>(nslots);
  int32_t* poff = B.get<int32_t>(nslots);
  int32_t* cnt2 = B.get<int32_t>(nkeys);
  int32_t* off2 = B.get<int32_t>(nkeys);
  int32_t* tmp = B.get<int32_t>(nkeys);
  int32_t* hdr = B.get<int32_t>(4);
  if (!B.ok) return FPHE_ERR_HIP;
  if (hipMemsetAsync(cnt2, 0, nkeys * 4, s) != hipSuccess || hipMemsetAsync(hdr, 0, 16, s) != hipSuccess ||
      (plan && hipMemsetAsync(pcnt, 0, nslots * 4, s) != hipSuccess))
    return FPHE_ERR_HIP;
  hipLaunchKernelGGL(k_gr_segcount, dim3(gr_grid(nslots, c->cus)), dim3(kGrBlock), 0, s, skey, T, (u32)r,
                     (const int32_t*)plan, pcnt, cnt2);
  if (dev_scan(c, pcnt, nslots, poff, hdr + 2, B) != FPHE_OK || dev_scan(c, cnt2, nkeys, off2, nullptr, B) != FPHE_OK)
    return FPHE_ERR_HIP;
  hipLaunchKernelGGL(k_gr_nchunks, dim3(gr_grid(nkeys, c->cus)), dim3(kGrBlock), 0, s, cnt2, nkeys, 1, tmp, hdr);
  if (hipMemcpyAsync(h, hdr, sizeof(h), hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
    return FPHE_ERR_HIP;
  const size_t nnz = (size_t)h[1];  // non-empty (segment, exponent) keys
  const size_t ub1 = nslots + nnz;
  FoldOut P{};
  P.rows = B.get<u32>(ub1 * L);
  P.sign = B.get<u8>(ub1);
  P.exp = B.get<int32_t>(ub1);
  P.key = B.get<int32_t>(ub1);
  if (!B.ok || sj.join() != FPHE_OK) return FPHE_ERR_HIP;
  hipLaunchKernelGGL(ksf, dim3(occ_grid(c, ksf, lds, (nslots + E - 1) / E, "segfold")), dim3(kBlock), lds, s, c->K,
                     rows, emin, (int32_t)NE, ord, skey, T, (u32)r, (const int32_t*)plan, poff, P.rows, P.sign, P.exp, P.key,
                     (u32)NL);
  P.cnt = cnt2;
  P.off = off2;
  P.n_dev = hdr + 2;
  P.n_ub = ub1;
  P.maxcnt = h[0];
  if (P.maxcnt > 1) {
    FoldOut Q{};
    FoldLevel lv{P.rows, P.sign, P.exp, nullptr, cnt2, off2, nkeys, ub1, P.maxcnt, nnz};
    if (fold_runs<L>(c, lv, Q, B, false) != FPHE_OK) return FPHE_ERR_HIP;
    P = Q;
  }
  // 5. merge each segment's per-exponent partials: align to the segment's least exponent, fold
  if (NE > 1) {
    const size_t np = P.n_ub;  // partials (bound); the exact count is P.n_dev
    int32_t* segmin = B.get<int32_t>(nseg);
    u8* lit = B.get<u8>(np);
    int32_t* gap = B.get<int32_t>(np);
    int32_t* skey = B.get<int32_t>(np);
    int32_t* scnt = B.get<int32_t>(nseg);
    int32_t* soff = B.get<int32_t>(nseg);
    int32_t* gh = B.get<int32_t>(2);
    if (!B.ok) return FPHE_ERR_HIP;
    if (hipMemsetD32Async((hipDeviceptr_t)segmin, kI32Max, nseg, s) != hipSuccess ||
        hipMemsetAsync(scnt, 0, nseg * 4, s) != hipSuccess || hipMemsetAsync(gh, 0, 8, s) != hipSuccess)
      return FPHE_ERR_HIP;
    const unsigned gp = gr_grid(np, c->cus);
    hipLaunchKernelGGL(k_gr_segmin<L>, dim3(gp), dim3(kGrBlock), 0, s, P.rows, P.sign, P.exp, P.key, P.n_dev,
                       (int32_t)NE, c->K.N2M1, (const u8*)raised, segmin, lit);
    hipLaunchKernelGGL(k_gr_gaps, dim3(gp), dim3(kGrBlock), 0, s, P.exp, P.key, lit, (const u8*)raised, P.n_dev,
                       (int32_t)NE, segmin, gap, skey, scnt, gh, err);
    // partials in descending-gap order (counting sort on NE - 1 - gap: every gap < NE), then
    // the alignment; waves whose partials all have gap 0 skip their tile at once
    const size_t ng = (size_t)NE;
    int32_t* gk = B.get<int32_t>(np);
    int32_t* gc = B.get<int32_t>(ng);
    int32_t* go = B.get<int32_t>(ng);
    int32_t* gf = B.get<int32_t>(ng);
    int32_t* gord = B.get<int32_t>(np);
    u32* tile_ctr = B.get<u32>(1);
    if (!B.ok) return FPHE_ERR_HIP;
    if (hipMemsetAsync(gc, 0, ng * 4, s) != hipSuccess || hipMemsetAsync(gf, 0, ng * 4, s) != hipSuccess ||
        hipMemsetAsync(tile_ctr, 0, 4, s) != hipSuccess)
      return FPHE_ERR_HIP;
    hipLaunchKernelGGL(k_gr_gapkeys, dim3(gp), dim3(kGrBlock), 0, s, gap, P.n_dev, (int32_t)(NE - 1), gk, gc);
    if (dev_scan(c, gc, ng, go, nullptr, B) != FPHE_OK) return FPHE_ERR_HIP;
    hipLaunchKernelGGL(k_gr_scatter_n, dim3(gp), dim3(kGrBlock), 0, s, gk, P.n_dev, go, gf, gord);
    auto ka = KS<TPI>::template align_rows<L>();
    set_lds(ka, lds);
    const unsigned ga = occ_grid(c, ka, lds, (np + E - 1) / E, "align_rows");
    hipLaunchKernelGGL(ka, dim3(ga), dim3(kBlock), lds, s, c->K, P.rows, P.sign, gap, gord, P.n_dev, tile_ctr,
                       (u32)NL);
    // the partials are in (segment, exponent) order: contiguous per segment
    if (dev_scan(c, scnt, nseg, soff, nullptr, B) != FPHE_OK) return FPHE_ERR_HIP;
    FoldOut Q{};
    FoldLevel lv2{P.rows, P.sign, P.exp, nullptr, scnt, soff, nseg, np, (int32_t)std::min<int64_t>(NE, (int64_t)np),
                  std::min(nseg, nnz)};
    if (fold_runs<L>(c, lv2, Q, B, false) != FPHE_OK) return FPHE_ERR_HIP;
    P = Q;
  }
  // 6. scatter to the output segments (keys are segment ids here)
  hipLaunchKernelGGL(k_gr_final<L>, dim3(gr_grid(P.n_ub * 64, c->cus)), dim3(kGrBlock), 0, s, P.rows, P.sign, P.exp,
                     P.key, P.n_dev, c->K.N2M1, litseg, Co, so, eo, present);
  // literal-1 results end on their segment's last term's exponent
  hipLaunchKernelGGL(k_gr_last, dim3(gr_grid(T, c->cus)), dim3(kGrBlock), 0, s, seg, T, litseg, last);
  hipLaunchKernelGGL(k_gr_litexp, dim3(gr_grid(nseg, c->cus)), dim3(kGrBlock), 0, s, nseg, litseg, last, idx, sexp, eo);
  return hip_ok(hipGetLastError());
}

// Largest element count whose C vector (count x L words) one k_add27 launch addresses
// through 32-bit buffer offsets (whole-vector descriptors, a margin below 4 GiB).
size_t add_max_count(int L) {
  return (((size_t)1 << 32) - ((size_t)1 << 20)) / ((size_t)L * 4) / FPHE_WAVE * FPHE_WAVE;
}

template <int L>
fphe_status launch_add27(fphe_ctx* c, const uint32_t* Ca, const uint8_t* sa, const int32_t* ea, const uint32_t* Cb,
                         const uint8_t* sb, const int32_t* eb, int bstride, size_t count, const int32_t* ord,
                         uint32_t* Co, uint8_t* so, int32_t* eo, int32_t* err, hipStream_t s) {
  constexpr int TPI = L / 32, E = FPHE_WAVE / TPI, NL = rad_ll(TPI) * TPI;
  auto kern = KS<TPI>::template add<L>();
  const size_t lds = (size_t)kWavesPerBlock * NL * E * 4;
  set_lds(kern, lds);
  const size_t cmax = add_max_count(L);
  if (ord && count > cmax) return FPHE_ERR_ARG;  // an order must stay inside one addressable chunk
  if (count == 0) return FPHE_OK;
  // the kernel's wave-tile counter lives in the context scratch (stream-owned, see ensure_scratch)
  constexpr size_t kCtrBytes = (size_t)kAddRegions * kAddCounterStride * 4;
  if (ensure_scratch(c, kCtrBytes, s) != FPHE_OK) return FPHE_ERR_HIP;
  u32* next_tile = c->scratch;
  for (size_t s0 = 0; s0 < count; s0 += cmax) {  // whole tiles per chunk: pointer offsets stay tile-aligned
    const size_t n = count - s0 < cmax ? count - s0 : cmax;
    const size_t wo = s0 / FPHE_WAVE * L * FPHE_WAVE;  // word offset of the chunk's first tile
    // a multiple of kAddRegions blocks: every run of wave tiles has its own blocks
    const unsigned g0 = occ_grid(c, kern, lds, (n + E - 1) / E, "add27");
    const unsigned grid = (g0 + kAddRegions - 1) / kAddRegions * kAddRegions;
    if (hipMemsetAsync(next_tile, 0, kCtrBytes, s) != hipSuccess) return FPHE_ERR_HIP;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kBlock), lds, s, c->K, Ca + wo, sa + s0, ea + s0,
                       bstride ? Cb + wo : Cb, bstride ? sb + s0 : sb, bstride ? eb + s0 : eb, bstride, n, ord,
                       Co + wo, so + s0, eo + s0, err, next_tile, (u32)NL);
  }
  return hip_ok(hipGetLastError());
}

template <int L>
fphe_status launch_sqmul27(fphe_ctx* c, const uint32_t* Ca, const uint32_t* Cb, const uint8_t* sb, int nsq,
                           size_t count, uint32_t* Co, uint8_t* so, hipStream_t s) {
  constexpr int TPI = L / 32, E = FPHE_WAVE / TPI, NL = rad_ll(TPI) * TPI;
  auto kern = KS<TPI>::template sqmul<L>();
  const size_t lds = (size_t)kWavesPerBlock * NL * E * 4;
  set_lds(kern, lds);
  const unsigned grid = occ_grid(c, kern, lds, (count + E - 1) / E, "sqmul27");
  hipLaunchKernelGGL(kern, dim3(grid), dim3(kBlock), lds, s, c->K, Ca, Cb, sb, nsq, count, Co, so, (u32)NL);
  return hip_ok(hipGetLastError());
}

template <int L>
fphe_status launch_align27(fphe_ctx* c, const uint32_t* Ca, const uint8_t* sa, const int32_t* gap, size_t count,
                           uint32_t* Co, uint8_t* so, hipStream_t s) {
  constexpr int TPI = L / 32, E = FPHE_WAVE / TPI, NL = rad_ll(TPI) * TPI;
  auto kern = KS<TPI>::template align<L>();
  const size_t lds = (size_t)kWavesPerBlock * NL * E * 4;
  set_lds(kern, lds);
  if (ensure_scratch(c, 256, s) != FPHE_OK) return FPHE_ERR_HIP;  // the wave-tile counter
  if (hipMemsetAsync(c->scratch, 0, sizeof(u32), s) != hipSuccess) return FPHE_ERR_HIP;
  const unsigned grid = occ_grid(c, kern, lds, (count + E - 1) / E, "align27");
  hipLaunchKernelGGL(kern, dim3(grid), dim3(kBlock), lds, s, c->K, Ca, sa, gap, count, Co, so, c->scratch, (u32)NL);
  return hip_ok(hipGetLastError());
}

// X0: scratch of ntiles * L1 * 64 words (the mod-n inverses between the two kernels)
template <int L>
void launch_inv27(fphe_ctx* c, const uint32_t* Ca, size_t count, const uint8_t* need, uint32_t* Co,
                  int32_t* err, u32* X0, hipStream_t s) {
  constexpr int TPIh = L / 64, Eh = FPHE_WAVE / TPIh, NLh = rad_ll(TPIh) * TPIh, L1 = L / 2;
  constexpr int TPI = L / 32, E = FPHE_WAVE / TPI, NL = rad_ll(TPI) * TPI;
  auto k1 = KS<TPIh>::template inv_n<L>();
  const size_t lds1 = (size_t)kWavesPerBlock * NLh * Eh * 4;
  set_lds(k1, lds1);
  const unsigned g1 = occ_grid(c, k1, lds1, (count + Eh - 1) / Eh, "inv_n27");
  (void)L1;
  hipLaunchKernelGGL(k1, dim3(g1), dim3(kBlock), lds1, s, c->K, Ca, count, need, X0, err, (u32)NLh);
  auto k2 = KS<TPI>::template inv_lift<L>();
  const size_t lds2 = (size_t)kWavesPerBlock * NL * E * 4;
  set_lds(k2, lds2);
  const unsigned g2 = occ_grid(c, k2, lds2, (count + E - 1) / E, "inv_lift27");
  hipLaunchKernelGGL(k2, dim3(g2), dim3(kBlock), lds2, s, c->K, Ca, count, need, X0, Co, (u32)NL);
}

// Batch inversion mod n^2 (kernels27.h k_binv_pre27 / k_binv_post27): Co[e] = Ca[e]^-1 for
// every element (need == nullptr) or those with need[e] != 0.  Scratch W (binv_scratch_bytes):
// the prefix table (608 B/element at 2048 bits), the group totals, their inverses, the
// inverse's mod-n intermediate.
template <int L>
size_t binv_scratch_bytes(size_t count) {
  constexpr int TPI = L / 32, E = FPHE_WAVE / TPI, PER = FPHE_WAVE / E, KB = 4 * PER;
  const size_t nwt = (ntiles_of(count) + 3) / 4, ntot = nwt * E;
  return nwt * KB * rad_ll(TPI) * FPHE_WAVE * 4 + 2 * (size_t)ntiles_of(ntot) * L * FPHE_WAVE * 4 +
         (size_t)ntiles_of(ntot) * (L / 2) * FPHE_WAVE * 4;
}

// Vectors from this many elements invert by batches; shorter ones with one inverse each.
size_t binv_min() {
  static const size_t v = getenv("FPHE_NEG_BATCH_MIN") ? (size_t)atoll(getenv("FPHE_NEG_BATCH_MIN")) : 4096;
  return v;
}

template <int L>
void launch_binv27(fphe_ctx* c, const uint32_t* Ca, size_t count, const uint8_t* need, uint32_t* Co, int32_t* err,
                   u32* W, hipStream_t s) {
  constexpr int TPI = L / 32, E = FPHE_WAVE / TPI, NL = rad_ll(TPI) * TPI, PER = FPHE_WAVE / E, KB = 4 * PER;
  const size_t nwt = (ntiles_of(count) + 3) / 4, ntot = nwt * E;
  const size_t tab_words = nwt * KB * rad_ll(TPI) * FPHE_WAVE;
  const size_t tot_words = (size_t)ntiles_of(ntot) * L * FPHE_WAVE;
  u32* Tab = W;
  u32* Tot = Tab + tab_words;
  u32* Inv = Tot + tot_words;
  u32* X0 = Inv + tot_words;
  const size_t lds = (size_t)kWavesPerBlock * NL * E * 4;
  auto k1 = KS<TPI>::template binv_pre<L>();
  set_lds(k1, lds);
  const unsigned g1 = occ_grid(c, k1, lds, nwt, "binv_pre27");
  hipLaunchKernelGGL(k1, dim3(g1), dim3(kBlock), lds, s, c->K, Ca, count, need, Tab, Tot, (u32)NL);
  launch_inv27<L>(c, Tot, ntot, nullptr, Inv, err, X0, s);
  auto k2 = KS<TPI>::template binv_post<L>();
  set_lds(k2, lds);
  const unsigned g2 = occ_grid(c, k2, lds, nwt, "binv_post27");
  hipLaunchKernelGGL(k2, dim3(g2), dim3(kBlock), lds, s, c->K, Ca, count, need, Tab, Inv, Co, (u32)NL);
}

template <int L>
fphe_status launch_mul27(fphe_ctx* c, const uint32_t* Ca, const uint8_t* sa, const int32_t* ea, const uint32_t* P,
                         uint32_t lp, const uint8_t* pneg, const int32_t* pexp, int pstride, size_t count,
                         uint32_t* Co, uint8_t* so, int32_t* eo, int32_t* err, hipStream_t s) {
  (void)sa;  // powm results are canonical whatever the base's sign (lib.rs:334-349)
  constexpr int TPI = L / 32, E = FPHE_WAVE / TPI, NL = rad_ll(TPI) * TPI, L1 = L / 2;
  auto kern = KS<TPI>::template mul<L, kWinMul>();
  const size_t lds = (size_t)kWavesPerBlock * NL * E * 4;
  set_lds(kern, lds);
  // spans as for encrypt: plaintexts that are encoded negative ints take k-bit exponents
  const size_t span = span_elems(c, kern, lds, E);
  const size_t m0 = count < span ? count : span;
  const unsigned grid = occ_grid(c, kern, lds, (m0 + E - 1) / E, "mul27");
  // scratch: [window tables][need T*64 B][ebits T*64 i32][E T*L1*64 w][Cinv T*L*64 w][X0 T*L1*64 w]
  const size_t nt = ntiles_of(m0);
  const size_t tbytes = (size_t)grid * kWavesPerBlock * (1u << kWinMul) * rad_ll(TPI) * FPHE_WAVE * 4;
  const size_t o_need = tbytes, o_eb = o_need + nt * FPHE_WAVE, o_E = o_eb + nt * FPHE_WAVE * 4;
  const size_t o_inv = o_E + nt * L1 * FPHE_WAVE * 4, o_x0 = o_inv + nt * L * FPHE_WAVE * 4;
  const size_t x0b = nt * L1 * FPHE_WAVE * 4, binvb = m0 >= binv_min() ? binv_scratch_bytes<L>(m0) : 0;
  if (ensure_scratch(c, o_x0 + (binvb > x0b ? binvb : x0b), s) != FPHE_OK) return FPHE_ERR_HIP;
  char* base = reinterpret_cast<char*>(c->scratch);
  u8* need = reinterpret_cast<u8*>(base + o_need);
  int32_t* eb = reinterpret_cast<int32_t*>(base + o_eb);
  u32* Ex = reinterpret_cast<u32*>(base + o_E);
  u32* Cinv = reinterpret_cast<u32*>(base + o_inv);
  u32* X0 = reinterpret_cast<u32*>(base + o_x0);
  for (size_t e0 = 0; e0 < count; e0 += span) {
    const size_t m = count - e0 < span ? count - e0 : span, t0 = e0 / FPHE_WAVE;
    const uint32_t* Cs = Ca + t0 * L * FPHE_WAVE;
    const uint32_t* Ps = pstride ? P + t0 * lp * FPHE_WAVE : P;
    const uint8_t* ns = pstride ? pneg + e0 : pneg;
    const int32_t* xs = pstride ? pexp + e0 : pexp;
    const unsigned pgrid = (unsigned)std::min<size_t>((m + 255) / 256, (size_t)c->cus * 8);
    hipLaunchKernelGGL(k_mul_prep<L>, dim3(pgrid), dim3(256), 0, s, c->K, Ps, lp, ns, pstride, m, need, Ex, eb, err);
    if (m >= binv_min())
      launch_binv27<L>(c, Cs, m, need, Cinv, err, X0, s);
    else
      launch_inv27<L>(c, Cs, m, need, Cinv, err, X0, s);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kBlock), lds, s, c->K, Cs, Cinv, need, ea + e0, Ex, eb, xs, pstride, m,
                       Co + t0 * L * FPHE_WAVE, so + e0, eo + e0, c->scratch, (u32)NL);
    if (hipGetLastError() != hipSuccess) return FPHE_ERR_HIP;
  }
  return FPHE_OK;
}



// ---- wire format: bincode(serde(rug::Integer)) records (fate_utils pickles) ------------
// A reference Ciphertext / Plaintext serializes (bincode 1.3 fixint, little endian) as
//   i32 radix | u64 len | len ASCII chars ("-"? + digits, no leading zeros) | i32 exp
// (BInt is a newtype over rug::Integer, math/src/rug/mod.rs:11; rug's serde writes an
// Integer as the struct {radix, value}; pickles are bincode::serialize, paillier.rs:219-226).
// rug picks the radix per value: decimal when the magnitude has at most 32 significant bits,
// lowercase hex otherwise (rug 1.20 integer/serde.rs; unpinned).  mag is
// element-major LSF uint32 [count][L] (fphe_export_signed).
__device__ __forceinline__ u32 dec_digits(u32 w) {
  u32 d = 1;
  for (u64 p = 10; p <= w; p *= 10) ++d;
  return d;
}

// digits and radix of one magnitude
__device__ __forceinline__ u32 wire_digits(const u32* __restrict__ m, u32 L, u32& radix) {
  int k = (int)L - 1;
  while (k > 0 && m[k] == 0) --k;
  const u32 w = m[k];
  if (k == 0) {
    radix = 10;
    return dec_digits(w);
  }
  radix = 16;
  const u32 nib = (32u - (u32)__builtin_clz(w) + 3u) / 4u;
  return (u32)k * 8u + nib;
}

__global__ __launch_bounds__(256) void k_wire_lengths(const u32* __restrict__ mag, const u8* __restrict__ neg, u32 L,
                                                      size_t count, int64_t* __restrict__ rec_len,
                                                      u8* __restrict__ radix) {
  const size_t e = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= count) return;
  u32 rdx;
  const u32 nd = wire_digits(mag + e * L, L, rdx);
  rec_len[e] = 4 + 8 + 4 + (int64_t)(neg[e] ? 1 : 0) + (int64_t)nd;
  radix[e] = (u8)rdx;
}

// one thread per (element, 32-bit word): for a hex record the word's 8 nibbles are digit
// positions 8k .. 8k+7 from the least significant end; word 0's thread also writes the
// header, the sign and the exponent, and all digits of a decimal (<= 32-bit) record.
__global__ __launch_bounds__(256) void k_wire_encode(const u32* __restrict__ mag, const u8* __restrict__ neg,
                                                     const int32_t* __restrict__ exp, u32 L, size_t count,
                                                     const int64_t* __restrict__ rec_off,
                                                     const int64_t* __restrict__ rec_len, const u8* __restrict__ radix,
                                                     u8* __restrict__ out) {
  const size_t t = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= count * L) return;
  const size_t e = t / L;
  const u32 k = (u32)(t % L);
  const u32* m = mag + e * L;
  const u32 sg = neg[e] ? 1u : 0u;
  const u32 digits = (u32)(rec_len[e] - 16 - sg);
  const u32 rdx = radix[e];
  if (rdx == 10 && k != 0) return;
  if (rdx != 10 && 8u * k >= digits) return;
  u8* r = out + rec_off[e];
  u8* d = r + 12 + sg;
  if (k == 0) {
    const uint64_t len = digits + sg;
    r[0] = (u8)rdx; r[1] = 0; r[2] = 0; r[3] = 0;
    for (int b = 0; b < 8; ++b) r[4 + b] = (u8)(len >> (8 * b));
    if (sg) r[12] = '-';
    const u32 x = (u32)exp[e];
    u8* ex = r + 12 + sg + digits;
    for (int b = 0; b < 4; ++b) ex[b] = (u8)(x >> (8 * b));
    if (rdx == 10) {
      u32 w = m[0];
      for (u32 j = 0; j < digits; ++j) {
        d[digits - 1 - j] = (u8)('0' + w % 10u);
        w /= 10u;
      }
      return;
    }
  }
  const u32 w = m[k];
  for (u32 i = 0; i < 8; ++i) {
    const u32 j = 8u * k + i;
    if (j >= digits) break;
    const u32 nib = (w >> (4 * i)) & 15u;
    d[digits - 1 - j] = (u8)(nib < 10 ? '0' + nib : 'a' + nib - 10);
  }
}

// digit strings back to magnitude words (radix 16: one thread per word; radix 10 with at
// most 19 digits: word 0's thread writes words 0 and 1; other radixes are parsed on the
// host).  err bit 0: a character that is not a digit of the radix, bit 1: a value wider
// than L words.
__global__ __launch_bounds__(256) void k_wire_decode(const u8* __restrict__ buf, const int64_t* __restrict__ dig_off,
                                                     const int32_t* __restrict__ dig_len, const int32_t* __restrict__ radix,
                                                     u32 L, size_t count, u32* __restrict__ mag,
                                                     int32_t* __restrict__ err) {
  const size_t t = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= count * L) return;
  const size_t e = t / L;
  const u32 k = (u32)(t % L);
  const int64_t off = dig_off[e];
  const u32 len = (u32)dig_len[e];
  u32 bad = 0;
  if (radix[e] == 10) {
    if (k == 0) {
      u64 v = 0;
      for (u32 i = 0; i < len; ++i) {
        const u32 ch = buf[off + i];
        if (ch < '0' || ch > '9') { bad |= 1u; break; }
        v = v * 10u + (ch - '0');
      }
      mag[e * L] = (u32)v;
      if (L > 1) mag[e * L + 1] = (u32)(v >> 32);
      else if (v >> 32) bad |= 2u;
    } else if (k > 1) {
      mag[e * L + k] = 0;
    }
    if (bad) atomicOr(err, (int32_t)bad);
    return;
  }
  u32 w = 0;
  for (u32 i = 0; i < 8; ++i) {
    const u32 j = 8u * k + i;
    if (j >= len) break;
    const u32 ch = buf[off + len - 1 - j];
    u32 v;
    if (ch >= '0' && ch <= '9') v = ch - '0';
    else if (ch >= 'a' && ch <= 'f') v = ch - 'a' + 10;
    else if (ch >= 'A' && ch <= 'F') v = ch - 'A' + 10;
    else { v = 0; bad |= 1u; }
    w |= v << (4 * i);
  }
  mag[e * L + k] = w;
  if (k == L - 1) {  // digits past the top word must be zeros
    for (u32 j = 8u * L; j < len; ++j) {
      const u32 ch = buf[off + len - 1 - j];
      if (ch != '0') { bad |= 2u; break; }
    }
  }
  if (bad) atomicOr(err, (int32_t)bad);
}

// ---- element permutation of tile-major vectors (gather / scatter) ---------------------
// One thread per 32-bit word of the contiguous side, so that side is read or written fully
// coalesced; the indexed side follows idx (stable sorts and slices keep it mostly local).
// Indexes outside [0, nspace) are skipped; the host checks them before the call.
template <bool SCATTER>
__global__ __launch_bounds__(256) void k_permute(const u32* __restrict__ Cin, const u8* __restrict__ sin,
                                                 const int32_t* __restrict__ ein, u32 L,
                                                 const int64_t* __restrict__ idx, size_t count, size_t nspace,
                                                 u32* __restrict__ Cout, u8* __restrict__ sout,
                                                 int32_t* __restrict__ eout) {
  const size_t per_tile = (size_t)L * FPHE_WAVE;
  const size_t total = ((count + FPHE_WAVE - 1) / FPHE_WAVE) * per_tile;
  for (size_t o = (size_t)blockIdx.x * blockDim.x + threadIdx.x; o < total; o += (size_t)gridDim.x * blockDim.x) {
    const size_t tile = o / per_tile, rem = o - tile * per_tile;
    const u32 w = (u32)(rem >> 6), col = (u32)(rem & 63);
    const size_t i = tile * FPHE_WAVE + col;  // position on the contiguous side
    if (i >= count) continue;
    const int64_t j = idx[i];
    if (j < 0 || (size_t)j >= nspace) continue;
    const size_t oj = ((size_t)j >> 6) * per_tile + (size_t)w * FPHE_WAVE + ((size_t)j & 63);
    if (SCATTER) {
      if (Cin) Cout[oj] = Cin[o];
      if (w == 0) {
        if (sin) sout[j] = sin[i];
        if (ein) eout[j] = ein[i];
      }
    } else {
      if (Cin) Cout[o] = Cin[oj];
      if (w == 0) {
        if (sin) sout[i] = sin[j];
        if (ein) eout[i] = ein[j];
      }
    }
  }
}

// ---- (C, sign) <-> the reference's signed integers ------------------------------------
// The reference's ciphertext is the signed rug::Integer C - sign n^2 (canonical C, SURVEY.md
// §0 fact 1).  Export writes its magnitude as element-major LSF words and a negative flag;
// import is the inverse.  One thread per element; the tile-major side is coalesced.
__global__ __launch_bounds__(256) void k_export_signed(const u32* __restrict__ N2, u32 L, const u32* __restrict__ C,
                                                       const u8* __restrict__ sign, size_t count,
                                                       u32* __restrict__ mag, u8* __restrict__ neg) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= count) return;
  const u32* c = C + (e >> 6) * (size_t)L * FPHE_WAVE + (e & 63);
  u32* m = mag + e * L;
  u32 nz = 0;
  for (u32 w = 0; w < L; ++w) nz |= c[(size_t)w * FPHE_WAVE];
  const bool ng = sign[e] != 0 && nz != 0;
  u32 borrow = 0;
  for (u32 w = 0; w < L; ++w) {
    const u32 cw = c[(size_t)w * FPHE_WAVE];
    if (ng) {  // n^2 - C
      const u64 d = (u64)N2[w] - cw - borrow;
      m[w] = (u32)d;
      borrow = (u32)(d >> 63);
    } else {
      m[w] = cw;
    }
  }
  neg[e] = ng ? 1 : 0;
}

__global__ __launch_bounds__(256) void k_import_signed(const u32* __restrict__ N2, u32 L, const u32* __restrict__ mag,
                                                       const u8* __restrict__ neg, size_t count, u32* __restrict__ C,
                                                       u8* __restrict__ sign) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= count) return;
  u32* c = C + (e >> 6) * (size_t)L * FPHE_WAVE + (e & 63);
  const u32* m = mag + e * L;
  u32 nz = 0;
  for (u32 w = 0; w < L; ++w) nz |= m[w];
  const bool ng = neg[e] != 0 && nz != 0;
  u32 borrow = 0;
  for (u32 w = 0; w < L; ++w) {
    if (ng) {  // canonical n^2 - |c|
      const u64 d = (u64)N2[w] - m[w] - borrow;
      c[(size_t)w * FPHE_WAVE] = (u32)d;
      borrow = (u32)(d >> 63);
    } else {
      c[(size_t)w * FPHE_WAVE] = m[w];
    }
  }
  sign[e] = ng ? 1 : 0;
}
}  // namespace

extern "C" {

fphe_status fphe_ctx_create(int device, uint32_t key_bits, const uint32_t* n_w, const uint32_t* p_w,
                            const uint32_t* q_w, fphe_ctx** out) {
  if (!out || !n_w) return FPHE_ERR_ARG;
  // any even size up to 4096 bits (paillier/src/lib.rs:72-87 accepts any even size): the
  // kernels run the 1024-, 2048- or 4096-bit geometry with n zero-padded to it (R >= 4N
  // holds, so the lazy Montgomery bounds are unchanged).  Above 2048 bits n^2 spans 8 lanes
  // per element (TPI 8, 296 limbs of 28 bits) and n, p^2, q^2 the TPI-4 geometry.
  if (key_bits < 256 || key_bits > 4096 || key_bits % 2) return FPHE_ERR_ARG;
  if ((p_w == nullptr) != (q_w == nullptr)) return FPHE_ERR_ARG;
  const int L1 = key_bits <= 1024 ? 32 : (key_bits <= 2048 ? 64 : 128), L2 = 2 * L1, LQ = L1 / 2;
  try {
    Limbs n = from_words(n_w, L1);
    if (n.empty() || !(n[0] & 1)) return FPHE_ERR_KEY;
    if (hbn::bitlen(n) != key_bits) return FPHE_ERR_KEY;  // paillier/src/lib.rs:82 keeps bits(n)==k
    Limbs N2 = hbn::mul(n, n);
    std::vector<std::pair<const char*, Limbs>> arrays;
    std::vector<u32> blob;
    auto put = [&](const Limbs& v, size_t len) -> size_t {
      const size_t off = blob.size();
      Limbs p = hbn::padded(v, len);
      blob.insert(blob.end(), p.begin(), p.end());
      while (blob.size() % 4) blob.push_back(0);  // 16-byte aligned sections
      return off;
    };
    const size_t o_N2 = put(N2, L2);
    const size_t o_N2R2 = put(hbn::pow2_mod((size_t)64 * L2, N2), L2);
    const size_t o_N2R1 = put(hbn::pow2_mod((size_t)32 * L2, N2), L2);
    const size_t o_n = put(n, L1 + 1);
    const size_t o_nm1 = put(hbn::sub(n, Limbs{1}), L1);
    Limbs max_int = n;  // floor(n/2)
    for (size_t i = 0; i < max_int.size(); ++i)
      max_int[i] = (max_int[i] >> 1) | (i + 1 < max_int.size() ? max_int[i + 1] << 31 : 0);
    max_int = hbn::norm(max_int);
    const size_t o_max = put(max_int, L1);
    const size_t o_nmm = put(hbn::sub(n, max_int), L1);
    // engine limbs: n^2 at TPI2 = L2/32 lanes, n / p^2 / q^2 at TPIh = L2/64, each in the
    // radix of its engine (mont27_dev.h: 27 bits at TPI 4, 28 below); R = 2^(LB NL)
    const int TPI2 = L2 / 32, TPIh = L2 / 64;
    const int LB2 = rad_lb(TPI2), LBh = rad_lb(TPIh);
    const int NL2 = rad_ll(TPI2) * TPI2, NLh = rad_ll(TPIh) * TPIh;
    auto to27 = [](const Limbs& v, int nl, int lb) { return to_radix(v, nl, lb); };
    const size_t o_N2_27 = put(to27(N2, NL2, LB2), NL2);
    const size_t o_N2R1_27 = put(to27(hbn::pow2_mod((size_t)LB2 * NL2, N2), NL2, LB2), NL2);
    const size_t o_N2R2_27 = put(to27(hbn::pow2_mod((size_t)2 * LB2 * NL2, N2), NL2, LB2), NL2);
    const size_t o_N2R3_27 = put(to27(hbn::pow2_mod((size_t)3 * LB2 * NL2, N2), NL2, LB2), NL2);
    const size_t o_N2M1 = put(hbn::pow2_mod((size_t)LB2 * NL2, N2), L2);
    const size_t o_Nn_27 = put(to27(n, NLh, LBh), NLh);
    const size_t o_NnR1_27 = put(to27(hbn::pow2_mod((size_t)LBh * NLh, n), NLh, LBh), NLh);
    const size_t o_NnR2_27 = put(to27(hbn::pow2_mod((size_t)2 * LBh * NLh, n), NLh, LBh), NLh);
    size_t o_P2_27 = 0, o_P2R1_27 = 0, o_P2R2_27 = 0, o_Q2_27 = 0, o_Q2R1_27 = 0, o_Q2R2_27 = 0;
    size_t o_P2 = 0, o_P2R3 = 0, o_pm1 = 0, o_p = 0, o_pinv2 = 0, o_hpR = 0;
    size_t o_Q2 = 0, o_Q2R3 = 0, o_qm1 = 0, o_q = 0, o_qinv2 = 0, o_hqR = 0, o_pinvqR = 0;
    u32 p2n0 = 0, pn0 = 0, q2n0 = 0, qn0 = 0;
    int pm1b = 0, qm1b = 0, epb = 0, eqb = 0;
    size_t o_ep = 0, o_eq = 0, o_KpR = 0, o_KqR = 0, o_P2RX_27 = 0, o_Q2RX_27 = 0;
    size_t o_Ps = 0, o_PsR2 = 0, o_PsR3 = 0, o_Qs = 0, o_QsR2 = 0, o_QsR3 = 0, o_e1p = 0, o_e1q = 0;
    u32 ps_np = 0, qs_np = 0;
    int e1pb = 0, e1qb = 0, pb = 0, qb = 0;
    bool kh_direct = false;
    const bool has_sk = p_w != nullptr;
    if (has_sk) {
      Limbs p = from_words(p_w, LQ), q = from_words(q_w, LQ);
      if (hbn::cmp(p, q) == 0) return FPHE_ERR_KEY;
      if (hbn::cmp(p, q) > 0) std::swap(p, q);  // SK::new keeps p < q (paillier/src/lib.rs:127)
      if (hbn::cmp(hbn::mul(p, q), n) != 0) return FPHE_ERR_KEY;
      if (!(p[0] & 1) || !(q[0] & 1)) return FPHE_ERR_KEY;
      Limbs P2 = hbn::mul(p, p), Q2 = hbn::mul(q, q);
      Limbs pm1 = hbn::sub(p, Limbs{1}), qm1 = hbn::sub(q, Limbs{1});
      // h_p = ((g^(p-1) mod p^2 - 1)/p)^{-1} mod p with g = n+1 (paillier/src/lib.rs:131-137);
      // (1+n)^(p-1) = 1 + (p-1) n (mod p^2), so the L-value is (p-1) q mod p.
      auto hval = [&](const Limbs& s, const Limbs& t) {
        Limbs Lv = hbn::mod(hbn::mul(hbn::sub(s, Limbs{1}), t), s);
        return hbn::inv_mod(Lv, s);
      };
      Limbs hp = hval(p, q), hq = hval(q, p);
      Limbs pinvq = hbn::inv_mod(p, q);
      o_P2 = put(P2, L1);
      o_P2R3 = put(hbn::pow2_mod((size_t)96 * L1, P2), L1);
      o_pm1 = put(pm1, LQ + 1);
      o_p = put(p, LQ);
      o_pinv2 = put(hbn::inv_pow2(p, LQ), LQ);
      o_hpR = put(hbn::mod(hbn::mul(hp, hbn::pow2_mod((size_t)32 * LQ, p)), p), LQ);
      o_Q2 = put(Q2, L1);
      o_Q2R3 = put(hbn::pow2_mod((size_t)96 * L1, Q2), L1);
      o_qm1 = put(qm1, LQ + 1);
      o_q = put(q, LQ);
      o_qinv2 = put(hbn::inv_pow2(q, LQ), LQ);
      o_hqR = put(hbn::mod(hbn::mul(hq, hbn::pow2_mod((size_t)32 * LQ, q)), q), LQ);
      o_pinvqR = put(hbn::mod(hbn::mul(pinvq, hbn::pow2_mod((size_t)32 * LQ, q)), q), LQ);
      o_P2_27 = put(to27(P2, NLh, LBh), NLh);
      o_P2R1_27 = put(to27(hbn::pow2_mod((size_t)LBh * NLh, P2), NLh, LBh), NLh);
      o_P2R2_27 = put(to27(hbn::pow2_mod((size_t)2 * LBh * NLh, P2), NLh, LBh), NLh);
      o_Q2_27 = put(to27(Q2, NLh, LBh), NLh);
      o_Q2R1_27 = put(to27(hbn::pow2_mod((size_t)LBh * NLh, Q2), NLh, LBh), NLh);
      o_Q2R2_27 = put(to27(hbn::pow2_mod((size_t)2 * LBh * NLh, Q2), NLh, LBh), NLh);
      // R_s^2 R^-1 mod s^2 (R of n^2, R_s of s^2): mont_s(M(c) mod s^2, .) = c R_s
      auto rx = [&](const Limbs& S2) {
        const Limbs Rn = hbn::pow2_mod((size_t)LB2 * NL2, S2);
        return hbn::mod(hbn::mul(hbn::pow2_mod((size_t)2 * LBh * NLh, S2), hbn::inv_mod(Rn, S2)), S2);
      };
      o_P2RX_27 = put(to27(rx(P2), NLh, LBh), NLh);
      o_Q2RX_27 = put(to27(rx(Q2), NLh, LBh), NLh);
      p2n0 = hbn::neg_inv32(P2[0]); pn0 = hbn::neg_inv32(p[0]);
      q2n0 = hbn::neg_inv32(Q2[0]); qn0 = hbn::neg_inv32(q[0]);
      pm1b = (int)hbn::bitlen(pm1); qm1b = (int)hbn::bitlen(qm1);
      // CRT encryption constants
      Limbs ep = hbn::mod(n, hbn::mul(p, pm1)), eq = hbn::mod(n, hbn::mul(q, qm1));
      o_ep = put(ep, L1);
      o_eq = put(eq, L1);
      epb = (int)hbn::bitlen(ep); eqb = (int)hbn::bitlen(eq);
      {  // the split key-holder modexp's constants (KeyArgs)
        const int TPIs = L2 >= 128 ? L2 / 128 : 1, LBs = rad_lb(TPIs), NLs = rad_ll(TPIs) * TPIs;
        o_Ps = put(to27(p, NLs, LBs), NLs);
        o_PsR2 = put(to27(hbn::pow2_mod((size_t)2 * LBs * NLs, p), NLs, LBs), NLs);
        o_PsR3 = put(to27(hbn::pow2_mod((size_t)3 * LBs * NLs, p), NLs, LBs), NLs);
        o_Qs = put(to27(q, NLs, LBs), NLs);
        o_QsR2 = put(to27(hbn::pow2_mod((size_t)2 * LBs * NLs, q), NLs, LBs), NLs);
        o_QsR3 = put(to27(hbn::pow2_mod((size_t)3 * LBs * NLs, q), NLs, LBs), NLs);
        ps_np = hbn::neg_inv32(p[0]) & ((1u << LBs) - 1u);
        qs_np = hbn::neg_inv32(q[0]) & ((1u << LBs) - 1u);
        const Limbs e1p = hbn::mod(q, pm1), e1q = hbn::mod(p, qm1);
        o_e1p = put(e1p, LQ);
        o_e1q = put(e1q, LQ);
        e1pb = (int)hbn::bitlen(e1p); e1qb = (int)hbn::bitlen(e1q);
        pb = (int)hbn::bitlen(p); qb = (int)hbn::bitlen(q);
        // p, q prime: gcd(q, p - 1) = 1 iff q does not divide p - 1 (and likewise)
        kh_direct = !hbn::is_zero(hbn::mod(pm1, q)) && !hbn::is_zero(hbn::mod(qm1, p));
      }
      const Limbs R27 = hbn::pow2_mod((size_t)LB2 * NL2, N2);
      const Limbs Kp = hbn::mul(Q2, hbn::inv_mod(hbn::mod(Q2, P2), P2));  // < n^2
      const Limbs Kq = hbn::mul(P2, hbn::inv_mod(hbn::mod(P2, Q2), Q2));
      o_KpR = put(to27(hbn::mod(hbn::mul(Kp, R27), N2), NL2, LB2), NL2);
      o_KqR = put(to27(hbn::mod(hbn::mul(Kq, R27), N2), NL2, LB2), NL2);
    }
    auto* c = new fphe_ctx();
    c->device = device; c->key_bits = key_bits; c->L1 = L1; c->L2 = L2; c->LQ = LQ; c->has_sk = has_sk;
    c->kh_direct = has_sk && kh_direct;
    c->wide_decrypt_max = env_i64("FPHE_WIDE_DECRYPT_MAX", 4096);
    c->wide_encrypt_max = env_i64("FPHE_WIDE_ENCRYPT_MAX", 2048);
    c->wide_kh_encrypt_max = env_i64("FPHE_WIDE_KH_ENCRYPT_MAX", 4096);
    c->kh_direct_z = env_i64("FPHE_KH_DIRECT_Z", 1) != 0;
    DevGuard g(device);
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) { delete c; return FPHE_ERR_HIP; }
    c->cus = prop.multiProcessorCount;
    {
      // fphe_fold_segments takes its scratch from the device's default stream-ordered pool:
      // keep up to 24 GiB of it cached across calls (the default threshold of 0 hands every
      // block back to the driver at each synchronisation, and a 1-GiB re-map costs ms; a
      // 200M-term histogram over 20M source ciphertexts uses ~12 GiB, of 288 GiB of HBM)
      hipMemPool_t pool;
      if (hipDeviceGetDefaultMemPool(&pool, device) == hipSuccess) {
        uint64_t keep = (uint64_t)24 << 30;
        (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
      }
    }
    if (hipMalloc(&c->blob, blob.size() * 4) != hipSuccess) { delete c; return FPHE_ERR_HIP; }
    if (hipMemcpy(c->blob, blob.data(), blob.size() * 4, hipMemcpyHostToDevice) != hipSuccess) {
      (void)hipFree(c->blob); delete c; return FPHE_ERR_HIP;
    }
    u32* b = c->blob;
    KeyArgs& K = c->K;
    K.N2 = b + o_N2; K.N2_R2 = b + o_N2R2; K.N2_R1 = b + o_N2R1; K.n = b + o_n; K.nm1 = b + o_nm1;
    K.max_int = b + o_max; K.n_mm = b + o_nmm;
    K.n2_n0inv = hbn::neg_inv32(N2[0]);
    K.nbits = (int)key_bits;
    K.N2_27 = b + o_N2_27; K.N2R1_27 = b + o_N2R1_27; K.N2R2_27 = b + o_N2R2_27;
    K.n2_np27 = K.n2_n0inv & ((1u << LB2) - 1u);
    K.N2R3_27 = b + o_N2R3_27;
    K.N2M1 = b + o_N2M1;
    K.Nn_27 = b + o_Nn_27; K.NnR1_27 = b + o_NnR1_27; K.NnR2_27 = b + o_NnR2_27;
    K.nn_np27 = hbn::neg_inv32(n[0]) & ((1u << LBh) - 1u);
    K.nn_inv27 = (0u - hbn::neg_inv32(n[0])) & ((1u << LBh) - 1u);
    if (has_sk) {
      K.P2 = b + o_P2; K.P2_R3 = b + o_P2R3; K.pm1 = b + o_pm1; K.p = b + o_p; K.pinv2 = b + o_pinv2; K.hpR = b + o_hpR;
      K.Q2 = b + o_Q2; K.Q2_R3 = b + o_Q2R3; K.qm1 = b + o_qm1; K.q = b + o_q; K.qinv2 = b + o_qinv2; K.hqR = b + o_hqR;
      K.pinvqR = b + o_pinvqR;
      K.p2_n0inv = p2n0; K.p_n0inv = pn0; K.q2_n0inv = q2n0; K.q_n0inv = qn0;
      K.pm1_bits = pm1b; K.qm1_bits = qm1b;
      K.P2_27 = b + o_P2_27; K.P2R1_27 = b + o_P2R1_27; K.P2R2_27 = b + o_P2R2_27;
      K.Q2_27 = b + o_Q2_27; K.Q2R1_27 = b + o_Q2R1_27; K.Q2R2_27 = b + o_Q2R2_27;
      K.p2_np27 = p2n0 & ((1u << LBh) - 1u); K.q2_np27 = q2n0 & ((1u << LBh) - 1u);
      K.ep = b + o_ep; K.eq = b + o_eq; K.ep_bits = epb; K.eq_bits = eqb;
      K.KpR_27 = b + o_KpR; K.KqR_27 = b + o_KqR;
      K.P2RX_27 = b + o_P2RX_27; K.Q2RX_27 = b + o_Q2RX_27;
      K.Ps_27 = b + o_Ps; K.PsR2_27 = b + o_PsR2; K.PsR3_27 = b + o_PsR3;
      K.Qs_27 = b + o_Qs; K.QsR2_27 = b + o_QsR2; K.QsR3_27 = b + o_QsR3;
      K.ps_np27 = ps_np; K.qs_np27 = qs_np;
      K.e1p = b + o_e1p; K.e1q = b + o_e1q;
      K.e1p_bits = e1pb; K.e1q_bits = e1qb; K.p_bits = pb; K.q_bits = qb;
    }
    *out = c;
    return FPHE_OK;
  } catch (...) {
    return FPHE_ERR_KEY;
  }
}

fphe_status fphe_ctx_destroy(fphe_ctx* c) {
  if (!c) return FPHE_ERR_ARG;
  {
    DevGuard g(c->device);
    if (c->blob) (void)hipFree(c->blob);
    if (c->scratch) (void)hipFree(c->scratch);
    if (c->side) (void)hipStreamDestroy(c->side);
    if (c->ev_fork) (void)hipEventDestroy(c->ev_fork);
    if (c->ev_join) (void)hipEventDestroy(c->ev_join);
  }
  delete c;
  return FPHE_OK;
}

fphe_status fphe_ctx_set_option(fphe_ctx* c, int option, int64_t value) {
  if (!c) return FPHE_ERR_ARG;
  std::lock_guard<std::mutex> lk(c->mu);  // not while a call of this context is being queued
  switch (option) {
    case FPHE_OPT_WIDE_DECRYPT_MAX: c->wide_decrypt_max = value; return FPHE_OK;
    case FPHE_OPT_WIDE_ENCRYPT_MAX: c->wide_encrypt_max = value; return FPHE_OK;
    case FPHE_OPT_WIDE_KH_ENCRYPT_MAX: c->wide_kh_encrypt_max = value; return FPHE_OK;
    case FPHE_OPT_KH_DIRECT_Z: c->kh_direct_z = value != 0; return FPHE_OK;
    default: return FPHE_ERR_ARG;
  }
}

fphe_status fphe_ctx_get_option(fphe_ctx* c, int option, int64_t* value) {
  if (!c || !value) return FPHE_ERR_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  switch (option) {
    case FPHE_OPT_WIDE_DECRYPT_MAX: *value = c->wide_decrypt_max; return FPHE_OK;
    case FPHE_OPT_WIDE_ENCRYPT_MAX: *value = c->wide_encrypt_max; return FPHE_OK;
    case FPHE_OPT_WIDE_KH_ENCRYPT_MAX: *value = c->wide_kh_encrypt_max; return FPHE_OK;
    case FPHE_OPT_KH_DIRECT_Z: *value = (c->kh_direct && c->kh_direct_z) ? 1 : 0; return FPHE_OK;
    default: return FPHE_ERR_ARG;
  }
}

fphe_status fphe_ctx_limbs(const fphe_ctx* c, uint32_t* l2, uint32_t* l1) {
  if (!c) return FPHE_ERR_ARG;
  if (l2) *l2 = (uint32_t)c->L2;
  if (l1) *l1 = (uint32_t)c->L1;
  return FPHE_OK;
}

fphe_status fphe_encode_f32(const fphe_ctx* c, const float* x, size_t count, uint32_t* P, uint8_t* neg,
                            int32_t* exp, int32_t* err, void* stream) {
  if (!c || !err) return FPHE_ERR_ARG;
  if (count == 0) return FPHE_OK;
  if (!x || !P || !neg || !exp) return FPHE_ERR_ARG;
  DevGuard g(c->device);
  const unsigned grid = (unsigned)std::min<size_t>((count + 255) / 256, (size_t)c->cus * 8);
  hipLaunchKernelGGL(k_encode_f32, dim3(grid), dim3(256), 0, (hipStream_t)stream, x, count, P, neg, exp, err);
  return hip_ok(hipGetLastError());
}

fphe_status fphe_encode_f64(const fphe_ctx* c, const double* x, size_t count, uint32_t* P, uint8_t* neg,
                            int32_t* exp, int32_t* err, void* stream) {
  if (!c || !err) return FPHE_ERR_ARG;
  if (count == 0) return FPHE_OK;
  if (!x || !P || !neg || !exp) return FPHE_ERR_ARG;
  DevGuard g(c->device);
  const unsigned grid = (unsigned)std::min<size_t>((count + 255) / 256, (size_t)c->cus * 8);
  hipLaunchKernelGGL(k_encode_f64, dim3(grid), dim3(256), 0, (hipStream_t)stream, x, count, P, neg, exp, err);
  return hip_ok(hipGetLastError());
}

fphe_status fphe_decode_f32(const fphe_ctx* c, const uint32_t* P, uint32_t lp, const int32_t* exp, size_t count,
                            float* out, int32_t* err, void* stream) {
  if (!c || !err) return FPHE_ERR_ARG;
  if (count == 0) return FPHE_OK;
  if (!P || !exp || !out || lp == 0) return FPHE_ERR_ARG;
  DevGuard g(c->device);
  const unsigned grid = (unsigned)std::min<size_t>((count + 255) / 256, (size_t)c->cus * 8);
  if (c->L1 == 128)
    hipLaunchKernelGGL(k_decode_f32<128>, dim3(grid), dim3(256), 0, (hipStream_t)stream, c->K, P, lp, exp, count, out, err);
  else if (c->L1 == 64)
    hipLaunchKernelGGL(k_decode_f32<64>, dim3(grid), dim3(256), 0, (hipStream_t)stream, c->K, P, lp, exp, count, out, err);
  else
    hipLaunchKernelGGL(k_decode_f32<32>, dim3(grid), dim3(256), 0, (hipStream_t)stream, c->K, P, lp, exp, count, out, err);
  return hip_ok(hipGetLastError());
}

fphe_status fphe_decode_f64(const fphe_ctx* c, const uint32_t* P, uint32_t lp, const int32_t* exp, size_t count,
                            double* out, int32_t* err, void* stream) {
  if (!c || !err) return FPHE_ERR_ARG;
  if (count == 0) return FPHE_OK;
  if (!P || !exp || !out || lp == 0) return FPHE_ERR_ARG;
  DevGuard g(c->device);
  const unsigned grid = (unsigned)std::min<size_t>((count + 255) / 256, (size_t)c->cus * 8);
  if (c->L1 == 128)
    hipLaunchKernelGGL(k_decode_f64<128>, dim3(grid), dim3(256), 0, (hipStream_t)stream, c->K, P, lp, exp, count, out, err);
  else if (c->L1 == 64)
    hipLaunchKernelGGL(k_decode_f64<64>, dim3(grid), dim3(256), 0, (hipStream_t)stream, c->K, P, lp, exp, count, out, err);
  else
    hipLaunchKernelGGL(k_decode_f64<32>, dim3(grid), dim3(256), 0, (hipStream_t)stream, c->K, P, lp, exp, count, out, err);
  return hip_ok(hipGetLastError());
}


fphe_status fphe_encode_i64(const fphe_ctx* c, const int64_t* x, size_t count, uint32_t* P, uint8_t* neg,
                            int32_t* exp, void* stream) {
  if (!c) return FPHE_ERR_ARG;
  if (count == 0) return FPHE_OK;
  if (!x || !P || !neg || !exp) return FPHE_ERR_ARG;
  DevGuard g(c->device);
  const unsigned grid = (unsigned)std::min<size_t>((count + 255) / 256, (size_t)c->cus * 8);
  if (c->L1 == 128)
    hipLaunchKernelGGL(k_encode_i64<128>, dim3(grid), dim3(256), 0, (hipStream_t)stream, c->K, x, count, P, neg, exp);
  else if (c->L1 == 64)
    hipLaunchKernelGGL(k_encode_i64<64>, dim3(grid), dim3(256), 0, (hipStream_t)stream, c->K, x, count, P, neg, exp);
  else
    hipLaunchKernelGGL(k_encode_i64<32>, dim3(grid), dim3(256), 0, (hipStream_t)stream, c->K, x, count, P, neg, exp);
  return hip_ok(hipGetLastError());
}

fphe_status fphe_decode_i64(const fphe_ctx* c, const uint32_t* P, uint32_t lp, const int32_t* exp, size_t count,
                            int64_t* out, int32_t* err, void* stream) {
  if (!c || !err) return FPHE_ERR_ARG;
  if (count == 0) return FPHE_OK;
  if (!P || !exp || !out || lp == 0) return FPHE_ERR_ARG;
  DevGuard g(c->device);
  const unsigned grid = (unsigned)std::min<size_t>((count + 255) / 256, (size_t)c->cus * 8);
  if (c->L1 == 128)
    hipLaunchKernelGGL(k_decode_i64<128>, dim3(grid), dim3(256), 0, (hipStream_t)stream, c->K, P, lp, exp, count, out, err);
  else if (c->L1 == 64)
    hipLaunchKernelGGL(k_decode_i64<64>, dim3(grid), dim3(256), 0, (hipStream_t)stream, c->K, P, lp, exp, count, out, err);
  else
    hipLaunchKernelGGL(k_decode_i64<32>, dim3(grid), dim3(256), 0, (hipStream_t)stream, c->K, P, lp, exp, count, out, err);
  return hip_ok(hipGetLastError());
}

fphe_status fphe_decode_i32(const fphe_ctx* c, const uint32_t* P, uint32_t lp, const int32_t* exp, size_t count,
                            int32_t* out, int32_t* err, void* stream) {
  if (!c || !err) return FPHE_ERR_ARG;
  if (count == 0) return FPHE_OK;
  if (!P || !exp || !out || lp == 0) return FPHE_ERR_ARG;
  DevGuard g(c->device);
  const unsigned grid = (unsigned)std::min<size_t>((count + 255) / 256, (size_t)c->cus * 8);
  if (c->L1 == 128)
    hipLaunchKernelGGL(k_decode_i32<128>, dim3(grid), dim3(256), 0, (hipStream_t)stream, c->K, P, lp, exp, count, out, err);
  else if (c->L1 == 64)
    hipLaunchKernelGGL(k_decode_i32<64>, dim3(grid), dim3(256), 0, (hipStream_t)stream, c->K, P, lp, exp, count, out, err);
  else
    hipLaunchKernelGGL(k_decode_i32<32>, dim3(grid), dim3(256), 0, (hipStream_t)stream, c->K, P, lp, exp, count, out, err);
  return hip_ok(hipGetLastError());
}

fphe_status fphe_pack_f64(const fphe_ctx* c, const double* x, size_t count, uint32_t offset_bit, uint32_t pack_num,
                          uint32_t precision, uint32_t* P, uint8_t* neg, int32_t* exp, int32_t* err, void* stream) {
  if (!c || !err || pack_num == 0) return FPHE_ERR_ARG;
  if (count == 0) return FPHE_OK;
  if (!x || !P || !neg || !exp) return FPHE_ERR_ARG;
  if ((uint64_t)offset_bit * pack_num > (uint64_t)32 * c->L1 + offset_bit) return FPHE_ERR_ARG;
  DevGuard g(c->device);
  const size_t nout = (count + pack_num - 1) / pack_num;
  const unsigned grid = (unsigned)std::min<size_t>((nout + 63) / 64, (size_t)c->cus * 16);
  if (c->L1 == 128)
    hipLaunchKernelGGL(k_pack_f64<128>, dim3(grid), dim3(64), 0, (hipStream_t)stream, x, count, offset_bit, pack_num,
                       precision, nout, P, neg, exp, err);
  else if (c->L1 == 64)
    hipLaunchKernelGGL(k_pack_f64<64>, dim3(grid), dim3(64), 0, (hipStream_t)stream, x, count, offset_bit, pack_num,
                       precision, nout, P, neg, exp, err);
  else
    hipLaunchKernelGGL(k_pack_f64<32>, dim3(grid), dim3(64), 0, (hipStream_t)stream, x, count, offset_bit, pack_num,
                       precision, nout, P, neg, exp, err);
  return hip_ok(hipGetLastError());
}

fphe_status fphe_unpack_f64(const fphe_ctx* c, const uint32_t* P, uint32_t lp, size_t npacked, uint32_t offset_bit,
                            uint32_t pack_num, uint32_t precision, size_t total, double* out, void* stream) {
  if (!c || pack_num == 0 || offset_bit == 0 || offset_bit > 128) return FPHE_ERR_ARG;
  if (npacked == 0 || total == 0) return FPHE_OK;
  if (!P || !out || lp == 0) return FPHE_ERR_ARG;
  DevGuard g(c->device);
  const unsigned grid = (unsigned)std::min<size_t>((npacked + 255) / 256, (size_t)c->cus * 8);
  if (c->L1 == 128)
    hipLaunchKernelGGL(k_unpack_f64<128>, dim3(grid), dim3(256), 0, (hipStream_t)stream, P, lp, npacked, offset_bit,
                       pack_num, precision, total, out);
  else if (c->L1 == 64)
    hipLaunchKernelGGL(k_unpack_f64<64>, dim3(grid), dim3(256), 0, (hipStream_t)stream, P, lp, npacked, offset_bit,
                       pack_num, precision, total, out);
  else
    hipLaunchKernelGGL(k_unpack_f64<32>, dim3(grid), dim3(256), 0, (hipStream_t)stream, P, lp, npacked, offset_bit,
                       pack_num, precision, total, out);
  return hip_ok(hipGetLastError());
}

fphe_status fphe_encrypt(fphe_ctx* c, const uint32_t* P, uint32_t lp, const uint8_t* neg, size_t count, int obf,
                         const uint32_t* r, const uint32_t rng_key[8], uint64_t nonce, uint32_t* C, uint8_t* sign,
                         void* stream) {
  if (!c) return FPHE_ERR_ARG;
  if (count == 0) return FPHE_OK;
  if (!P || !neg || !C || !sign || lp == 0 || lp > (uint32_t)c->L1) return FPHE_ERR_ARG;
  if (count >= (1ull << 32)) return FPHE_ERR_ARG;
  if (obf && !r && !rng_key) return FPHE_ERR_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DevGuard g(c->device);
  if (c->L2 == 256)
    return launch_encrypt27<256>(c, P, lp, neg, count, obf, r, rng_key, nonce, C, sign, (hipStream_t)stream);
  if (c->L2 == 128)
    return launch_encrypt27<128>(c, P, lp, neg, count, obf, r, rng_key, nonce, C, sign, (hipStream_t)stream);
  return launch_encrypt27<64>(c, P, lp, neg, count, obf, r, rng_key, nonce, C, sign, (hipStream_t)stream);
}


fphe_status fphe_encrypt_crt(fphe_ctx* c, const uint32_t* P, uint32_t lp, const uint8_t* neg, size_t count,
                             const uint32_t* r, const uint32_t rng_key[8], uint64_t nonce, uint32_t* C,
                             uint8_t* sign, void* stream) {
  if (!c) return FPHE_ERR_ARG;
  if (!c->has_sk) return FPHE_ERR_NO_SK;
  if (count == 0) return FPHE_OK;
  if (!P || !neg || !C || !sign || lp == 0 || lp > (uint32_t)c->L1) return FPHE_ERR_ARG;
  if (count >= (1ull << 32)) return FPHE_ERR_ARG;
  if (!r && !rng_key) return FPHE_ERR_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DevGuard g(c->device);
  if (c->L2 == 256)
    return launch_encrypt_crt27<256>(c, P, lp, neg, count, r, rng_key, nonce, C, sign, (hipStream_t)stream);
  if (c->L2 == 128)
    return launch_encrypt_crt27<128>(c, P, lp, neg, count, r, rng_key, nonce, C, sign, (hipStream_t)stream);
  return launch_encrypt_crt27<64>(c, P, lp, neg, count, r, rng_key, nonce, C, sign, (hipStream_t)stream);
}


fphe_status fphe_fold(fphe_ctx* c, const uint32_t* Src, const uint8_t* ssign, const int32_t* sexp,
                      const int64_t* ord, const int64_t* cstart, const int32_t* clen, size_t nchunks,
                      uint32_t* Co, uint8_t* so, int32_t* eo, void* stream) {
  if (!c) return FPHE_ERR_ARG;
  if (nchunks == 0) return FPHE_OK;
  if (!Src || !ssign || !sexp || !ord || !cstart || !clen || !Co || !so || !eo) return FPHE_ERR_ARG;
  if (nchunks >= (1ull << 32)) return FPHE_ERR_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DevGuard g(c->device);
  if (c->L2 == 256)
    return launch_fold27<256>(c, Src, ssign, sexp, ord, cstart, clen, nchunks, Co, so, eo, (hipStream_t)stream);
  if (c->L2 == 128)
    return launch_fold27<128>(c, Src, ssign, sexp, ord, cstart, clen, nchunks, Co, so, eo, (hipStream_t)stream);
  return launch_fold27<64>(c, Src, ssign, sexp, ord, cstart, clen, nchunks, Co, so, eo, (hipStream_t)stream);
}


fphe_status fphe_fold_segments(fphe_ctx* c, const uint32_t* Src, const uint8_t* ssign, const int32_t* sexp,
                               size_t nsrc, const int32_t* idx, const int32_t* seg, size_t nterms, size_t nseg,
                               uint32_t* Co, uint8_t* so, int32_t* eo, uint8_t* present, int32_t* err, void* stream) {
  if (!c) return FPHE_ERR_ARG;
  if (nseg == 0) return nterms ? FPHE_ERR_ARG : FPHE_OK;
  if (!Co || !so || !eo || !err || (nterms && (!Src || !ssign || !sexp || !seg))) return FPHE_ERR_ARG;
  if (nterms >= (1ull << 31) || nsrc >= (1ull << 31) || nseg >= (1ull << 31)) return FPHE_ERR_ARG;
  if (nterms && !idx && nsrc < nterms) return FPHE_ERR_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DevGuard g(c->device);
  if (c->L2 == 256)
    return launch_fold_segments<256>(c, Src, ssign, sexp, nsrc, idx, seg, nterms, nseg, Co, so, eo, present, err,
                                     (hipStream_t)stream);
  if (c->L2 == 128)
    return launch_fold_segments<128>(c, Src, ssign, sexp, nsrc, idx, seg, nterms, nseg, Co, so, eo, present, err,
                                     (hipStream_t)stream);
  return launch_fold_segments<64>(c, Src, ssign, sexp, nsrc, idx, seg, nterms, nseg, Co, so, eo, present, err,
                                  (hipStream_t)stream);
}


fphe_status fphe_positions_terms(const void* positions, int pos_i64, size_t ns, size_t npos, int32_t stride,
                                 size_t nslots, int32_t* src, int32_t* slot, void* stream) {
  StreamDevGuard sdg(stream);
  if (stride < 1 || npos >= (1ull << 32)) return FPHE_ERR_ARG;
  const size_t npairs = ns * npos;
  if (npairs == 0) return FPHE_OK;
  if (!positions || !src || !slot) return FPHE_ERR_ARG;
  // every src and slot value fits int32 (fphe_fold_segments' widths): terms and samples
  if (npairs > ((1ull << 31) - 1) / (size_t)stride || ns > ((1ull << 31) - 1) / (size_t)stride ||
      nslots >= (1ull << 31))
    return FPHE_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  const int64_t lim = (int64_t)(nslots / (size_t)stride);
  const unsigned grid = (unsigned)std::min<size_t>((npairs + 255) / 256, 4096);
  if (pos_i64)
    hipLaunchKernelGGL(k_positions_terms<int64_t>, dim3(grid), dim3(256), 0, s, (const int64_t*)positions, npairs,
                       (uint32_t)npos, stride, lim, src, slot);
  else
    hipLaunchKernelGGL(k_positions_terms<int32_t>, dim3(grid), dim3(256), 0, s, (const int32_t*)positions, npairs,
                       (uint32_t)npos, stride, lim, src, slot);
  return hip_ok(hipGetLastError());
}

fphe_status fphe_decrypt(fphe_ctx* c, const uint32_t* C, size_t count, uint32_t* P, void* stream) {
  if (!c) return FPHE_ERR_ARG;
  if (!c->has_sk) return FPHE_ERR_NO_SK;
  if (count == 0) return FPHE_OK;
  if (!C || !P) return FPHE_ERR_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DevGuard g(c->device);
  if (c->L2 == 256) return launch_decrypt27<256>(c, C, count, P, (hipStream_t)stream);
  if (c->L2 == 128) return launch_decrypt27<128>(c, C, count, P, (hipStream_t)stream);
  return launch_decrypt27<64>(c, C, count, P, (hipStream_t)stream);
}


fphe_status fphe_add_ordered(fphe_ctx* c, const uint32_t* Ca, const uint8_t* sa, const int32_t* ea,
                             const uint32_t* Cb, const uint8_t* sb, const int32_t* eb, int b_stride, size_t count,
                             const int32_t* order, uint32_t* Co, uint8_t* so, int32_t* eo, int32_t* err,
                             void* stream) {
  if (!c) return FPHE_ERR_ARG;
  if (count == 0) return FPHE_OK;
  if (!Ca || !sa || !ea || !Cb || !sb || !eb || !Co || !so || !eo) return FPHE_ERR_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DevGuard g(c->device);
  if (c->L2 == 256)
    return launch_add27<256>(c, Ca, sa, ea, Cb, sb, eb, b_stride, count, order, Co, so, eo, err, (hipStream_t)stream);
  if (c->L2 == 128)
    return launch_add27<128>(c, Ca, sa, ea, Cb, sb, eb, b_stride, count, order, Co, so, eo, err, (hipStream_t)stream);
  return launch_add27<64>(c, Ca, sa, ea, Cb, sb, eb, b_stride, count, order, Co, so, eo, err, (hipStream_t)stream);
}

fphe_status fphe_add_order(const int32_t* ea, const int32_t* eb, size_t count, uint32_t L2, int32_t* order,
                           void* stream) {
  StreamDevGuard sdg(stream);
  if (count == 0) return FPHE_OK;
  if (!ea || !eb || !order || (L2 != 64 && L2 != 128 && L2 != 256)) return FPHE_ERR_ARG;
  if (count >= (1ull << 31)) return FPHE_ERR_ARG;
  static_assert(kAoRuns == (int)kAddRegions, "the order's runs are k_add27's XCD runs");
  hipStream_t s = (hipStream_t)stream;
  const size_t E = FPHE_WAVE / (L2 / 32), nwt = (count + E - 1) / E;
  const size_t run = (nwt + kAoRuns - 1) / kAoRuns * E;      // elements per run (whole wave tiles)
  const u32 nbr = (u32)((run + kAoBlock - 1) / kAoBlock);    // blocks per run
  const u32 nblk = (u32)kAoRuns * nbr;
  CallBufs B(s);
  int32_t* counts = B.get<int32_t>((size_t)nblk * kAoBins);
  int32_t* offsets = B.get<int32_t>((size_t)nblk * kAoBins);
  if (!B.ok) return FPHE_ERR_HIP;
  hipLaunchKernelGGL(k_ao_count, dim3(nblk), dim3(kGrBlock), 0, s, ea, eb, count, run, nbr, counts);
  hipLaunchKernelGGL(k_ao_scan, dim3(kAoRuns), dim3(kGrBlock), 0, s, counts, run, nbr, offsets);
  hipLaunchKernelGGL(k_ao_scatter, dim3(nblk), dim3(kGrBlock), 0, s, ea, eb, count, run, nbr, offsets, order);
  return hip_ok(hipGetLastError());
}

fphe_status fphe_add(fphe_ctx* c, const uint32_t* Ca, const uint8_t* sa, const int32_t* ea, const uint32_t* Cb,
                     const uint8_t* sb, const int32_t* eb, int b_stride, size_t count, uint32_t* Co, uint8_t* so,
                     int32_t* eo, int32_t* err, void* stream) {
  return fphe_add_ordered(c, Ca, sa, ea, Cb, sb, eb, b_stride, count, nullptr, Co, so, eo, err, stream);
}


fphe_status fphe_neg(fphe_ctx* c, const uint32_t* Ca, size_t count, uint32_t* Co, int32_t* err, void* stream) {
  if (!c || !err) return FPHE_ERR_ARG;
  if (count == 0) return FPHE_OK;
  if (!Ca || !Co) return FPHE_ERR_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DevGuard g(c->device);
  // large vectors: one inverse per group of 16 (8 at 1024 bits) elements (Montgomery's trick)
  if (count >= binv_min()) {
    const size_t w = c->L2 == 256 ? binv_scratch_bytes<256>(count)
                     : c->L2 == 128 ? binv_scratch_bytes<128>(count) : binv_scratch_bytes<64>(count);
    if (ensure_scratch(c, w, (hipStream_t)stream) != FPHE_OK) return FPHE_ERR_HIP;
    if (c->L2 == 256)
      launch_binv27<256>(c, Ca, count, nullptr, Co, err, c->scratch, (hipStream_t)stream);
    else if (c->L2 == 128)
      launch_binv27<128>(c, Ca, count, nullptr, Co, err, c->scratch, (hipStream_t)stream);
    else
      launch_binv27<64>(c, Ca, count, nullptr, Co, err, c->scratch, (hipStream_t)stream);
    return hip_ok(hipGetLastError());
  }
  const size_t xbytes = (size_t)ntiles_of(count) * c->L1 * FPHE_WAVE * 4;
  if (ensure_scratch(c, xbytes, (hipStream_t)stream) != FPHE_OK) return FPHE_ERR_HIP;
  if (c->L2 == 256) launch_inv27<256>(c, Ca, count, nullptr, Co, err, c->scratch, (hipStream_t)stream);
  else if (c->L2 == 128) launch_inv27<128>(c, Ca, count, nullptr, Co, err, c->scratch, (hipStream_t)stream);
  else launch_inv27<64>(c, Ca, count, nullptr, Co, err, c->scratch, (hipStream_t)stream);
  return hip_ok(hipGetLastError());
}


fphe_status fphe_sqmul(fphe_ctx* c, const uint32_t* Ca, const uint32_t* Cb, const uint8_t* sb, uint32_t nsq,
                       size_t count, uint32_t* Co, uint8_t* so, void* stream) {
  if (!c) return FPHE_ERR_ARG;
  if (count == 0) return FPHE_OK;
  if (!Ca || !Cb || !sb || !Co || !so || nsq > (1u << 20)) return FPHE_ERR_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DevGuard g(c->device);
  if (c->L2 == 256) return launch_sqmul27<256>(c, Ca, Cb, sb, (int)nsq, count, Co, so, (hipStream_t)stream);
  if (c->L2 == 128) return launch_sqmul27<128>(c, Ca, Cb, sb, (int)nsq, count, Co, so, (hipStream_t)stream);
  return launch_sqmul27<64>(c, Ca, Cb, sb, (int)nsq, count, Co, so, (hipStream_t)stream);
}


// pack_squeeze with one chunk per wave (wide_dev.h): for few chunks, where the throughput
// engine would run each squaring step as a launch of nearly empty waves
fphe_status fphe_pack_squeeze(fphe_ctx* c, const uint32_t* C, const uint8_t* sign, size_t count, uint32_t pack_num,
                              uint32_t shift_bit, uint32_t* Co, uint8_t* so, void* stream) {
  if (!c) return FPHE_ERR_ARG;
  if (count == 0) return FPHE_OK;
  if (!C || !sign || !Co || !so || pack_num == 0 || shift_bit > (1u << 20)) return FPHE_ERR_ARG;
  const size_t nch = (count + pack_num - 1) / pack_num;
  if (nch > (size_t)1 << 31) return FPHE_ERR_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DevGuard g(c->device);
  hipStream_t s = (hipStream_t)stream;
  if (c->L2 == 256)
    hipLaunchKernelGGL(k_squeeze_wide<256>, dim3((unsigned)nch), dim3(64), 0, s, c->K, C, sign, count, (int)pack_num,
                       (int)shift_bit, Co, so);
  else if (c->L2 == 128)
    hipLaunchKernelGGL(k_squeeze_wide<128>, dim3((unsigned)nch), dim3(64), 0, s, c->K, C, sign, count, (int)pack_num,
                       (int)shift_bit, Co, so);
  else
    hipLaunchKernelGGL(k_squeeze_wide<64>, dim3((unsigned)nch), dim3(64), 0, s, c->K, C, sign, count, (int)pack_num,
                       (int)shift_bit, Co, so);
  return hip_ok(hipGetLastError());
}

fphe_status fphe_align(fphe_ctx* c, const uint32_t* Ca, const uint8_t* sa, const int32_t* gap, size_t count,
                       uint32_t* Co, uint8_t* so, void* stream) {
  if (!c) return FPHE_ERR_ARG;
  if (count == 0) return FPHE_OK;
  if (!Ca || !sa || !gap || !Co || !so) return FPHE_ERR_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DevGuard g(c->device);
  if (c->L2 == 256) return launch_align27<256>(c, Ca, sa, gap, count, Co, so, (hipStream_t)stream);
  if (c->L2 == 128) return launch_align27<128>(c, Ca, sa, gap, count, Co, so, (hipStream_t)stream);
  return launch_align27<64>(c, Ca, sa, gap, count, Co, so, (hipStream_t)stream);
}


fphe_status fphe_mul(fphe_ctx* c, const uint32_t* Ca, const uint8_t* sa, const int32_t* ea, const uint32_t* P,
                     uint32_t lp, const uint8_t* pneg, const int32_t* pexp, int p_stride, size_t count, uint32_t* Co,
                     uint8_t* so, int32_t* eo, int32_t* err, void* stream) {
  if (!c || !err) return FPHE_ERR_ARG;
  if (count == 0) return FPHE_OK;
  if (!Ca || !sa || !ea || !P || !pneg || !pexp || !Co || !so || !eo || lp == 0) return FPHE_ERR_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DevGuard g(c->device);
  if (c->L2 == 256)
    return launch_mul27<256>(c, Ca, sa, ea, P, lp, pneg, pexp, p_stride, count, Co, so, eo, err, (hipStream_t)stream);
  if (c->L2 == 128)
    return launch_mul27<128>(c, Ca, sa, ea, P, lp, pneg, pexp, p_stride, count, Co, so, eo, err, (hipStream_t)stream);
  return launch_mul27<64>(c, Ca, sa, ea, P, lp, pneg, pexp, p_stride, count, Co, so, eo, err, (hipStream_t)stream);
}

fphe_status fphe_chacha20_blocks(const uint32_t key[8], uint32_t counter, const uint32_t nonce[3], size_t nblocks,
                                 uint32_t* out, void* stream) {
  StreamDevGuard sdg(stream);
  if (!key || !nonce || (nblocks && !out)) return FPHE_ERR_ARG;
  if (nblocks == 0) return FPHE_OK;
  ChaChaKey ck;
  for (int i = 0; i < 8; ++i) ck.k[i] = key[i];
  const unsigned grid = (unsigned)std::min<size_t>((nblocks + 255) / 256, 1024);
  hipLaunchKernelGGL(k_chacha_blocks, dim3(grid), dim3(256), 0, (hipStream_t)stream, ck, counter, nonce[0], nonce[1],
                     nonce[2], nblocks, out);
  return hip_ok(hipGetLastError());
}

fphe_status fphe_permute(const uint32_t* Cin, const uint8_t* sin, const int32_t* ein, uint32_t L,
                         const int64_t* idx, size_t count, size_t nspace, int scatter, uint32_t* Cout,
                         uint8_t* sout, int32_t* eout, void* stream) {
  StreamDevGuard sdg(stream);
  if (count == 0) return FPHE_OK;
  if (!idx || L == 0 || (Cin && !Cout) || (sin && !sout) || (ein && !eout)) return FPHE_ERR_ARG;
  const size_t words = ((count + FPHE_WAVE - 1) / FPHE_WAVE) * (size_t)L * FPHE_WAVE;
  const unsigned grid = (unsigned)std::min<size_t>((words + 255) / 256, (size_t)1 << 20);
  if (scatter)
    hipLaunchKernelGGL(k_permute<true>, dim3(grid), dim3(256), 0, (hipStream_t)stream, Cin, sin, ein, L, idx, count,
                       nspace, Cout, sout, eout);
  else
    hipLaunchKernelGGL(k_permute<false>, dim3(grid), dim3(256), 0, (hipStream_t)stream, Cin, sin, ein, L, idx, count,
                       nspace, Cout, sout, eout);
  return hipGetLastError() == hipSuccess ? FPHE_OK : FPHE_ERR_HIP;
}

fphe_status fphe_export_signed(fphe_ctx* c, const uint32_t* C, const uint8_t* sign, size_t count, uint32_t* mag,
                               uint8_t* neg, void* stream) {
  if (!c) return FPHE_ERR_ARG;
  if (count == 0) return FPHE_OK;
  if (!C || !sign || !mag || !neg) return FPHE_ERR_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DevGuard g(c->device);
  hipStream_t s = (hipStream_t)stream;
  // out of the Montgomery-resident form into a stream-ordered scratch of at most
  // kExportSpan elements, then the reference's signed integers, span by span: peak memory is
  // the vector, the magnitudes and ~0.5 GB (at 2048 bits), not a second copy of the vector
  // (config 5's 100M-element vectors are ~52 GB each)
  constexpr size_t kExportSpan = (size_t)1 << 20;  // whole tiles
  const size_t span = count < kExportSpan ? count : kExportSpan;
  CallBufs B(s);
  u32* plain = B.get<u32>((size_t)ntiles_of(span) * c->L2 * FPHE_WAVE);
  if (!B.ok) return FPHE_ERR_HIP;
  for (size_t e0 = 0; e0 < count; e0 += span) {
    const size_t m = count - e0 < span ? count - e0 : span;
    const uint32_t* Cs = C + (e0 / FPHE_WAVE) * c->L2 * FPHE_WAVE;
    fphe_status st = c->L2 == 256   ? launch_mont_const27<256>(c, Cs, m, nullptr, plain, s)
                     : c->L2 == 128 ? launch_mont_const27<128>(c, Cs, m, nullptr, plain, s)
                                    : launch_mont_const27<64>(c, Cs, m, nullptr, plain, s);
    if (st != FPHE_OK) return st;
    hipLaunchKernelGGL(k_export_signed, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, c->K.N2, (u32)c->L2,
                       plain, sign + e0, m, mag + e0 * c->L2, neg + e0);
    if (hipGetLastError() != hipSuccess) return FPHE_ERR_HIP;
  }
  return FPHE_OK;
}

fphe_status fphe_import_signed(fphe_ctx* c, const uint32_t* mag, const uint8_t* neg, size_t count, uint32_t* C,
                               uint8_t* sign, void* stream) {
  if (!c) return FPHE_ERR_ARG;
  if (count == 0) return FPHE_OK;
  if (!C || !sign || !mag || !neg) return FPHE_ERR_ARG;
  std::lock_guard<std::mutex> lk(c->mu);
  DevGuard g(c->device);
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(k_import_signed, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, s, c->K.N2, (u32)c->L2, mag,
                     neg, count, C, sign);
  // into the Montgomery-resident form, in place
  return c->L2 == 256   ? launch_mont_const27<256>(c, C, count, c->K.N2R2_27, C, s)
         : c->L2 == 128 ? launch_mont_const27<128>(c, C, count, c->K.N2R2_27, C, s)
                        : launch_mont_const27<64>(c, C, count, c->K.N2R2_27, C, s);
}

fphe_status fphe_ctx_mont_one(const fphe_ctx* c, uint32_t* one) {
  if (!c || !one) return FPHE_ERR_ARG;
  DevGuard g(c->device);
  return hip_ok(hipMemcpy(one, c->K.N2M1, (size_t)c->L2 * 4, hipMemcpyDeviceToHost));
}


// ---- (8) wire format (see k_wire_encode) ----------------------------------------------
fphe_status fphe_wire_lengths(const uint32_t* mag, const uint8_t* neg, uint32_t L, size_t count, int64_t* rec_len,
                              uint8_t* radix, void* stream) {
  StreamDevGuard sdg(stream);
  if (count == 0) return FPHE_OK;
  if (!mag || !neg || !rec_len || !radix || L == 0) return FPHE_ERR_ARG;
  hipLaunchKernelGGL(k_wire_lengths, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, (hipStream_t)stream, mag,
                     neg, L, count, rec_len, radix);
  return hip_ok(hipGetLastError());
}

fphe_status fphe_wire_encode(const uint32_t* mag, const uint8_t* neg, const int32_t* exp, uint32_t L, size_t count,
                             const int64_t* rec_off, const int64_t* rec_len, const uint8_t* radix, uint8_t* out,
                             void* stream) {
  StreamDevGuard sdg(stream);
  if (count == 0) return FPHE_OK;
  if (!mag || !neg || !exp || !rec_off || !rec_len || !radix || !out || L == 0) return FPHE_ERR_ARG;
  const size_t threads = count * L;
  hipLaunchKernelGGL(k_wire_encode, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, (hipStream_t)stream, mag,
                     neg, exp, L, count, rec_off, rec_len, radix, out);
  return hip_ok(hipGetLastError());
}

fphe_status fphe_wire_scan(const uint8_t* buf, size_t nbytes, size_t pos, size_t count, int64_t* dig_off,
                           int32_t* dig_len, uint8_t* neg, int32_t* exp, int32_t* radix, size_t* end) {
  if (!buf && nbytes) return FPHE_ERR_ARG;
  if (count && (!dig_off || !dig_len || !neg || !exp || !radix)) return FPHE_ERR_ARG;
  auto rd = [&](size_t at, int nb) {
    uint64_t v = 0;
    for (int b = 0; b < nb; ++b) v |= (uint64_t)buf[at + b] << (8 * b);
    return v;
  };
  for (size_t e = 0; e < count; ++e) {
    if (pos + 12 > nbytes) return FPHE_ERR_ARG;
    const int32_t rdx = (int32_t)(uint32_t)rd(pos, 4);
    const uint64_t len = rd(pos + 4, 8);
    pos += 12;
    if (rdx < 2 || rdx > 36 || len == 0 || len > nbytes - pos || nbytes - pos - len < 4) return FPHE_ERR_ARG;
    size_t d = pos, n = (size_t)len;
    uint8_t sg = 0;
    if (buf[d] == '-' || buf[d] == '+') {
      sg = buf[d] == '-';
      ++d;
      --n;
      if (n == 0) return FPHE_ERR_ARG;
    }
    if (n > INT32_MAX) return FPHE_ERR_ARG;
    dig_off[e] = (int64_t)d;
    dig_len[e] = (int32_t)n;
    neg[e] = sg;
    radix[e] = rdx;
    pos += (size_t)len;
    exp[e] = (int32_t)(uint32_t)rd(pos, 4);
    pos += 4;
  }
  if (end) *end = pos;
  return FPHE_OK;
}

fphe_status fphe_wire_decode(const uint8_t* buf, const int64_t* dig_off, const int32_t* dig_len, const int32_t* radix,
                             uint32_t L, size_t count, uint32_t* mag, int32_t* err, void* stream) {
  StreamDevGuard sdg(stream);
  if (count == 0) return FPHE_OK;
  if (!buf || !dig_off || !dig_len || !radix || !mag || !err || L == 0) return FPHE_ERR_ARG;
  const size_t threads = count * L;
  hipLaunchKernelGGL(k_wire_decode, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, (hipStream_t)stream, buf,
                     dig_off, dig_len, radix, L, count, mag, err);
  return hip_ok(hipGetLastError());
}

// Shader-clock stamps (diagnostics; bench.py's per-leg clock).  `blocks`
// one-wave workgroups; lane 0 of block b writes {its CU's place -- XCC id << 16 | the SE, SH
// and CU fields of HW_ID --, the shader-clock counter (clock64: s_memtime, counts SCLK
// cycles), the constant-rate counter (wall_clock64)} to out[3b .. 3b+2] with vector stores.
// The shader-clock counters of different CUs are not synchronised (a before/after pair from
// two CUs of one XCD can even run backwards), so the host pairs two stamps queued around a
// launch by CU; with a few thousand blocks every CU is stamped on both sides.
__global__ __launch_bounds__(64) void k_clock_stamp(unsigned long long* __restrict__ out) {
  if (threadIdx.x != 0) return;
  const unsigned long long c = clock64();
  const unsigned long long w = wall_clock64();
  const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 15u;   // HW_REG_XCC_ID
  const unsigned hw = __builtin_amdgcn_s_getreg((7 << 11) | (8 << 6) | 4) & 255u;    // HW_ID[15:8]
  out[3 * blockIdx.x] = (xcc << 16) | hw;
  out[3 * blockIdx.x + 1] = c;
  out[3 * blockIdx.x + 2] = w;
}

fphe_status fphe_clock_stamp(uint64_t* out, uint32_t blocks, uint32_t* wall_khz, void* stream) {
  StreamDevGuard sdg(stream);
  if (!out || blocks == 0 || blocks > 65536) return FPHE_ERR_ARG;
  if (wall_khz) {
    int dev = 0, khz = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess)
      return FPHE_ERR_HIP;
    *wall_khz = (uint32_t)khz;
  }
  hipLaunchKernelGGL(k_clock_stamp, dim3(blocks), dim3(64), 0, (hipStream_t)stream, (unsigned long long*)out);
  return hip_ok(hipGetLastError());
}

}  // extern "C"
