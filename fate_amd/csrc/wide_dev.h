// Latency-bound chains of Montgomery products: one element per wave.
//
// The throughput engine (mont_engine.inc) spreads an element over TPI adjacent lanes and
// fills a wave with 64 / TPI elements, so a launch that holds only a few elements -- the
// squaring chains of pack_squeeze (fixedpoint_paillier/src/lib.rs:439-450: acc^(2^shift) per
// packed value, 12 x 148 sequential squarings for config 4's 13-way squeeze), or the
// decryption of a handful of squeezed histograms or of a Hetero-LR gradient -- runs one
// nearly empty wave per chain at that wave's per-row latency (~22 us per 4096-bit squaring,
// ~20 us per 2048-bit product of a decrypt half).  Here one element spans a whole wave: lane
// l < NLANE holds the K = TPI limbs [K l, K l + K) (the same 28-bit limbs and the same
// R = 2^(LB NL) as the throughput engine of that modulus, so M-form values need no
// conversion), a row is K operand + K reduction MACs per lane, the row's multiplier comes
// from its lane by v_readlane, m from lane 0 by v_readfirstlane and two SALU ops, and the
// reduction word crosses lanes by one wavefront-wide DPP shift.  A row is ~16 instructions instead of ~72, so a chain runs
// several times faster; per element it issues ~2.3x the MACs of the throughput engine, so
// the launchers use it only when a call has few chains.
//
// Lanes NLANE..63 hold zero limbs (A = N = 0) and stay zero: their T never receives anything
// (the top lane keeps its carry, below), so no lane masks are needed in the rows.
#pragma once

namespace wide {

template <int TPI_>
struct Geo {
  static constexpr int TPI = TPI_;
  static constexpr int LB = fphe::rad_lb(TPI);
  static constexpr int NLANE = fphe::rad_ll(TPI);  // lanes holding limbs (37, or 38 at 27 bits)
  static constexpr int K = TPI;                    // limbs per lane
  static constexpr int NL = NLANE * K;             // the throughput engine's NL: same R
  static constexpr u32 MASK = (1u << LB) - 1u;
  // a slot takes <= 2 products < 2^(2 LB + 0.01) per row (operand, reduction): a carry sweep
  // after every GP groups of K rows (the rows of one lane's limbs of B) keeps it in 64 bits
  static constexpr int GP = ((1 << (64 - 2 * LB)) - 4) / 2 / K;
  static_assert(GP >= 1 && 2 * K * GP + 4 <= (1 << (64 - 2 * LB)), "rows between sweeps overflow a slot");
  static_assert(NLANE <= 64, "one element per wave");
};

__device__ __forceinline__ u64 wmads(u32 a, u32 b_uniform, u64 c) {  // a * b + c, b in an SGPR
  u64 d;
  asm("v_mad_u64_u32 %0, vcc, %1, %2, %3" : "=v"(d) : "v"(a), "s"(b_uniform), "v"(c) : "vcc");
  return d;
}

// lane i <- lane i + 1 (lane 63 <- 0) / lane i <- lane i - 1 (lane 0 <- 0): the GFX9
// wavefront-wide DPP shifts wave_shl:1 / wave_shr:1, which gfx950 executes
// (tools/probe/dpp_wave_probe.hip on MI355X, profiles/r05/r05e_dpp_wave_probe.txt): one
// instruction where row_shl:1 needed a v_readlane / v_writelane patch per 16-lane row end
__device__ __forceinline__ u32 from_next(u32 x) {
  return (u32)__builtin_amdgcn_update_dpp(0, (int)x, 0x130, 0xf, 0xf, true);
}
__device__ __forceinline__ u32 from_prev(u32 x) {
  return (u32)__builtin_amdgcn_update_dpp(0, (int)x, 0x138, 0xf, 0xf, true);
}
__device__ __forceinline__ u64 from_prev64(u64 x) {
  return ((u64)from_prev((u32)(x >> 32)) << 32) | from_prev((u32)x);
}

// CIOS row of A * B: T += A b (b = B's limb i, wave-uniform in an SGPR); m = T_0 n' mod 2^LB
// (lane 0's: its low word to an SGPR, then s_mul_i32 / s_and_b32); T = (T + m N) / 2^LB with
// the positions shifted down one limb: a lane's bottom word X keeps its high part (X >> LB
// stays at the new bottom) and hands X mod 2^LB to the lane below's top.
template <int TPI>
__device__ __forceinline__ void row(u64 (&T)[TPI], const u32 (&A)[TPI], u32 b, const u32 (&N)[TPI], u32 np) {
  using G = Geo<TPI>;
  constexpr int K = G::K;
  T[0] = wmads(A[0], b, T[0]);
  const u32 m = ((u32)__builtin_amdgcn_readfirstlane((int)(u32)T[0]) * np) & G::MASK;
#pragma unroll
  for (int k = 1; k < K; ++k) T[k] = wmads(A[k], b, T[k]);
  const u64 X = wmads(N[0], m, T[0]);
#pragma unroll
  for (int k = 1; k < K; ++k) T[k - 1] = wmads(N[k], m, T[k]);
  const u32 up = from_next((u32)X & G::MASK);
  if constexpr (K > 1) {
    T[K - 1] = up;
    T[0] += X >> G::LB;
  } else {
    T[0] = (u64)up + (X >> G::LB);
  }
}

// every slot keeps its low LB bits plus the high part of the slot below (value-preserving);
// the top lane's top slot keeps its high part (nothing above it), so the zero lanes stay zero
template <int TPI>
__device__ __forceinline__ void sweep(u64 (&T)[TPI], int lane) {
  using G = Geo<TPI>;
  constexpr int K = G::K;
  const bool top = lane == G::NLANE - 1;
  const u64 cin = from_prev64(top ? 0ull : (T[K - 1] >> G::LB));
  const u64 keep_top = top ? ~0ull : (u64)G::MASK;
  if constexpr (K > 1) {
    T[K - 1] = (T[K - 1] & keep_top) + (T[K - 2] >> G::LB);
#pragma unroll
    for (int j = K - 2; j >= 1; --j) T[j] = (T[j] & (u64)G::MASK) + (T[j - 1] >> G::LB);
    T[0] = (T[0] & (u64)G::MASK) + cin;
  } else {
    T[0] = (T[0] & keep_top) + cin;
  }
}

// T -> almost normalised limbs (< 2^LB + 2^10): carries within the lane, then the lane below's
// carry into the bottom limb and its overflow one limb up (the next lane's bottom when K = 1).
// The top lane's own carry is 0 (every value here is < R).
template <int TPI>
__device__ __forceinline__ void normalize(const u64 (&T)[TPI], u32 (&A)[TPI]) {
  using G = Geo<TPI>;
  constexpr int K = G::K;
  u64 c = 0;
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const u64 v = T[j] + c;
    A[j] = (u32)v & G::MASK;
    c = v >> G::LB;
  }
  const u64 v = (u64)A[0] + from_prev64(c);
  A[0] = (u32)v & G::MASK;
  if constexpr (K > 1) A[1] += (u32)(v >> G::LB);
  else A[0] += from_prev((u32)(v >> G::LB));
}

// A <- A * B * R^-1 mod N for any A, B < 2N (values < 4N against one < N also give < 2N).
// getb(l, k) returns the multiplier of row K l + k as a wave-uniform value; A is rewritten only
// at the end, so B may be A itself.
template <int TPI, class GetB>
__device__ __forceinline__ void mul(u32 (&A)[TPI], GetB getb, const u32 (&N)[TPI], u32 np, int lane) {
  using G = Geo<TPI>;
  constexpr int K = G::K;
  u64 T[K];
#pragma unroll
  for (int k = 0; k < K; ++k) T[k] = 0;
#pragma unroll 1
  for (int l = 0; l < G::NLANE; ++l) {
    if (l && l % G::GP == 0) sweep<TPI>(T, lane);  // wave-uniform
#pragma unroll
    for (int k = 0; k < K; ++k) row<TPI>(T, A, getb(l, k), N, np);
  }
  normalize<TPI>(T, A);
}
// B in registers: row K l + k's multiplier is lane l's limb k
template <int TPI>
__device__ __forceinline__ void mul_reg(u32 (&A)[TPI], const u32 (&B)[TPI], const u32 (&N)[TPI], u32 np, int lane) {
  mul<TPI>(A, [&](int l, int k) { return (u32)__builtin_amdgcn_readlane((int)B[k], l); }, N, np, lane);
}

// this lane's limbs of a constant held as NL limbs (e.g. R^2 mod N, the _27 key arrays)
template <int TPI>
__device__ __forceinline__ void const_limbs(const u32* __restrict__ c, u32 (&B)[TPI], int lane) {
#pragma unroll
  for (int k = 0; k < TPI; ++k) B[k] = lane < Geo<TPI>::NLANE ? c[TPI * lane + k] : 0u;
}

// This lane's limbs of the number whose bit 0 is bit `bit0` of element e of a tile-major
// [.][rows][64] u32 vector (exact limbs, zeros past the element's `rows` words).  The element
// is staged in the LDS word row wl (rows + 3 words).
template <int TPI>
__device__ __forceinline__ void load_limbs(const u32* __restrict__ C, u32 rows, size_t e, u32 bit0, u32* wl,
                                           u32 (&A)[TPI], int lane) {
  using G = Geo<TPI>;
  __syncthreads();
  const u32* src = C + (e >> 6) * (size_t)rows * 64 + (e & 63);
  for (u32 w = (u32)lane; w < rows + 3; w += 64) wl[w] = w < rows ? src[(size_t)w * 64] : 0u;
  __syncthreads();
#pragma unroll
  for (int k = 0; k < TPI; ++k) {
    u32 v = 0;
    if (lane < G::NLANE) {
      const u32 bit = bit0 + (u32)(G::LB * (TPI * lane + k)), w = bit >> 5, off = bit & 31;
      if (w + 1 < rows + 3) v = (u32)((((u64)wl[w + 1] << 32) | wl[w]) >> off) & G::MASK;
    }
    A[k] = v;
  }
}

// this lane's limbs of the number in the LDS word row wl (nwords words, then >= 2 zero words)
template <int TPI>
__device__ __forceinline__ void limbs_from_words(const u32* wl, u32 (&A)[TPI], int lane) {
  using G = Geo<TPI>;
#pragma unroll
  for (int k = 0; k < TPI; ++k) {
    u32 v = 0;
    if (lane < G::NLANE) {
      const u32 bit = (u32)(G::LB * (TPI * lane + k)), w = bit >> 5, off = bit & 31;
      v = (u32)((((u64)wl[w + 1] << 32) | wl[w]) >> off) & G::MASK;
    }
    A[k] = v;
  }
}

// this lane's limbs to an LDS row of NL limbs, and back
template <int TPI>
__device__ __forceinline__ void to_row(const u32 (&A)[TPI], u32* row_, int lane) {
  if (lane < Geo<TPI>::NLANE) {
#pragma unroll
    for (int k = 0; k < TPI; ++k) row_[TPI * lane + k] = A[k];
  }
}
template <int TPI>
__device__ __forceinline__ void from_row(const u32* row_, u32 (&A)[TPI], int lane) {
#pragma unroll
  for (int k = 0; k < TPI; ++k) A[k] = lane < Geo<TPI>::NLANE ? row_[TPI * lane + k] : 0u;
}

// A (< 2N) -> canonical residue, written as `nwords` words at rows [w0, w0 + nwords) of
// element e of a tile-major [.][rows][64] u32 vector.  The exact carry chain and the
// comparison with N run on lane 0 over the limbs in the LDS row bl (NL + 3 limbs), once per
// chain.
template <int TPI>
__device__ __forceinline__ void store_limbs(const u32 (&A)[TPI], u32* bl, const u32* __restrict__ Nl,
                                            u32* __restrict__ Co, u32 rows, size_t e, u32 w0, u32 nwords, int lane) {
  using G = Geo<TPI>;
  constexpr int NL = G::NL;
  __syncthreads();
  to_row<TPI>(A, bl, lane);
  __syncthreads();
  if (lane == 0) {
    u64 c = 0;
    for (int i = 0; i < NL; ++i) {
      const u64 v = (u64)bl[i] + c;
      bl[i] = (u32)v & G::MASK;
      c = v >> G::LB;
    }
    int cmp = 0;
    for (int i = NL - 1; i >= 0 && cmp == 0; --i) cmp = bl[i] > Nl[i] ? 1 : (bl[i] < Nl[i] ? -1 : 0);
    if (cmp >= 0) {
      int br = 0;
      for (int i = 0; i < NL; ++i) {
        const int v = (int)bl[i] - (int)Nl[i] + br;
        bl[i] = (u32)v & G::MASK;
        br = v >> G::LB;  // 0 or -1
      }
    }
    bl[NL] = bl[NL + 1] = bl[NL + 2] = 0;
  }
  __syncthreads();
  u32* dst = Co + (e >> 6) * (size_t)rows * 64 + (e & 63);
  for (u32 w = (u32)lane; w < nwords; w += 64) {
    const u32 bit = 32 * w, j = bit / G::LB, off = bit % G::LB;
    const u64 v = (u64)bl[j] | ((u64)bl[j + 1] << G::LB) | ((u64)bl[j + 2] << (2 * G::LB));
    dst[(size_t)(w0 + w) * 64] = (u32)(v >> off);
  }
}

// X^E for the wave-uniform exponent Ex (ebits bits), X = A in Montgomery form (< 2N): the
// throughput engine's sliding window (kernels_engine.inc powm27) with the odd powers
// X, X^3, ..., X^(2^W - 1) as LDS rows of NL limbs (tab, 2^(W-1) rows).
template <int TPI, int W>
__device__ __forceinline__ void powm(u32 (&A)[TPI], u32* tab, const u32 (&N)[TPI], u32 np, const u32* __restrict__ Ex,
                                     int ebits, int lane) {
  constexpr int NL = Geo<TPI>::NL;
  constexpr int kOdd = 1 << (W - 1);
  __syncthreads();
  to_row<TPI>(A, tab, lane);
  u32 X2[TPI];
#pragma unroll
  for (int k = 0; k < TPI; ++k) X2[k] = A[k];
  mul_reg<TPI>(X2, A, N, np, lane);  // X^2
#pragma unroll 1
  for (int k = 1; k < kOdd; ++k) {
    mul_reg<TPI>(A, X2, N, np, lane);  // X^(2k+1)
    to_row<TPI>(A, tab + k * NL, lane);
  }
  __syncthreads();
  auto bit = [&](int i) -> u32 { return (Ex[i >> 5] >> (i & 31)) & 1u; };
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
  from_row<TPI>(tab + (v >> 1) * NL, A, lane);
  i = j - 1;
#pragma unroll 1
  while (i >= 0) {
    int nsq = 0;
    while (i >= 0 && !bit(i)) {
      ++nsq;
      --i;
    }
    const bool mulw = i >= 0;
    if (mulw) {
      v = window(i, j);
      nsq += i - j + 1;
      i = j - 1;
    }
#pragma unroll 1
    for (int t = 0; t < nsq; ++t) mul_reg<TPI>(A, A, N, np, lane);
    if (mulw) {  // the table row into registers first: no LDS read on a row's critical path
      u32 Bt[TPI];
      from_row<TPI>(tab + (v >> 1) * NL, Bt, lane);
      mul_reg<TPI>(A, Bt, N, np, lane);
    }
  }
}

}  // namespace wide

// pack_squeeze (fixedpoint_paillier/src/lib.rs:439-450), one chunk per wave: acc = x_0 (its
// sign), then for each further y: acc = acc^(2^shift) (canonical: sign 0) * y (sign of y).
// M-form in, M-form out, exp 0 (set by the caller).
template <int L>
__global__ __launch_bounds__(64) void k_squeeze_wide(KeyArgs K, const u32* __restrict__ C, const u8* __restrict__ sign,
                                                     size_t count, int pack_num, int shift, u32* __restrict__ Co,
                                                     u8* __restrict__ so) {
  constexpr int TPI = L / 32;
  using G = wide::Geo<TPI>;
  __shared__ u32 wl[L + 3];
  __shared__ u32 bl[G::NL + 3];
  const int lane = (int)threadIdx.x;
  const size_t chunk = blockIdx.x;
  const size_t h = chunk * (size_t)pack_num;
  if (h >= count) return;  // block-uniform
  const int len = (int)(count - h < (size_t)pack_num ? count - h : (size_t)pack_num);
  u32 N[TPI];
  wide::const_limbs<TPI>(K.N2_27, N, lane);
  const u32 np = K.n2_np27;
  u32 A[TPI];
  wide::load_limbs<TPI>(C, L, h, 0, wl, A, lane);
  u8 sg = sign[h];
  for (int k = 1; k < len; ++k) {
    for (int t = 0; t < shift; ++t) wide::mul_reg<TPI>(A, A, N, np, lane);  // acc^(2^shift)
    u32 B[TPI];
    wide::load_limbs<TPI>(C, L, h + k, 0, wl, B, lane);
    wide::mul_reg<TPI>(A, B, N, np, lane);
    sg = sign[h + k];
  }
  wide::store_limbs<TPI>(A, bl, K.N2_27, Co, L, chunk, 0, L, lane);
  if (lane == 0) so[chunk] = sg;
}

// Decrypt's half-size modexps for few elements (k_pow_half27<L, W, false> of the throughput
// engine, same inputs and outputs): block 2e + h computes y_s = c^(s-1) mod s^2 for element
// e, s = p (h = 0) or q (h = 1) (paillier/src/lib.rs:174-176, the pow_mod of h_function), into
// Y[tile][2 L1][64] rows [h L1, h L1 + L1); k_decrypt_crt finishes.  The vector holds
// M(c) = c R_n mod n^2: with m_lo, m_hi the limbs of M(c) below and above s^2's R = 2^(LB NL),
// mont(m_lo, R mod s^2) + mont(m_hi, R^2 mod s^2) = M(c) mod s^2 (< 4N), and one product with
// R_s^2 R_n^-1 mod s^2 gives c R_s, the Montgomery form the modexp takes (as pow_half27).
template <int L, int W>
__global__ __launch_bounds__(64) void k_pow_half_wide(KeyArgs K, const u32* __restrict__ C, size_t count,
                                                      u32* __restrict__ Y) {
  constexpr int TPI = L / 64;  // p^2, q^2: 74 limbs on 37 lanes for 2048-bit keys, 37 for 1024
  using G = wide::Geo<TPI>;
  constexpr int NL = G::NL;
  constexpr u32 L1 = L / 2;
  __shared__ u32 wl[L + 3];
  __shared__ u32 bl[NL + 3];
  __shared__ u32 tab[(1 << (W - 1)) * NL];
  const int lane = (int)threadIdx.x;
  const size_t e = blockIdx.x >> 1;
  const bool hq = (blockIdx.x & 1) != 0;
  if (e >= count) return;  // block-uniform
  const u32* S2 = hq ? K.Q2_27 : K.P2_27;
  const u32 np = hq ? K.q2_np27 : K.p2_np27;
  u32 N[TPI], B[TPI], A[TPI], Cst[TPI];
  wide::const_limbs<TPI>(S2, N, lane);
  wide::load_limbs<TPI>(C, L, e, (u32)(G::LB * NL), wl, B, lane);  // m_hi
  wide::const_limbs<TPI>(hq ? K.Q2R2_27 : K.P2R2_27, Cst, lane);
  wide::mul_reg<TPI>(B, Cst, N, np, lane);
  wide::load_limbs<TPI>(C, L, e, 0, wl, A, lane);  // m_lo
  wide::const_limbs<TPI>(hq ? K.Q2R1_27 : K.P2R1_27, Cst, lane);
  wide::mul_reg<TPI>(A, Cst, N, np, lane);
  {
    u64 T[TPI];
#pragma unroll
    for (int k = 0; k < TPI; ++k) T[k] = (u64)A[k] + B[k];
    wide::normalize<TPI>(T, A);  // < 4N, only ever multiplied by R_s^2 R_n^-1 < N next
  }
  wide::const_limbs<TPI>(hq ? K.Q2RX_27 : K.P2RX_27, Cst, lane);
  wide::mul_reg<TPI>(A, Cst, N, np, lane);  // c R_s, < 2N
  wide::powm<TPI, W>(A, tab, N, np, hq ? K.qm1 : K.pm1, hq ? K.qm1_bits : K.pm1_bits, lane);
#pragma unroll
  for (int k = 0; k < TPI; ++k) Cst[k] = (lane == 0 && k == 0) ? 1u : 0u;
  wide::mul_reg<TPI>(A, Cst, N, np, lane);  // leave Montgomery form (< 2N)
  wide::store_limbs<TPI>(A, bl, S2, Y, 2 * L1, e, hq ? L1 : 0u, L1, lane);
}

// The key holder's half-size modexps for few elements (k_pow_half27<L, W, true, true> of the
// throughput engine, same inputs and outputs): block 2e + h raises element e's drawn z_s
// (k_draw_z: words [h ZW, h ZW + ZW) of Z[tile][2 ZW][64], z_s < s) to x_s = z_s^s mod s^2,
// canonical, into Y rows [h L1, h L1 + L1); k_encrypt_crt27 recombines.  The chain is decrypt's
// (a |s|-bit exponent mod s^2) without the c mod s^2 prologue.
template <int L, int W>
__global__ __launch_bounds__(64) void k_pow_half_enc_wide(KeyArgs K, const u32* __restrict__ Z, size_t count,
                                                          u32* __restrict__ Y) {
  constexpr int TPI = L / 64;
  using G = wide::Geo<TPI>;
  constexpr int NL = G::NL;
  constexpr u32 L1 = L / 2, ZW = 32u * (L >= 128 ? L / 128 : 1);  // kZWords<L>
  __shared__ u32 wl[L + 3];
  __shared__ u32 bl[NL + 3];
  __shared__ u32 tab[(1 << (W - 1)) * NL];
  const int lane = (int)threadIdx.x;
  const size_t e = blockIdx.x >> 1;
  const u32 h = blockIdx.x & 1u;
  if (e >= count) return;  // block-uniform
  const u32* S2 = h ? K.Q2_27 : K.P2_27;
  const u32 np = h ? K.q2_np27 : K.p2_np27;
  u32 N[TPI], A[TPI], Cst[TPI];
  wide::const_limbs<TPI>(S2, N, lane);
  // this half's ZW words only (the other half's follow them in the element's rows)
  __syncthreads();
  const u32* src = Z + (e >> 6) * (size_t)(2 * ZW) * 64 + (e & 63) + (size_t)h * ZW * 64;
  for (u32 w = (u32)lane; w < L + 3; w += 64) wl[w] = w < ZW ? src[(size_t)w * 64] : 0u;
  __syncthreads();
  wide::limbs_from_words<TPI>(wl, A, lane);
  wide::const_limbs<TPI>(h ? K.Q2R2_27 : K.P2R2_27, Cst, lane);
  wide::mul_reg<TPI>(A, Cst, N, np, lane);  // z R_s
  wide::powm<TPI, W>(A, tab, N, np, h ? K.q : K.p, h ? K.q_bits : K.p_bits, lane);
#pragma unroll
  for (int k = 0; k < TPI; ++k) Cst[k] = (lane == 0 && k == 0) ? 1u : 0u;
  wide::mul_reg<TPI>(A, Cst, N, np, lane);  // leave Montgomery form (< 2N)
  wide::store_limbs<TPI>(A, bl, S2, Y, 2 * L1, e, h ? L1 : 0u, L1, lane);
}

// Obfuscated public-key encryption of few elements (k_encrypt27 + k_mont_const27 of the
// throughput engine, same integers): one element per wave.  nude = 1 + m n mod n^2 with the
// sign of m (paillier/src/lib.rs:104-121, the truncating %; m > n/4 encodes a negative integer
// and 1 + m n is then the canonical inverse the reference takes), r^n by the sliding window
// from r R, and M(C) = mont(r^n R, nude R) = C R straight into the Montgomery-resident form.
// r: tile-major [.][L/2][64] (injected, or drawn by k_draw_r).
template <int L, int W>
__global__ __launch_bounds__(64) void k_encrypt_wide(KeyArgs K, const u32* __restrict__ P, u32 lp,
                                                     const u8* __restrict__ neg, size_t count,
                                                     const u32* __restrict__ R, u32* __restrict__ Co,
                                                     u8* __restrict__ so) {
  constexpr int TPI = L / 32;  // n^2: 148 limbs on 37 lanes for 2048-bit keys
  using G = wide::Geo<TPI>;
  constexpr int NL = G::NL;
  constexpr u32 L1 = L / 2;
  __shared__ u32 wl[L + 3];
  __shared__ u32 bl[NL + 3];
  __shared__ u32 tab[(1 << (W - 1)) * NL];
  __shared__ u32 mneg_s;
  const int lane = (int)threadIdx.x;
  const size_t e = blockIdx.x;
  if (e >= count) return;  // block-uniform
  u32 N[TPI], A[TPI], Nd[TPI], Cst[TPI];
  wide::const_limbs<TPI>(K.N2_27, N, lane);
  const u32 np = K.n2_np27;
  // the nude ciphertext in 32-bit words (as nude_to_slot), on lane 0
  for (u32 w = (u32)lane; w < L + 3; w += 64) wl[w] = 0u;
  __syncthreads();
  if (lane == 0) {
    const u32* pe = P + (e >> 6) * (size_t)lp * 64 + (e & 63);
    u32 any = 0;
    for (u32 k = 0; k < lp; ++k) {
      const u32 pk = pe[(size_t)k * 64];
      any |= pk;
      u64 acc = 0;
      for (u32 j = 0; j < L1; ++j) {
        acc = (u64)pk * K.n[j] + wl[k + j] + (acc >> 32);
        wl[k + j] = (u32)acc;
      }
      wl[k + L1] = (u32)(acc >> 32);
    }
    const bool mneg = neg[e] != 0 && any != 0;
    if (mneg) {  // n^2 - |m| n
      u32 br = 0;
      for (u32 j = 0; j < L; ++j) {
        const u64 d = (u64)K.N2[j] - wl[j] - br;
        wl[j] = (u32)d;
        br = (u32)(d >> 63);
      }
    }
    u32 c = 1;  // + 1
    for (u32 j = 0; j < L && c; ++j) {
      const u64 t = (u64)wl[j] + c;
      wl[j] = (u32)t;
      c = (u32)(t >> 32);
    }
    mneg_s = mneg ? 1u : 0u;
  }
  __syncthreads();
  wide::limbs_from_words<TPI>(wl, Nd, lane);
  wide::load_limbs<TPI>(R, L1, e, 0, wl, A, lane);  // r < n
  wide::const_limbs<TPI>(K.N2R2_27, Cst, lane);
  wide::mul_reg<TPI>(A, Cst, N, np, lane);   // r R
  wide::mul_reg<TPI>(Nd, Cst, N, np, lane);  // nude R
  wide::powm<TPI, W>(A, tab, N, np, K.n, K.nbits, lane);  // r^n R
  wide::mul_reg<TPI>(A, Nd, N, np, lane);    // r^n nude R = M(C), < 2N
  wide::store_limbs<TPI>(A, bl, K.N2_27, Co, L, e, 0, L, lane);
  if (lane == 0) so[e] = (u8)mneg_s;
}
