// Latency-bound chains of Montgomery products: one element per wave.
//
// The throughput engine (mont_engine.inc) spreads an element over TPI adjacent lanes and
// fills a wave with 64 / TPI elements, so a launch that holds only a few elements -- the
// squaring chains of pack_squeeze (fixedpoint_paillier/src/lib.rs:439-450: acc^(2^shift) per
// packed value, 12 x 148 sequential squarings for config 4's 13-way squeeze) -- runs one
// nearly empty wave per chain at that wave's per-row latency (~22 us per 4096-bit squaring).
// Here one element spans a whole wave: lane l < NLANE holds the K = TPI limbs [K l, K l + K)
// (the same 28-bit limbs and the same R = 2^(LB NL) as the throughput engine, so M-form
// vectors need no conversion), a row is K operand + K reduction MACs per lane, the row's
// multiplier comes from its lane by v_readlane, m from lane 0 by v_readfirstlane and two SALU
// ops, and the reduction word crosses lanes by one wavefront-wide DPP shift.  A row is ~16
// instructions instead of ~72, so a chain runs several times faster; per element it issues
// ~2.3x the MACs of the throughput engine, so the launchers use it only when a call has few
// chains.
//
// Lanes NLANE..63 hold zero limbs (A = N = 0) and stay zero: their T never receives anything
// (the top lane keeps its carry, below), so no lane masks are needed in the rows.
#pragma once

namespace wide {

template <int L>
struct Geo {
  static constexpr int TPI = L / 32;
  static constexpr int LB = fphe::rad_lb(TPI);
  static constexpr int NLANE = fphe::rad_ll(TPI);  // lanes holding limbs (37, or 38 at 27 bits)
  static constexpr int K = TPI;                    // limbs per lane
  static constexpr int NL = NLANE * K;             // the throughput engine's NL: same R
  static constexpr u32 MASK = (1u << LB) - 1u;
  // LDS words an element's number is read through: every limb's two words exist (zeros past L)
  static constexpr int WL = (NL * LB) / 32 + 3;
  // a slot takes <= 2 products < 2^(2 LB + 0.01) per row (operand, reduction): a carry sweep
  // after every GP groups of K rows (the rows of one lane's limbs of B) keeps it in 64 bits
  static constexpr int GP = ((1 << (64 - 2 * LB)) - 4) / 2 / K;
  static_assert(GP >= 1 && 2 * K * GP + 4 <= (1 << (64 - 2 * LB)), "rows between sweeps overflow a slot");
  static_assert(NLANE <= 64, "one element per wave");
};

__device__ __forceinline__ u64 wmad(u32 a, u32 b, u64 c) {  // a * b + c, b in a VGPR
  u64 d;
  asm("v_mad_u64_u32 %0, vcc, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c) : "vcc");
  return d;
}
__device__ __forceinline__ u64 wmads(u32 a, u32 b_uniform, u64 c) {  // b in an SGPR
  u64 d;
  asm("v_mad_u64_u32 %0, vcc, %1, %2, %3" : "=v"(d) : "v"(a), "s"(b_uniform), "v"(c) : "vcc");
  return d;
}

// lane i <- lane i + 1 (lane 63 <- 0) / lane i <- lane i - 1 (lane 0 <- 0): the GFX9
// wavefront-wide DPP shifts wave_shl:1 / wave_shr:1, which gfx950 executes
// (tools/probe/dpp_wave_probe.hip on MI355X, profiles/r05/r05e_dpp_wave_probe.txt): one
// instruction where row_shl:1 needed a v_readlane / v_writelane patch per 16-lane row end
template <int NLANE>
__device__ __forceinline__ u32 from_next(u32 x) {
  return (u32)__builtin_amdgcn_update_dpp(0, (int)x, 0x130, 0xf, 0xf, true);
}
template <int NLANE>
__device__ __forceinline__ u32 from_prev(u32 x) {
  return (u32)__builtin_amdgcn_update_dpp(0, (int)x, 0x138, 0xf, 0xf, true);
}
template <int NLANE>
__device__ __forceinline__ u64 from_prev64(u64 x) {
  return ((u64)from_prev<NLANE>((u32)(x >> 32)) << 32) | from_prev<NLANE>((u32)x);
}

// CIOS row i of A * B: T += A b (b = B's limb i, wave-uniform in an SGPR); m = T_0 n' mod 2^LB
// (lane 0's, broadcast through an SGPR);
// T = (T + m N) / 2^LB with the positions shifted down one limb: a lane's bottom word X keeps
// its high part (X >> LB stays at the new bottom) and hands X mod 2^LB to the lane below's top.
template <int L>
__device__ __forceinline__ void row(u64 (&T)[Geo<L>::K], const u32 (&A)[Geo<L>::K], u32 b, const u32 (&N)[Geo<L>::K],
                                    u32 np) {
  using G = Geo<L>;
  constexpr int K = G::K;
  T[0] = wmads(A[0], b, T[0]);
  // m on the scalar unit: lane 0's low word to an SGPR, then s_mul_i32 / s_and_b32
  const u32 m = ((u32)__builtin_amdgcn_readfirstlane((int)(u32)T[0]) * np) & G::MASK;
#pragma unroll
  for (int k = 1; k < K; ++k) T[k] = wmads(A[k], b, T[k]);
  const u64 X = wmads(N[0], m, T[0]);
#pragma unroll
  for (int k = 1; k < K; ++k) T[k - 1] = wmads(N[k], m, T[k]);
  const u32 up = from_next<G::NLANE>((u32)X & G::MASK);
  if constexpr (K > 1) {
    T[K - 1] = up;
    T[0] += X >> G::LB;
  } else {
    T[0] = (u64)up + (X >> G::LB);
  }
}

// every slot keeps its low LB bits plus the high part of the slot below (value-preserving);
// the top lane's top slot keeps its high part (nothing above it), so the zero lanes stay zero
template <int L>
__device__ __forceinline__ void sweep(u64 (&T)[Geo<L>::K], int lane) {
  using G = Geo<L>;
  constexpr int K = G::K;
  const bool top = lane == G::NLANE - 1;
  const u64 cin = from_prev64<G::NLANE>(top ? 0ull : (T[K - 1] >> G::LB));
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

// T -> almost normalised limbs: carries within the lane, then the lane below's carry into the
// bottom limb (and its overflow into limb 1).  The top lane's own carry is 0 (value < 2N < R).
template <int L>
__device__ __forceinline__ void normalize(const u64 (&T)[Geo<L>::K], u32 (&A)[Geo<L>::K]) {
  using G = Geo<L>;
  constexpr int K = G::K;
  static_assert(K >= 2, "one element per wave needs >= 2 limbs per lane");
  u64 c = 0;
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const u64 v = T[j] + c;
    A[j] = (u32)v & G::MASK;
    c = v >> G::LB;
  }
  const u64 v = (u64)A[0] + from_prev64<G::NLANE>(c);
  A[0] = (u32)v & G::MASK;
  A[1] += (u32)(v >> G::LB);
}

// A <- A * B * R^-1 mod N (B may be A itself: A is rewritten only at the end).  Row i's
// multiplier b_i = B's limb i is read from lane i / K with v_readlane (rows unrolled by K)
template <int L>
__device__ __forceinline__ void mul(u32 (&A)[Geo<L>::K], const u32 (&B)[Geo<L>::K], const u32 (&N)[Geo<L>::K], u32 np,
                                    int lane) {
  using G = Geo<L>;
  constexpr int K = G::K;
  u64 T[K];
#pragma unroll
  for (int k = 0; k < K; ++k) T[k] = 0;
#pragma unroll 1
  for (int l = 0; l < G::NLANE; ++l) {
    if (l && l % G::GP == 0) sweep<L>(T, lane);  // wave-uniform
#pragma unroll
    for (int k = 0; k < K; ++k) row<L>(T, A, (u32)__builtin_amdgcn_readlane((int)B[k], l), N, np);
  }
  normalize<L>(T, A);
}

// the element's limbs into the LDS row the products read (each lane its K)
template <int L>
__device__ __forceinline__ void to_lds(const u32 (&A)[Geo<L>::K], u32* bl, int lane) {
  using G = Geo<L>;
  __syncthreads();  // earlier readers of bl are done
  if (lane < G::NLANE) {
#pragma unroll
    for (int k = 0; k < G::K; ++k) bl[G::K * lane + k] = A[k];
  }
  __syncthreads();
}

// element e of a tile-major [.][L][64] vector -> this lane's limbs (exact), through the LDS
// word row wl (G::WL words; those past the number's L stay 0)
template <int L>
__device__ __forceinline__ void load_elem(const u32* __restrict__ C, size_t e, u32* wl, u32 (&A)[Geo<L>::K], int lane) {
  using G = Geo<L>;
  __syncthreads();
  const u32* src = C + (e >> 6) * (size_t)L * 64 + (e & 63);
  for (int w = lane; w < G::WL; w += 64) wl[w] = w < L ? src[(size_t)w * 64] : 0u;
  __syncthreads();
#pragma unroll
  for (int k = 0; k < G::K; ++k) {
    const int j = G::K * lane + k;
    u32 v = 0;
    if (lane < G::NLANE) {
      const int bit = G::LB * j, w = bit >> 5, off = bit & 31;
      v = (u32)((((u64)wl[w + 1] << 32) | wl[w]) >> off) & G::MASK;
    }
    A[k] = v;
  }
}

// A (< 2N) -> canonical residue, written as element e of a tile-major vector.  The exact
// carry chain and the comparison with N run on lane 0 over the limbs in LDS (once per chain).
template <int L>
__device__ __forceinline__ void store_elem(const u32 (&A)[Geo<L>::K], u32* bl, const u32* __restrict__ Nl, u32* __restrict__ Co,
                                           size_t e, int lane) {
  using G = Geo<L>;
  constexpr int NL = G::NL;
  to_lds<L>(A, bl, lane);
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
  u32* dst = Co + (e >> 6) * (size_t)L * 64 + (e & 63);
  for (int w = lane; w < L; w += 64) {
    const int bit = 32 * w, j = bit / G::LB, off = bit % G::LB;
    const u64 v = (u64)bl[j] | ((u64)bl[j + 1] << G::LB) | ((u64)bl[j + 2] << (2 * G::LB));
    dst[(size_t)w * 64] = (u32)(v >> off);
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
  using G = wide::Geo<L>;
  __shared__ u32 wl[G::WL];
  __shared__ u32 bl[G::NL + 3];
  const int lane = (int)threadIdx.x;
  const size_t chunk = blockIdx.x;
  const size_t h = chunk * (size_t)pack_num;
  if (h >= count) return;  // block-uniform
  const int len = (int)(count - h < (size_t)pack_num ? count - h : (size_t)pack_num);
  u32 N[G::K];
#pragma unroll
  for (int k = 0; k < G::K; ++k) N[k] = lane < G::NLANE ? K.N2_27[G::K * lane + k] : 0u;
  const u32 np = K.n2_np27;
  u32 A[G::K];
  wide::load_elem<L>(C, h, wl, A, lane);
  u8 sg = sign[h];
  for (int k = 1; k < len; ++k) {
    for (int t = 0; t < shift; ++t) wide::mul<L>(A, A, N, np, lane);  // acc^(2^shift)
    u32 B[G::K];
    wide::load_elem<L>(C, h + k, wl, B, lane);
    wide::mul<L>(A, B, N, np, lane);
    sg = sign[h + k];
  }
  wide::store_elem<L>(A, bl, K.N2_27, Co, chunk, lane);
  if (lane == 0) so[chunk] = sg;
}
