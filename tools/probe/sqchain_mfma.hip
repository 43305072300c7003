// Probe (round-3 prep, not part of libfatephe): a 4096-bit Montgomery squaring whose
// reduction runs on the i8 matrix cores, built INTO the engine's TPI-4 layout, against the
// engine's own VALU squaring (fate_amd/csrc/mont_engine.inc sqr<4>) on the same inputs.
//
// One wave = 16 elements.  Phase A (VALU, TPI-4 layout, lane = 4e + q): the half-product
// squaring rows of mont_sqr WITHOUT the reduction MACs (19 mads per row instead of 56).  The
// frame still shifts one limb per row; the limb leaving the element's bottom slot is final
// (no later row adds to it) and lane q = 0 writes it into the LDS slot the row just consumed,
// so after 148 rows the slots hold T_low (148 exact 28-bit limbs) and the accumulators hold
// T_high (64-bit column sums).
// Phase B (MFMA layout, lane = 16g + c: element c, k/row group g), R = 2^4144 = 128^592:
//   q = T_low * N' mod R   37 output tiles of 16 base-128 digits, v_mfma_i32_16x16x64_i8 with
//                          Toeplitz(N') A fragments read from one 10 KB LDS table (W1) and the
//                          T_low digits as B fragments (10 K-tiles, built once); three
//                          parallel carry-save steps leave balanced digits within +-70
//   P = q * N              output tiles 36..73 (Toeplitz(N) table W2, K order matching the
//                          C layout q comes out in), tile 36 only for the carry of the low
//                          half: c = (T_low + P_low)/R, estimated from positions 576..591 in
//                          double and rounded (the rest weighs < 2^-100)
//   U + N = T_high + P_high + c + N: each lane's 4 digit sums become one 28-bit limb + a
//          signed carry to the next limb, staged in the wave's slot rows.
// Phase C (VALU): per limb, T_high + stage + N + a bias that sums to exactly 2^4144 (2^28 at
// limb 0, 2^28 - 1 above) so every lane's local value is positive and the top lane's local
// carry is exactly 1; normalize_almost drops it.  Output < 1.56 N, almost normalised, i.e.
// the contract of sqr<4>.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../fate_amd/csrc/mont27_dev.h"

using namespace fphe;
using namespace fphe::r28;

typedef int v4i __attribute__((ext_vector_type(4)));

constexpr int kT = 4, kE = 16, kNL = 148;
constexpr int kRows = 148;               // slot rows per wave
constexpr int kWave = kRows * 16;
#ifndef SQ_BLOCK_WAVES
#define SQ_BLOCK_WAVES 6
#endif
constexpr int kBW = SQ_BLOCK_WAVES;      // waves per block (6: two blocks of LDS fit a CU at 3 waves/SIMD)
constexpr int kW1 = 640, kW1Off = 48;    // W1[b + 48], b in [-48, 591]: bytes N'[b - j]
constexpr int kW2 = 668, kW2Off = 12;    // W2[b + 12], b in [-12, 655]: bytes N[b - 16(j>>2) - (j&3)]
static_assert(LL == 37 && LB == 28, "the digit layout assumes 28-bit limbs, 37 per lane");

__device__ __forceinline__ u32 spread7(u32 L) {  // 28-bit limb -> its four 7-bit digits as bytes
  return (L & 0x7Fu) | ((L << 1) & 0x7F00u) | ((L << 2) & 0x7F0000u) | ((L << 3) & 0x7F000000u);
}
// value of lane (l - 16) mod 64, i.e. row g <- row g-1 of the wave, from two lane swaps
// (VALU, no LDS round trip): permlane16_swap(x, x) = {[x0,x0,x2,x2], [x1,x1,x3,x3]} by rows,
// permlane32_swap of the second = {[x1,x1,x1,x1], [x3,x3,x3,x3]}.
#ifndef SQ_STAGGER
#define SQ_STAGGER 0
#endif
#ifndef SQ_STAMPS
#define SQ_STAMPS 0
#endif
#if SQ_STAMPS
__device__ unsigned long long g_stamp[8];
#define STAMP(k) do { const unsigned long long _t = __builtin_amdgcn_s_memtime(); st[k] += _t - st_last; st_last = _t; } while (0)
#else
#define STAMP(k) do {} while (0)
#endif
#ifndef SQ_SPLIT_ACC
#define SQ_SPLIT_ACC 1
#endif
#ifndef SQ_PERMLANE
#define SQ_PERMLANE 1
#endif
__device__ __forceinline__ int from_below16(int x) {
#if SQ_PERMLANE
  const int g = (int)((threadIdx.x >> 4) & 3u);
  const auto p16 = __builtin_amdgcn_permlane16_swap((unsigned)x, (unsigned)x, false, false);
  const auto p32 = __builtin_amdgcn_permlane32_swap(p16[1], p16[1], false, false);
  return (g & 1) ? (int)p16[0] : (g == 2 ? (int)p32[0] : (int)p32[1]);
#else
  return __builtin_amdgcn_ds_bpermute((int)(((threadIdx.x - 16u) & 63u) << 2), x);
#endif
}

#ifndef SQ_EARLY_B
#define SQ_EARLY_B 1
#endif
// ---- phase A: squaring rows without reduction ---------------------------------------------
template <int a>
__device__ __forceinline__ void sqz_rows(u64 (&T)[LL], const L27& A, u32& b, u32* bs, const u32* bnext,
                                         u32 shf, u32 mkf, u32 mkx) {
  // the slot holds 2a (fused-path convention): bf = 2a (q > s), a (q == s) or 0 (q < s)
  const u32 bf = __builtin_amdgcn_ubfe(b, shf, mkf);
  // b_{i+1} is read before the row's MACs so its LDS latency hides under them (read after
  // the row it was waited for ~8 instructions later, one exposed LDS latency per row)
  u32 bn;
#if SQ_EARLY_B
  if constexpr (a + 1 < LL) bn = bs[(a + 1) * kE];
  else bn = bnext[0];
  r27_sqrow<a>(T, A, bf, b, 0u);
#else
  r27_sqrow<a>(T, A, bf, b, 0u);
  if constexpr (a + 1 < LL) bn = bs[(a + 1) * kE];
  else bn = bnext[0];
#endif
  const u64 X = T[0];
#pragma unroll
  for (int j = 0; j < LL - 1; ++j) T[j] = T[j + 1];
  T[0] += X >> LB;
  T[LL - 1] = (u64)(dpp_from_next((u32)X) & mkx);  // the top lane (q = 3) takes 0: nothing crosses elements
  // limb 37s + a of T_low (lane 0's X) into the slot the row consumed: broadcast over the
  // element's 4 lanes, which then all store the same word
  bs[a * kE] = dpp_bcast<kT>((u32)X) & MASK;
  asm volatile("" : "+v"(bn));
  b = bn;
  if constexpr (a + 1 < LL) sqz_rows<a + 1>(T, A, b, bs, bnext, shf, mkf, mkx);
}

// ---- phase B helpers ------------------------------------------------------------------------
// q digits from a C-layout tile (lane group g: positions 4g + r, r = 0..3, i.e. one 28-bit
// limb position; column sums of unsigned 7-bit digits, < 592 * 127^2 < 2^23.2).  The lane's
// four sums form v = sum acc_r 2^(7r) (|v| < 2^44.3); ONE parallel carry-save step in base
// 2^28 (keep the balanced low 28 bits, add the carry of the limb below, |carry| < 2^16.3)
// leaves |x| <= 2^27 + 2^16.3, whose balanced 7-bit digits lie in [-64, 63] except the top
// one, in [-65, 64].  prev: the previous tile's top-limb carry (valid in lane group 0).
#ifndef SQ_QSTEP28
#define SQ_QSTEP28 1
#endif
__device__ __forceinline__ u32 q_digits(const v4i& acc, int& prev0, int& prev1, int g) {
#if SQ_QSTEP28
  (void)prev1;
  const int w0 = acc[0] + (acc[1] << 7), w1 = acc[2] + (acc[3] << 7);
  const long long v = (long long)w1 * 16384 + (long long)w0;
  const int c = (int)((v + (1ll << 27)) >> 28);
  const int d = (int)((u32)v - ((u32)c << 28));
  const int rot = from_below16(c);
  const int cin = g > 0 ? rot : prev0;
  prev0 = rot;
  const int x = d + cin;
  const int d0 = __builtin_amdgcn_sbfe(x, 0, 7);
  const int x1 = (x - d0) >> 7;
  const int d1 = __builtin_amdgcn_sbfe(x1, 0, 7);
  const int x2 = (x1 - d1) >> 7;
  const int d2 = __builtin_amdgcn_sbfe(x2, 0, 7);
  const int d3 = (x2 - d2) >> 7;
  return (u32)(d0 & 255) | ((u32)(d1 & 255) << 8) | ((u32)(d2 & 255) << 16) | ((u32)d3 << 24);
#else
  int w0 = acc[0] + (acc[1] << 7);
  int w1 = acc[2] + (acc[3] << 7);
#pragma unroll
  for (int st = 0; st < 2; ++st) {
    const int d0 = __builtin_amdgcn_sbfe(w0, 0, 14), d1 = __builtin_amdgcn_sbfe(w1, 0, 14);
    const int c0 = (w0 - d0) >> 14, c1 = (w1 - d1) >> 14;
    const int rot = from_below16(c1);
    int& prev = st == 0 ? prev0 : prev1;
    const int cin = g > 0 ? rot : prev;
    prev = rot;
    w0 = d0 + cin;
    w1 = d1 + c0;
  }
  const int l0 = __builtin_amdgcn_sbfe(w0, 0, 7), l1 = __builtin_amdgcn_sbfe(w1, 0, 7);
  const int h0 = (w0 - l0) >> 7, h1 = (w1 - l1) >> 7;
  return (u32)(l0 & 255) | ((u32)(h0 & 255) << 8) | ((u32)(l1 & 255) << 16) | ((u32)h1 << 24);
#endif
}

// Scheduling of one product tile's table reads and MFMAs: with SQ_LOOKAHEAD = L > 0 the
// first L ds_read_b128 are issued together and every MFMA is followed by the read L places
// ahead, so an MFMA waits for a read issued L MFMAs (>= 16 L cycles) earlier instead of the
// one issued just before it (the compiler's own schedule keeps one read in flight).
#ifndef SQ_LOOKAHEAD
#define SQ_LOOKAHEAD 0
#endif
__device__ __forceinline__ void lookahead_groups(int n) {
#if SQ_LOOKAHEAD
  constexpr int L = SQ_LOOKAHEAD;
#pragma unroll
  for (int i = 0; i < (n < L ? n : L); ++i) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
#pragma unroll
  for (int i = 0; i < n; ++i) {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    if (i + L < n) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
  }
#else
  (void)n;
#endif
}

template <int SKIP>
__device__ __forceinline__ void mfma_sqr(L27& A, u32* bcol, u32 qoff, u32* wb, const v4i* W1s,
                                         const v4i* W2s, const u32* Nq, int q, unsigned long long* st,
                                         unsigned long long& st_last) {
  (void)st;
  (void)st_last;
  // phase A
#pragma unroll
  for (int j = 0; j < LL; ++j) bcol[qoff + j * kE] = A[j] << 1;
  u64 T[LL];
#pragma unroll
  for (int j = 0; j < LL; ++j) T[j] = 0;
  {
    u32 b = bcol[0];
    const u32 mkx = q == kT - 1 ? 0u : MASK;
#pragma unroll 1
    for (int s = 0; s < (SKIP == 1 ? 0 : kT); ++s) {
      const u32 shf = q == s ? 1u : 0u;
      const u32 mkf = q > s ? 31u : (q == s ? 30u : 0u);
      u32* bs = bcol + s * LL * kE;
      const u32* bnext = s + 1 < kT ? bs + LL * kE : bcol;
      sqz_rows<0>(T, A, b, bs, bnext, shf, mkf, mkx);
    }
  }
  STAMP(0);
  L27 H;  // T_high as almost-normalised limbs (< 2^4050: no carry leaves the top lane)
  normalize_almost<kT>(T, H, q);
  // phase B
  const int l = (int)(threadIdx.x & 63u), g = l >> 4, c16 = l & 15;
  if constexpr (SKIP != 2) {
  v4i tf[10];
#pragma unroll
  for (int kt = 0; kt < 10; ++kt) {
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      int row = 16 * kt + 4 * g + w;
      if (kt == 9) row = g == 0 ? row : 0;  // rows 148..159 are zero digits
      u32 L = wb[row * kE + c16];
      if (kt == 9) L = g == 0 ? L : 0u;
      tf[kt][w] = (int)spread7(L);
    }
  }
  // T_high -> the slot rows (after the reads above: one wave, LDS in order); product 2 adds
  // its limbs to them, so no T_high registers stay live across the MFMA phase
#pragma unroll
  for (int j = 0; j < LL; ++j) bcol[qoff + j * kE] = H[j];
  STAMP(1);
  const int w1l = kW1Off + c16 - 16 * g;
  v4i qv[10];  // q as B fragments: K-tile kt = output tiles 4kt..4kt+3 (37..39 zero)
  qv[9] = v4i{0, 0, 0, 0};
  int pr0 = 0, pr1 = 0;
  // software-pipelined: the MFMAs of tile m+1 are issued before the digit VALU work of tile m
  auto chain1 = [&](int m) {
    // two independent accumulators (even / odd K-tiles) so dependent MFMAs do not wait on
    // each other back to back
    v4i acc = {0, 0, 0, 0}, acc2 = {0, 0, 0, 0};
#pragma unroll
    for (int kt = 0; kt <= m / 4; ++kt) {
      if (SQ_SPLIT_ACC && (kt & 1))
        acc2 = __builtin_amdgcn_mfma_i32_16x16x64_i8(W1s[16 * (m - 4 * kt) + w1l], tf[kt], acc2, 0, 0, 0);
      else
        acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(W1s[16 * (m - 4 * kt) + w1l], tf[kt], acc, 0, 0, 0);
    }
    lookahead_groups(m / 4 + 1);
    return SQ_SPLIT_ACC ? acc + acc2 : acc;
  };
  v4i cur = chain1(0);
#pragma unroll
  for (int m = 0; m < 37; ++m) {
    __builtin_amdgcn_sched_barrier(0);
    v4i nxt = {0, 0, 0, 0};
    if (m + 1 < 37) nxt = chain1(m + 1);
    __builtin_amdgcn_sched_barrier(0);
    qv[m / 4][m % 4] = (int)q_digits(cur, pr0, pr1, g);
    cur = nxt;
  }
  STAMP(2);
  const int w2l = kW2Off + c16 - 4 * g;
  int cval = 0, phi = 0;
  auto chain2 = [&](int t) {
    v4i acc = {0, 0, 0, 0}, acc2 = {0, 0, 0, 0};
    const int k0 = t > 40 ? (t - 40 + 3) / 4 : 0;
    const int k1 = t / 4 < 9 ? t / 4 : 9;
#pragma unroll
    for (int kt = k0; kt <= k1; ++kt) {
      if (SQ_SPLIT_ACC && ((kt - k0) & 1))
        acc2 = __builtin_amdgcn_mfma_i32_16x16x64_i8(W2s[16 * (t - 4 * kt) + w2l], qv[kt], acc2, 0, 0, 0);
      else
        acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(W2s[16 * (t - 4 * kt) + w2l], qv[kt], acc, 0, 0, 0);
    }
    lookahead_groups(k1 - k0 + 1);
    return SQ_SPLIT_ACC ? acc + acc2 : acc;
  };
  v4i cur2 = chain2(36);
#pragma unroll
  for (int t = 36; t < 74; ++t) {
    __builtin_amdgcn_sched_barrier(0);
    v4i nxt = {0, 0, 0, 0};
    if (t + 1 < 74) nxt = chain2(t + 1);
    __builtin_amdgcn_sched_barrier(0);
    const v4i acc = cur2;
    cur2 = nxt;
    if (t == 36) {
      // (T_low + P_low) / R from positions 576..591: this lane's rows 576 + 4g + r, plus the
      // T digits of limbs 144..147 (K-tile 9, group 0)
      double s = 0.0;
#pragma unroll
      for (int r = 0; r < 4; ++r) s += (double)acc[r] * __builtin_ldexp(1.0, 7 * (4 * g + r - 16));
      if (g == 0) {
#pragma unroll
        for (int w = 0; w < 4; ++w)
#pragma unroll
          for (int y = 0; y < 4; ++y)
            s += (double)((tf[9][w] >> (8 * y)) & 127) * __builtin_ldexp(1.0, 7 * (4 * w + y - 16));
      }
      s += __shfl_xor(s, 16, 64);
      s += __shfl_xor(s, 32, 64);
      cval = (int)__builtin_rint(s);
    } else {
      // limb value acc0 + 2^7 acc1 + 2^14 acc2 + 2^21 acc3 (|acc| < 2^22.3): two 32-bit
      // halves, one signed 64-bit mad, then the 28-bit limb and the carry above it
      const int w0 = acc[0] + (acc[1] << 7), w1 = acc[2] + (acc[3] << 7);
      const long long v = (long long)w1 * 16384 + (long long)w0;
      const int lo = (int)((u32)v & MASK);
      const int hi = (int)(v >> LB);
      const int rot = from_below16(hi);
      const int hin = g > 0 ? rot : phi;
      phi = rot;
      int val = lo + hin;
      if (t == 37 && g == 0) val += cval;
      if (t == 73 && g == 3) val += hi << LB;  // limb 148's carry, as 2^28 units of limb 147
      u32* rp = wb + (4 * (t - 37) + g) * kE + c16;
      *rp = *rp + (u32)val;
    }
  }
  }
  STAMP(3);
  // phase C
#pragma unroll
  for (int j = 0; j < LL; ++j) {
    const int sv = (int)bcol[qoff + j * kE];
    const u32 bias = (j == 0 && q == 0) ? (1u << LB) : ((1u << LB) - 1u);
    T[j] = (u64)(long long)sv + (u64)Nq[j] + (u64)bias;  // sv = T_high limb + P_high part
  }
  normalize_almost<kT>(T, A, q);
  STAMP(4);
}

__device__ int g_roles[16];
extern "C" int sqchain_roles(int* out) { return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_roles), sizeof(int) * 16); }
#ifndef SQ_TILE_BARRIER
#define SQ_TILE_BARRIER 1
#endif
#ifndef SQ_WAVES
#define SQ_WAVES 2
#endif
template <int V, int BW = (V == 0 ? 4 : kBW)>
__global__ __launch_bounds__(64 * BW) __attribute__((amdgpu_waves_per_eu(V >= 1 ? SQ_WAVES : 3))) void k_sqchain(const u32* __restrict__ X, u32* __restrict__ Y,
                                                 const u32* __restrict__ Nl, u32 np, const v4i* __restrict__ W,
                                                 int nelem, int S) {
  extern __shared__ __attribute__((aligned(16))) u32 lds[];
  v4i* Ws = reinterpret_cast<v4i*>(lds + BW * kWave);
  u32* Ns = reinterpret_cast<u32*>(Ws + kW1 + kW2);
  if (V >= 1) {
    for (int i = threadIdx.x; i < kW1 + kW2; i += blockDim.x) Ws[i] = W[i];
    for (int i = threadIdx.x; i < kNL; i += blockDim.x) Ns[i] = Nl[i];
    __syncthreads();
  }
  const int wib = (int)(threadIdx.x >> 6);
  bool role_b = false;
  if constexpr (V == 4) {
    // SIMD of this wave from HW_ID bits 5:4 (gfx9 layout), then an arrival order per SIMD
    __shared__ int simd_cnt[4];
    if (threadIdx.x < 4) simd_cnt[threadIdx.x] = 0;
    __syncthreads();
    const int simd = (__builtin_amdgcn_s_getreg(4 | (4 << 6) | (1 << 11))) & 3;
    int k = 0;
    if ((threadIdx.x & 63) == 0) k = atomicAdd(&simd_cnt[simd], 1);
    k = __builtin_amdgcn_readfirstlane(k);
    role_b = k == 0;
    if ((threadIdx.x & 63) == 0 && blockIdx.x == 0) g_roles[wib] = simd * 16 + k;
  }
  const int wave = (int)(blockIdx.x * BW + wib);
  if (wave * kE >= nelem) return;
  Geo<kT> geo;
  u32* wb = lds + wib * kWave;
  u32* bcol = wb + geo.e;
  const u32 qoff = lds_qoff<kT>(geo.q);
  Mod<kT> N;
  if constexpr (V == 0) N.init(Nl, geo.q);
  const u32* x = X + (size_t)(wave * kE + geo.e) * kNL + LL * geo.q;
  L27 A;
#pragma unroll
  for (int k = 0; k < LP; ++k) A.set2(k, x[2 * k], 2 * k + 1 < LL ? x[2 * k + 1] : 0u);
#if SQ_STAGGER
  // waves sharing a SIMD (wib, wib + 4, wib + 8 of a 12-wave block) start a third of a
  // squaring apart, so their product phases do not coincide
  if (V == 1) {
    const int lag = (int)(wib / 4);
    for (int i = 0; i < lag * SQ_STAGGER; ++i) __builtin_amdgcn_s_sleep(127);
  }
#endif
  unsigned long long st[5] = {0, 0, 0, 0, 0};
  unsigned long long st_last = SQ_STAMPS ? __builtin_amdgcn_s_memtime() : 0;
#pragma unroll 1
  for (int s = 0; s < S; ++s) {
    if constexpr (V == 0) sqr<kT>(A, bcol, qoff, N, np, geo.q);
    else if constexpr (V == 4) {
      // overlap test: the first wave to arrive on each SIMD runs only the product phase,
      // the others only the rows: two row waves and one product wave per SIMD
      if (role_b) mfma_sqr<1>(A, bcol, qoff, wb, Ws, Ws + kW1, Ns + LL * geo.q, geo.q, st, st_last);
      else mfma_sqr<2>(A, bcol, qoff, wb, Ws, Ws + kW1, Ns + LL * geo.q, geo.q, st, st_last);
    } else mfma_sqr<V - 1>(A, bcol, qoff, wb, Ws, Ws + kW1, Ns + LL * geo.q, geo.q, st, st_last);
  }
#if SQ_STAMPS
  if (V >= 1 && (threadIdx.x & 63) == 0)
    for (int k = 0; k < 5; ++k) atomicAdd(&g_stamp[k], st[k]);
#endif
  u32* y = Y + (size_t)(wave * kE + geo.e) * kNL + LL * geo.q;
#pragma unroll
  for (int j = 0; j < LL; ++j) y[j] = A[j];
}

template <int V>
static void launch(const void* X, void* Y, const void* Nl, unsigned np, const void* W, int nelem, int S,
                   hipStream_t stream) {
  constexpr int BW = V == 0 ? 4 : kBW;
  const int waves = nelem / kE;
  const int blocks = (waves + BW - 1) / BW;
  const size_t lds = (size_t)BW * kWave * 4 + (V ? (size_t)(kW1 + kW2) * 16 + kNL * 4 : 0);
  hipLaunchKernelGGL((k_sqchain<V>), dim3(blocks), dim3(64 * BW), lds, stream, (const u32*)X, (u32*)Y,
                     (const u32*)Nl, np, (const v4i*)W, nelem, S);
}

extern "C" int sqchain_launch(int variant, const void* X, void* Y, const void* Nl, unsigned np, const void* W,
                              int nelem, int S, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (variant == 0) launch<0>(X, Y, Nl, np, W, nelem, S, st);
  else if (variant == 1) launch<1>(X, Y, Nl, np, W, nelem, S, st);
  else if (variant == 2) launch<2>(X, Y, Nl, np, W, nelem, S, st);
  else if (variant == 3) launch<3>(X, Y, Nl, np, W, nelem, S, st);
  else launch<4>(X, Y, Nl, np, W, nelem, S, st);
  return (int)hipGetLastError();
}

extern "C" int sqchain_stamps(unsigned long long* out) {
#if SQ_STAMPS
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamp), sizeof(unsigned long long) * 5);
#else
  (void)out;
  return -1;
#endif
}
