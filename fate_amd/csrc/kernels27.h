// Reduced-radix modexp kernels: encrypt, decrypt (modexp phase), ct-add, ct x pt, folds,
// inverses.  Included by fate_phe.hip after KeyArgs / nude_to_slot / helpers.
// Geometry: TPI adjacent lanes per element (r27::Geo), E = 64/TPI elements per wave; a
// wave's E elements always sit in one 64-element memory tile, so the memory tile index is
// wave-uniform and only the column (element % 64) is per lane.
#pragma once
#include "mont27_dev.h"

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
// r02f_ab_occ3_ops.txt: add +5%, ct x pt +1%); the segmented fold stays at 2 (-7% at 3;
// again -7% in round 6 with 308 B/lane spilled, profiles/r06/r06x_ab_fold_occ3_negative.txt).
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
// the fold's term prefetch one product ahead (35 VGPRs held across the product: 2 waves)
#ifndef FPHE_FOLD_PF
#define FPHE_FOLD_PF 1
#endif
#define FPHE_OCC_MISC __attribute__((amdgpu_waves_per_eu(FPHE_MISC_OCC)))
// ct-add: both operands held in registers across the alignment squarings (read once, no
// copy-through re-reads for literal 1s), at the 2-wave register budget: same-box A/B
// (profiles/r03/r03n_ab_add.txt) 7.58 ms per 2^20 against 7.90 at 3 waves with the re-reads
// (92 dwords spilled there), HBM traffic 5.8 KB/element against 12.9
#ifndef FPHE_ADD_KEEPY
#define FPHE_ADD_KEEPY 1
#endif
#ifndef FPHE_ADD_OCC
#define FPHE_ADD_OCC 2
#endif
#define FPHE_OCC_ADD __attribute__((amdgpu_waves_per_eu(FPHE_ADD_OCC)))
#define FPHE_OCC_FOLD __attribute__((amdgpu_waves_per_eu(FPHE_FOLD_OCC)))
// the balanced first fold level (k_segfold27) on its own: its occupancy, and whether it fetches
// the next term's words during the current product (35 VGPRs held across it) or right before
// its own product (nothing but index state across a product)
#ifndef FPHE_SEGFOLD_OCC
#define FPHE_SEGFOLD_OCC FPHE_FOLD_OCC
#endif
#ifndef FPHE_SEGFOLD_PF
#define FPHE_SEGFOLD_PF 1
#endif
#define FPHE_OCC_SEGFOLD __attribute__((amdgpu_waves_per_eu(FPHE_SEGFOLD_OCC)))
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

using fphe::rad_ll;
using fphe::rad_lb;

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

// key-holder encrypt in two modexp steps (k_pow_small27, then k_pow_half27<., ., true>);
// 0: one |n|-bit exponent mod s^2 per half (A/B)
#ifndef FPHE_KH_SPLIT
#define FPHE_KH_SPLIT 1
#endif
// words per half of the step-1 values z_s (< s): one lane's 32-word chunk per lane of s's
// engine (TPIs = L/128 lanes, at least 1)
template <int L>
constexpr uint32_t kZWords = 32u * (L >= 128 ? L / 128 : 1);
// the split pays where s runs on a smaller engine than s^2 (keys > 1024 bits); at 1024 bits
// both are 37-limb TPI-1 engines and the split only adds work (same-box -1.5%)
template <int L>
constexpr bool kKhSplit = FPHE_KH_SPLIT && L >= 128;
constexpr int kFoldMax = 64;  // terms per k_fold27 chunk
// items per wave slot of the balanced first fold level (k_segfold27), at most
constexpr int kSegFoldMax = 1024;
// Slot plan of the balanced first fold level (fphe_fold_segments, group_dev.h k_gr_plan):
// the sorted items cut into regions -- stretches packed at `rlen` items per wave slot, and the
// runs of "raised" keys (far above their segment's least exponent), each cut into slots of
// fewer items so that a slot's products plus its closing 4 gap squarings take about as long as
// a stretch slot.  k_segfold27 raises such a slot's partial to the segment's least exponent
// itself, inside the balanced launch, instead of leaving a 4-gap-squaring chain on one wave
// after it (the exponent merge).  One int32 buffer:
//   [0] regions, [1] slots, then kPlanRegions entries each of rslot (first slot; rslot of the
//   last region + its slots = total), rstart, rend (items), rlen (items per slot), rgap, rexp.
constexpr int kRaiseMax = 512;                     // raised keys per call, at most
constexpr int kPlanRegions = 2 * kRaiseMax + 1;
constexpr int kPlanWords = 2 + 6 * kPlanRegions;
// the slot-plan weight of raising a partial by 16^gap: 4 gap squarings, each a product of the
// partial with itself in k_segfold27's loop
__host__ __device__ constexpr long long raise_cost(long long gap) { return 4 * gap; }
struct SlotRange {
  int64_t p0, p1;  // items [p0, p1)
  int gap;         // raise the slot's partial by 16^gap (0: a stretch slot)
  int ex;          // ... to this exponent
};
__device__ __forceinline__ SlotRange plan_range(const int32_t* __restrict__ plan, size_t slot) {
  const int32_t nreg = plan[0];
  const int32_t* rslot = plan + 2;
  int lo = 0, hi = nreg - 1;  // the last region whose first slot is <= slot
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if ((size_t)rslot[mid] <= slot) lo = mid;
    else hi = mid - 1;
  }
  const int32_t* f = plan + 2 + lo;
  SlotRange s;
  const int64_t len = f[3 * kPlanRegions], end = f[2 * kPlanRegions];
  s.p0 = (int64_t)f[kPlanRegions] + (int64_t)(slot - (size_t)f[0]) * len;
  s.p0 = s.p0 < end ? s.p0 : end;  // a region's padding slots are empty
  s.p1 = s.p0 + len < end ? s.p0 + len : end;
  s.gap = f[4 * kPlanRegions];
  s.ex = f[5 * kPlanRegions];
  return s;
}

// slot -> items: the plan's, or i r .. (i + 1) r without one
__device__ __forceinline__ void slot_items(const int32_t* __restrict__ plan, size_t i, size_t T, uint32_t r, size_t& p0,
                                           size_t& p1) {
  if (plan) {
    const SlotRange sr = plan_range(plan, i);
    p0 = (size_t)sr.p0;
    p1 = (size_t)sr.p1;
  } else {
    p0 = i * r;
    p1 = p0 + r < T ? p0 + r : T;
  }
}

// largest exponent gap k_add27 / k_align27 act on (4 kMaxGap squarings, ~7 s on one wave):
// far beyond the reference encoders' exponent range (f64: [-282, 242]); fphe_align rejects
// larger gaps on the host side (fate_amd/paillier.py), k_add27 caps them
constexpr int kMaxGap = 1 << 16;

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

// ---- the engine's kernels, once per radix -------------------------------------------------
namespace k27 {
using namespace fphe::r27;
#include "kernels_engine.inc"
}  // namespace k27
namespace k28 {
using namespace fphe::r28;
#include "kernels_engine.inc"
}  // namespace k28

// the radix namespace of a TPI (mont27_dev.h rad_lb: 28 everywhere unless FPHE_RADIX4=27)
template <int TPI>
using KS = std::conditional_t<fphe::rad_lb(TPI) == 27, k27::Kern, k28::Kern>;

}  // namespace
