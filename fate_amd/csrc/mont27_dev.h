// Reduced-radix Montgomery arithmetic for gfx950: 27- or 28-bit limbs, 64-bit lazy accumulators.
//
// Why (measured): on gfx950 v_mad_u64_u32, v_add_co_u32 and v_addc_co_u32
// all issue at half rate, so a 32-bit-limb CIOS MAC (mad + add_co + addc) costs three
// half-rate issues.  With 27-bit limbs a product is < 2^54 and a 64-bit accumulator
// absorbs every product a column ever receives (<= 2*152 products < 2^62.3), so a MAC
// is ONE v_mad_u64_u32 (D64 = a*b + acc64) with no carry handling inside the product.
// 152 limbs cover 4096-bit moduli (4104 bits): 1.41x the MACs of 128 x 32-bit limbs at
// one third of the instructions.
//
// Layout: an element's NL = LL*TPI limbs are spread over TPI in {1,2,4} ADJACENT lanes
// (lane = TPI*e + q); lane q holds limbs [LL q, LL q + LL) of A (u32) and T (u64), and of the
// modulus N (u32 VGPRs when TPI > 1; wave-uniform scalar loads when TPI == 1).  Per CIOS
// row the lanes of an element exchange two values with DPP (full-rate VALU, no LDS):
//   m      : quad_perm broadcast from the element's lane 0        (lane i <- lane i&~(TPI-1))
//   X      : the reduction word leaving lane q's bottom limb goes to lane q-1's top limb
//            (row_shl:1: lane i <- lane i+1)
// DPP semantics verified on MI355X by tools/probe/dpp_probe.hip.
//
// Lazy Montgomery: R = 2^(LB*NL) >= 4N for every modulus used here, so a product of two
// operands < 2N is < 2N again ((4N^2 + RN)/R <= 2N) and no conditional subtraction is
// needed between products; an operand >= 2N is allowed only against a second operand
// < N with the first < R (then (RN + RN)/R = 2N).  finalize() maps a final value < 2N
// to its canonical residue with one subtraction.
//
// Two radices, one engine text (mont_engine.inc, inv_engine.inc) compiled in two namespaces:
//   r28: 28-bit limbs, 37 per lane (1036 bits) -- every modulus (the engine in use): a
//        product is < 2^56 and a column takes <= 3 products per row span; at NL <= 74 that
//        fits 64 bits outright (< 2^63.8), at NL = 148 (TPI 4, the 4096-bit n^2 of 2048-bit
//        keys) a carry sweep after half the rows bounds the slots again (mont_engine.inc
//        sweep()).  37 limbs per lane instead of 38 cut a product's MACs by (NL'/NL)^2 and a
//        squaring row to 19 + 37 MACs (odd LL: no half-window column), against 20 + 38.
//   r27: 27-bit limbs, 38 per lane (1026 bits) -- round 1's engine, no sweep needed
//        (< 2^62.3 at NL = 152); kept for same-box A/B (FPHE_RADIX4=27 builds TPI 4 on it).
// kernels27.h instantiates every kernel in both and the launchers pick by TPI (KS<TPI>).
#pragma once
#include "mont_dev.h"

#ifndef FPHE_TAB_BATCH
#define FPHE_TAB_BATCH 1
#endif
#ifndef FPHE_PIN_BNEXT
#define FPHE_PIN_BNEXT 1
#endif
#ifndef FPHE_FUSED
#define FPHE_FUSED 1
#endif
// general-product rows per loop iteration: 2 (same-box, profiles/r03/r03l_ab_row_unroll.txt:
// ct-add -3%, ct x pt -4%, the histogram fold -4%, encrypt and decrypt unchanged); 4 compiles
// for ~17 min into a 17 MB library
#ifndef FPHE_ROW_UNROLL
#define FPHE_ROW_UNROLL 2
#endif
#define FPHE_PRAGMA_(x) _Pragma(#x)
#define FPHE_UNROLL_(n) FPHE_PRAGMA_(unroll n)
#define FPHE_UNROLL(n) FPHE_UNROLL_(n)

namespace fphe {
namespace r27 {
constexpr int LB = 27;
constexpr int LL = 38;
#define RG_GEN_FILE "mont_gen_ll38.h"
#define RG_SECTION 1
#include RG_GEN_FILE
#undef RG_SECTION
#include "mont_engine.inc"
#include "inv_engine.inc"
#define RG_SECTION 4
#include RG_GEN_FILE
#undef RG_SECTION
#undef RG_GEN_FILE
}  // namespace r27

namespace r28 {
constexpr int LB = 28;
constexpr int LL = 37;
#define RG_GEN_FILE "mont_gen_ll37.h"
#define RG_SECTION 1
#include RG_GEN_FILE
#undef RG_SECTION
#include "mont_engine.inc"
#include "inv_engine.inc"
#define RG_SECTION 4
#include RG_GEN_FILE
#undef RG_SECTION
#undef RG_GEN_FILE
}  // namespace r28

// limb geometry of the engine a TPI runs on (host and device): 28 x 37, or 27 x 38 for the
// 4096-bit geometry when built with FPHE_RADIX4=27
#ifndef FPHE_RADIX4
#define FPHE_RADIX4 28
#endif
constexpr int rad_lb(int tpi) { return tpi == 4 ? FPHE_RADIX4 : 28; }
constexpr int rad_ll(int tpi) { return rad_lb(tpi) == 27 ? 38 : 37; }
}  // namespace fphe
