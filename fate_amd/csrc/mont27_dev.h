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
//   r27: 27-bit limbs, 38 per lane (1026 bits) -- TPI = 4, the 4096-bit n^2 of 2048-bit keys:
//        a column takes <= 2 x 152 products < 2^54, < 2^62.3;
//   r28: 28-bit limbs, 37 per lane (1036 bits) -- TPI = 1, 2, every modulus up to 2048 bits
//        (p^2, q^2 and n of 2048-bit keys; all moduli of <= 1024-bit keys): a column takes
//        <= 2 x 74 products < 2^56.01, < 2^63.3.  74 limbs instead of 76 cut the MACs of a
//        product by (74/76)^2 and a squaring row to 19 + 37 MACs (odd LL: no half-window
//        column), against 20 + 38.  At TPI = 4, 28-bit limbs would overflow a 64-bit column
//        (2 x 148 x 2^56 > 2^64), so the 4096-bit engine stays at 27 bits.
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

// limb geometry of the engine a TPI runs on (host and device)
constexpr int rad_lb(int tpi) { return tpi == 4 ? 27 : 28; }
constexpr int rad_ll(int tpi) { return tpi == 4 ? 38 : 37; }
}  // namespace fphe
