#!/usr/bin/env python3
"""Generate fate_amd/csrc/mont_asm_gen.h: the inline-asm MAC groups of the CIOS
Montgomery multiplication used by fate_amd/csrc/mont_dev.h.

Why asm: hipcc lowers `acc = (u64)a*b + t + (acc>>32)` to v_mad_u64_u32 + zero-extension
moves + a 64-bit add and keeps T[] as 64-bit pairs (2x the VGPRs).  The hand schedule is
3 VALU ops per 32x32 MAC (v_mad_u64_u32, v_add_co_u32, v_addc_co_u32) with the running
carry kept in a fixed aligned pair {v0,v1=0} (operand-product chain) / {v4,v5=0}
(reduction chain), so the carry feeds the next v_mad_u64_u32 as its 64-bit addend with
no extra moves.  The two chains of one CIOS row are interleaved for ILP.

Run: python3 tools/gen_mont_asm.py > fate_amd/csrc/mont_asm_gen.h
"""
G = 16  # limbs per asm block


def std_group() -> str:
    """Limbs j0..j0+15 of one CIOS row (j0 >= 16).
    t_k <-> T[j0-1+k] (k = 0..16), a_k <-> A[j0+k], n_k <-> N[j0+k]."""
    s = ["v_mov_b32 v0, %[c1]", "v_mov_b32 v1, 0", "v_mov_b32 v4, %[c2]", "v_mov_b32 v5, 0"]
    for k in range(G):
        s += [
            f"v_mad_u64_u32 v[2:3], vcc, %[a{k}], %[b], v[0:1]",
            f"v_mad_u64_u32 v[6:7], %[k2], %[m], %[n{k}], v[4:5]",
            f"v_add_co_u32 %[t{k+1}], vcc, %[t{k+1}], v2",
            "v_addc_co_u32 v0, vcc, v3, 0, vcc",
            f"v_add_co_u32 %[t{k}], %[k2], %[t{k+1}], v6",
            "v_addc_co_u32 v4, %[k2], v7, 0, %[k2]",
        ]
    s += ["v_mov_b32 %[c1], v0", "v_mov_b32 %[c2], v4"]
    return "\\n\\t".join(s)


def first_group() -> str:
    """Limbs 0..15 of one CIOS row; computes m = T0 * n0inv after the first MAC.
    t_k <-> T[k] (k = 0..15)."""
    s = [
        "v_mad_u64_u32 v[2:3], vcc, %[a0], %[b], 0",
        "v_add_co_u32 %[t0], vcc, %[t0], v2",
        "v_addc_co_u32 v0, vcc, v3, 0, vcc",
        "v_mov_b32 v1, 0",
        "v_mul_lo_u32 %[m], %[t0], %[ninv]",
        "v_mov_b32 v5, 0",
        "v_mov_b32 v4, %[t0]",
        "v_mad_u64_u32 v[6:7], %[k2], %[m], %[n0], v[4:5]",
        "v_mov_b32 v4, v7",
    ]
    for k in range(1, G):
        s += [
            f"v_mad_u64_u32 v[2:3], vcc, %[a{k}], %[b], v[0:1]",
            f"v_mad_u64_u32 v[6:7], %[k2], %[m], %[n{k}], v[4:5]",
            f"v_add_co_u32 %[t{k}], vcc, %[t{k}], v2",
            "v_addc_co_u32 v0, vcc, v3, 0, vcc",
            f"v_add_co_u32 %[t{k-1}], %[k2], %[t{k}], v6",
            "v_addc_co_u32 v4, %[k2], v7, 0, %[k2]",
        ]
    s += ["v_mov_b32 %[c1], v0", "v_mov_b32 %[c2], v4"]
    return "\\n\\t".join(s)


def sub_group(first: bool) -> str:
    """a_k = t_k - n_k - borrow over 16 limbs; borrow in/out as a 0/1 VGPR (%[bw])."""
    s = [] if first else ["v_cmp_ne_u32 vcc, 0, %[bw]"]
    # gfx9 constant-bus limit: an SGPR operand plus the VCC carry-in is two scalar reads,
    # so N_k goes through a VGPR (v0) first.
    for k in range(G):
        s.append(f"v_mov_b32 v0, %[n{k}]")
        if first and k == 0:
            s.append(f"v_sub_co_u32 %[a{k}], vcc, %[t{k}], v0")
        else:
            s.append(f"v_subb_co_u32 %[a{k}], vcc, %[t{k}], v0, vcc")
    s.append("v_cndmask_b32 %[bw], 0, 1, vcc")
    return "\\n\\t".join(s)


def first_group_tpi2() -> str:
    """TPI=2 (an element spread over lanes l and l+32, 64 limbs each): limbs 0..15 of one
    CIOS row.  m is computed in the low half and broadcast to the high half with
    v_permlane32_swap; the reduction chain's j=0 low word %[x] is kept (the high half
    sends it to the low half at the end of the row).  N is a per-lane VGPR operand."""
    s = [
        "v_mad_u64_u32 v[2:3], vcc, %[a0], %[b], 0",
        "v_add_co_u32 %[t0], vcc, %[t0], v2",
        "v_addc_co_u32 v0, vcc, v3, 0, vcc",
        "v_mov_b32 v1, 0",
        "v_mul_lo_u32 %[m], %[t0], %[ninv]",
        "v_mov_b32 v4, %[m]",
        "s_nop 1",
        "v_permlane32_swap_b32 %[m], v4",   # gfx950: vdst[32..63] <-> vsrc[0..31] => m[32..63] = m[0..31]
        "s_nop 1",
        "v_mov_b32 v5, 0",
        "v_mov_b32 v4, %[t0]",
        "v_mad_u64_u32 v[6:7], %[k2], %[m], %[n0], v[4:5]",
        "v_mov_b32 %[x], v6",
        "v_mov_b32 v4, v7",
    ]
    for k in range(1, G):
        s += [
            f"v_mad_u64_u32 v[2:3], vcc, %[a{k}], %[b], v[0:1]",
            f"v_mad_u64_u32 v[6:7], %[k2], %[m], %[n{k}], v[4:5]",
            f"v_add_co_u32 %[t{k}], vcc, %[t{k}], v2",
            "v_addc_co_u32 v0, vcc, v3, 0, vcc",
            f"v_add_co_u32 %[t{k-1}], %[k2], %[t{k}], v6",
            "v_addc_co_u32 v4, %[k2], v7, 0, %[k2]",
        ]
    s += ["v_mov_b32 %[c1], v0", "v_mov_b32 %[c2], v4"]
    return "\\n\\t".join(s)


def tail_tpi2() -> str:
    """End of a TPI=2 row: the high half's reduction low word x goes to the low half
    (v_permlane32_swap), then every lane forms T[63] = lo(xs + c1 + c2 + e0), e0 = hi(...)
    -- the low half's e0 is the carry pending at global limb 64, the high half's e0 is
    global limb 128."""
    s = [
        "v_mov_b32 v2, 0",
        "v_mov_b32 v3, %[x]",
        "s_nop 1",
        "v_permlane32_swap_b32 v3, v2",     # v2[0..31] <- x[32..63]; v2[32..63] stays 0
        "s_nop 1",
        "v_add_co_u32 v2, vcc, v2, %[c1]",
        "v_addc_co_u32 v3, vcc, 0, 0, vcc",
        "v_add_co_u32 v2, vcc, v2, %[c2]",
        "v_addc_co_u32 v3, vcc, v3, 0, vcc",
        "v_add_co_u32 %[tl], vcc, v2, %[e0]",
        "v_addc_co_u32 %[e0], vcc, v3, 0, vcc",
    ]
    return "\\n\\t".join(s)


def addsmall_group(first: bool) -> str:
    """t_k += carry chain over 16 limbs; first group adds %[z] at limb 0.  Carry in/out
    as a 0/1 VGPR %[cw]."""
    s = []
    for k in range(G):
        if first and k == 0:
            s.append("v_add_co_u32 %[t0], vcc, %[t0], %[z]")
        else:
            if not first and k == 0:
                s.append("v_cmp_ne_u32 vcc, 0, %[cw]")
            s.append(f"v_addc_co_u32 %[t{k}], vcc, %[t{k}], 0, vcc")
    s.append("v_cndmask_b32 %[cw], 0, 1, vcc")
    return "\\n\\t".join(s)


def subv_group() -> str:
    """a_k = t_k - n_k - borrow over 16 limbs, N in VGPRs; borrow in/out in %[bw]."""
    s = ["v_cmp_ne_u32 vcc, 0, %[bw]"]
    for k in range(G):
        s.append(f"v_subb_co_u32 %[a{k}], vcc, %[t{k}], %[n{k}], vcc")
    s.append("v_cndmask_b32 %[bw], 0, 1, vcc")
    return "\\n\\t".join(s)


def main() -> None:
    out = []
    out.append("// GENERATED by tools/gen_mont_asm.py -- do not edit by hand.")
    out.append("#pragma once")
    out.append(f"#define FPHE_MAC_G {G}")
    out.append(f'#define FPHE_ASM_STD_GROUP "{std_group()}"')
    out.append(f'#define FPHE_ASM_FIRST_GROUP "{first_group()}"')
    # operand lists (named) as macros taking the C++ array expressions
    t_std = ", ".join(f'[t{k}] "+v"(T[J0 - 1 + {k}])' for k in range(G + 1))
    a_std = ", ".join(f'[a{k}] "v"(A[J0 + {k}])' for k in range(G))
    n_std = ", ".join(f'[n{k}] "s"(NR[J0 + {k}])' for k in range(G))
    out.append("#define FPHE_STD_OUTS(T, J0, C1, C2, K2) " + t_std + ', [c1] "+v"(C1), [c2] "+v"(C2), [k2] "=&s"(K2)')
    out.append("#define FPHE_STD_INS(A, NR, J0, B, M) " + a_std + ", " + n_std + ', [b] "v"(B), [m] "v"(M)')
    t_first = ", ".join(f'[t{k}] "+v"(T[{k}])' for k in range(G))
    a_first = ", ".join(f'[a{k}] "v"(A[{k}])' for k in range(G))
    n_first = ", ".join(f'[n{k}] "s"(NR[{k}])' for k in range(G))
    out.append("#define FPHE_FIRST_OUTS(T, C1, C2, M, K2) " + t_first +
               ', [c1] "=&v"(C1), [c2] "=&v"(C2), [m] "=&v"(M), [k2] "=&s"(K2)')
    out.append("#define FPHE_FIRST_INS(A, NR, B, NINV) " + a_first + ", " + n_first + ', [b] "v"(B), [ninv] "s"(NINV)')
    out.append(f'#define FPHE_ASM_SUB_FIRST "{sub_group(True)}"')
    out.append(f'#define FPHE_ASM_SUB_STD "{sub_group(False)}"')
    a_sub = ", ".join(f'[a{k}] "=&v"(A[J0 + {k}])' for k in range(G))
    tn_sub = ", ".join(f'[t{k}] "v"(T[J0 + {k}])' for k in range(G)) + ", " + \
        ", ".join(f'[n{k}] "s"(NR[J0 + {k}])' for k in range(G))
    out.append("#define FPHE_SUB_OUTS(A, J0, BW) " + a_sub + ', [bw] "+v"(BW)')
    out.append("#define FPHE_SUB_INS(T, NR, J0) " + tn_sub)
    out.append(f'#define FPHE_ASM_FIRST_GROUP_TPI2 "{first_group_tpi2()}"')
    out.append(f'#define FPHE_ASM_TAIL_TPI2 "{tail_tpi2()}"')
    nv_first = ", ".join(f'[n{k}] "v"(NV[{k}])' for k in range(G))
    nv_std = ", ".join(f'[n{k}] "v"(NV[J0 + {k}])' for k in range(G))
    out.append("#define FPHE_FIRST2_OUTS(T, C1, C2, M, X, K2) " + t_first +
               ', [c1] "=&v"(C1), [c2] "=&v"(C2), [m] "=&v"(M), [x] "=&v"(X), [k2] "=&s"(K2)')
    out.append("#define FPHE_FIRST2_INS(A, NV, B, NINV) " + a_first + ", " + nv_first + ', [b] "v"(B), [ninv] "s"(NINV)')
    out.append("#define FPHE_STD2_INS(A, NV, J0, B, M) " + a_std + ", " + nv_std + ', [b] "v"(B), [m] "v"(M)')
    out.append('#define FPHE_TAIL2_OUTS(TL, E0) [tl] "=&v"(TL), [e0] "+v"(E0)')
    out.append('#define FPHE_TAIL2_INS(X, C1, C2) [x] "v"(X), [c1] "v"(C1), [c2] "v"(C2)')
    out.append(f'#define FPHE_ASM_ADDSMALL_FIRST "{addsmall_group(True)}"')
    out.append(f'#define FPHE_ASM_ADDSMALL_STD "{addsmall_group(False)}"')
    t_j = ", ".join(f'[t{k}] "+v"(T[J0 + {k}])' for k in range(G))
    out.append("#define FPHE_ADDSMALL_OUTS(T, J0, CW) " + t_j + ', [cw] "+v"(CW)')
    out.append(f'#define FPHE_ASM_SUBV "{subv_group()}"')
    tv = ", ".join(f'[t{k}] "v"(T[J0 + {k}])' for k in range(G)) + ", " + \
        ", ".join(f'[n{k}] "v"(NV[J0 + {k}])' for k in range(G))
    out.append("#define FPHE_SUBV_INS(T, NV, J0) " + tv)
    out.append('#define FPHE_MAC_CLOBBERS "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "vcc"')
    print("\n".join(out))


if __name__ == "__main__":
    main()
