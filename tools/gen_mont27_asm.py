"""Generate fate_amd/csrc/mont_gen_ll38.h (27-bit limbs, 38 per lane) and mont_gen_ll37.h
(28-bit limbs, 37 per lane): the CIOS rows of the reduced-radix engine as asm blocks, each
MAC one v_mad_u64_u32 on a 64-bit lazy accumulator.  Emitting a whole row per asm
statement keeps the compiler's conservative inline-asm hazard padding (s_nop) at block
boundaries instead of between every MAC.

Each file has sections, picked by RG_SECTION before each #include (mont_engine.inc):
  1  macros   RG_OPROW      t_j += a_j * b                          (LL MACs, general product)
              RG_REDROW     x = m n_0 + t_0 ; t_{j-1} = m n_j + t_j  (LL MACs, reduction + shift)
              RG_SQROW_<a>  the squaring row for lane-slice row index a (0 <= a < LL): MACs on
                            the circular window of positions (a + s) mod LL, s = 0..W-1 with
                            W = LL/2 + 1, multiplier bf at s = 0, bm inside, and for even LL
                            bl at s = W-1 (odd LL needs no half-window column).  See
                            mont_engine.inc mont_sqr for why this covers each limb pair once.
              RGF_ROW / RGF_SQROW_<a>  fused rows (below)
              RG_OPROW_Z / RG_REDROW_Z / RG_SQROZ_<a>, RG_OPROW_F / RG_SQROW_F0 / RG_REDROW_F0
                            TPI-1 rows that keep t_{LL-1} logically zero and a product's first
                            rows over an all-zero accumulator (no 64-bit zero stores)
  2  dispatchers r27_sqrow<a>, r27_sqrow_z<a>, r27_sqrow_f0   (after the limb vector type)
  3  dispatchers r27f_sqrow<TPI, a>, r27f_row<TPI>  (after Mod)
  4  #undef of every macro of section 1, so the other radix can define them again
"""
import os

HERE = os.path.dirname(__file__)


def sq_window(LL, a):
    """(lane-local position, multiplier) of squaring row a: positions (a + s) mod LL for
    s < LL/2 + 1; bf at s = 0, bl at the last s when LL is even, bm otherwise."""
    WIN = LL // 2 + 1
    pos = []
    for s in range(WIN):
        k = (a + s) % LL
        if s == 0:
            mul = "bf"
        elif s == WIN - 1 and LL % 2 == 0:
            mul = "bl"
        else:
            mul = "bm"
        pos.append((k, mul))
    pos.sort()  # ascending position: t0 (read next by the m computation) is written first
    return pos


def gen(LL, LB):
    def window(a):
        return sq_window(LL, a)

    macros = []
    row = "".join(f'"v_mad_u64_u32 %[t{j}], vcc, %[a{j}], %[b], %[t{j}]\\n\\t" ' for j in range(LL))
    macros.append(("RG_OPROW", row))
    red = '"v_mad_u64_u32 %[x], vcc, %[m], %[n0], %[t0]\\n\\t" '
    red += "".join(f'"v_mad_u64_u32 %[t{j-1}], vcc, %[m], %[n{j}], %[t{j}]\\n\\t" ' for j in range(1, LL))
    macros.append(("RG_REDROW", red))
    for a in range(LL):
        body = "".join(f'"v_mad_u64_u32 %[t{k}], vcc, %[a{k}], %[{mul}], %[t{k}]\\n\\t" ' for k, mul in window(a))
        macros.append((f"RG_SQROW_{a}", body))
    # TPI-1 rows with the top accumulator limb kept logically zero instead of zeroed after every
    # reduction row (FPHE_TPI1_TOPZ, mont_engine.inc): the operand row writing t_{LL-1} first
    # adds to the constant 0 (its operand is output-only), and a reduction row after an operand
    # row that left t_{LL-1} alone reads 0 in its place
    top = LL - 1
    macros.append(("RG_OPROW_Z", "".join(
        f'"v_mad_u64_u32 %[t{j}], vcc, %[a{j}], %[b], {"0" if j == top else f"%[t{j}]"}\\n\\t" ' for j in range(LL))))
    macros.append(("RG_REDROW_Z", red.replace(f"%[t{top}]\\n", "0\\n")))
    for a in range(LL):
        if any(k == top for k, _ in window(a)):
            body = "".join(f'"v_mad_u64_u32 %[t{k}], vcc, %[a{k}], %[{mul}], {"0" if k == top else f"%[t{k}]"}\\n\\t" '
                           for k, mul in window(a))
            macros.append((f"RG_SQROZ_{a}", body))
    # ... and a product's first rows over an accumulator that is still all zero, so no
    # 64-bit zero stores start the product: RG_OPROW_F writes every limb over 0, RG_SQROW_F0
    # squaring row 0's window over 0, RG_REDROW_F0 the reduction row after it (reads 0 for the
    # limbs outside that window)
    live0 = sorted(k for k, _ in window(0))
    macros.append(("RG_OPROW_F", "".join(f'"v_mad_u64_u32 %[t{j}], vcc, %[a{j}], %[b], 0\\n\\t" ' for j in range(LL))))
    macros.append(("RG_SQROW_F0", "".join(f'"v_mad_u64_u32 %[t{k}], vcc, %[a{k}], %[{mul}], 0\\n\\t" ' for k, mul in window(0))))
    redf = '"v_mad_u64_u32 %[x], vcc, %[m], %[n0], %[t0]\\n\\t" '
    redf += "".join(f'"v_mad_u64_u32 %[t{j-1}], vcc, %[m], %[n{j}], {f"%[t{j}]" if j in live0 else "0"}\\n\\t" '
                    for j in range(1, LL))
    macros.append(("RG_REDROW_F0", redf))
    macros.append(("RG_T_OUT_ALL(T)", ", ".join(f'[t{j}] "=&v"(T[{j}])' for j in range(LL))))
    macros.append(("RG_T_SQ0_OUT(T)", ", ".join(f'[t{k}] "=&v"(T[{k}])' for k in live0)))
    macros.append(("RG_T_F0_OPS(T)", ", ".join(
        f'[t{j}] "+v"(T[{j}])' if j in live0 else f'[t{j}] "=&v"(T[{j}])' for j in range(LL - 1))))
    macros.append(("RG_T_TOP_OUT(T)", f'[t{top}] "=&v"(T[{top}])'))
    macros.append(("RG_T_OPS_LO(T)", ", ".join(f'[t{j}] "+v"(T[{j}])' for j in range(LL - 1))))
    macros.append(("RG_T_OPS(T)", ", ".join(f'[t{j}] "+v"(T[{j}])' for j in range(LL))))
    macros.append(("RG_A_INS(A)", ", ".join(f'[a{j}] "v"(A[{j}])' for j in range(LL))))
    macros.append(("RG_N_INS(N, C)", ", ".join(f'[n{j}] C(N({j}))' for j in range(LL))))

    # ---- fused rows: operand MACs + m + reduction MACs + the X fix-up in ONE asm block ---
    # The accumulator limbs 0 and LL-1 are pinned to v[2:3] / v[4:5] and the row's
    # temporaries to v6..v11, so the block can address their 32-bit halves (inline asm has no
    # sub-register syntax).  Order inside the block:
    #   t0's operand MAC (if the row has one) -> v_mul_lo (m = t0 n' mod 2^LB, broadcast from
    #   the element's lane 0 by the DPP AND) issued under the remaining operand MACs, then the
    #   reduction MACs with X = m n0 + t0 first; X >> LB is added to the new t0 in the shadow
    #   of the later MACs, and X mod 2^LB moves to the lane below's top limb with a DPP AND.
    # Hazards honoured by construction: >= 2 VALU instructions between the VALU write of v10
    # and its DPP read; X (v6) is written ~LL instructions before its DPP read.
    # BC is the DPP broadcast control string for TPI (quad_perm:[0,0,0,0] / [0,0,2,2]).
    def treg(k):
        return "v[2:3]" if k == 0 else ("v[4:5]" if k == LL - 1 else f"%[t{k}]")

    def fused(pos, spread, carry64=True, half_row=False):
        # half_row (TPI 8): the element spans 8 lanes, so m's broadcast takes a second DPP
        # step -- the upper quad of each half row (banks 1, 3) copies the lower quad's value
        # by row_half_mirror -- at least two VALU instructions after the first (DPP read of a
        # VALU-written VGPR), still ahead of the reduction MACs that read m
        m_gap, x_gap, c_gap = spread
        opm = [f"v_mad_u64_u32 {treg(k)}, vcc, %[a{k}], %[{mul}], {treg(k)}" for k, mul in pos]
        seq = []
        if pos and pos[0][0] == 0:
            seq.append(opm.pop(0))
        seq.append("v_mul_lo_u32 v10, v2, %[np]")
        lead = opm[:m_gap]
        seq += lead
        if len(lead) < 2:
            seq.append("s_nop 1")
        seq.append("@BC@")
        rest = opm[m_gap:]
        if half_row:
            seq += rest[:2]
            if len(rest) < 2:
                seq.append("s_nop 1")
            seq.append("v_mov_b32_dpp v11, v11 row_half_mirror row_mask:0xf bank_mask:0xa")
            rest = rest[2:]
        seq += rest
        redm = [f"v_mad_u64_u32 {treg(j - 1)}, vcc, v11, %[n{j}], {treg(j)}" for j in range(1, LL)]
        seq.append("v_mad_u64_u32 v[6:7], vcc, v11, %[n0], v[2:3]")
        seq += redm[:x_gap]
        # X >> LB: one 64-bit shift (v_alignbit_b32 is half rate on gfx950 like the shift,
        # tools/probe/instr_probe.hip) -- same-box +2.9% for the TPI-4 kernels -- or the
        # alignbit + lshrrev pair, which the TPI-2 kernels keep (the shift measured -1% there,
        # profiles/r02/r02z15_ab_carry_per_tpi.txt)
        if carry64:
            seq.append(f"v_lshrrev_b64 v[8:9], {LB}, v[6:7]")
        else:
            seq.append(f"v_alignbit_b32 v8, v7, v6, {LB}")
            seq.append(f"v_lshrrev_b32 v9, {LB}, v7")
        seq += redm[x_gap:x_gap + c_gap]
        seq.append("v_lshl_add_u64 v[2:3], v[8:9], 0, v[2:3]")
        seq += redm[x_gap + c_gap:]
        seq.append("v_and_b32_dpp v4, v6, %[mk] row_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1")
        seq.append("v_mov_b32 v5, 0")
        parts = []
        for s_ in seq:
            if s_ == "@BC@":
                parts.append('"v_and_b32_dpp v11, v10, %[mk] " BC " row_mask:0xf bank_mask:0xf\\n\\t"')
            else:
                parts.append(f'"{s_}\\n\\t"')
        return " ".join(parts)

    macros.append(("RGF_T_OPS(T)", f'[t0p] "+{{v[2:3]}}"(T[0]), [tlp] "+{{v[4:5]}}"(T[{LL - 1}]), '
                   + ", ".join(f'[t{j}] "+v"(T[{j}])' for j in range(1, LL - 1))))
    macros.append(("RGF_CLOB", '"v6", "v7", "v8", "v9", "v10", "v11", "vcc", "memory"'))
    # FPHE_FUSED_SPREAD selects the instruction spacing of the two dependency chains
    SPREADS = {0: (3, 2, 1), 1: (6, 8, 8)}
    spread_macros = {}
    for sp, spread in SPREADS.items():
        lst = []
        # RGF: TPI 4 rows, RGF2: TPI 2 rows, RGF8: TPI 8 rows (keys above 2048 bits)
        for fam, c64, hr in (("RGF", True, False), ("RGF2", False, False), ("RGF8", True, True)):
            lst.append((f"{fam}_ROW(BC)", fused([(k, "b") for k in range(LL)], spread, c64, hr)))
            for a in range(LL):
                lst.append((f"{fam}_SQROW_{a}(BC)", fused(window(a), spread, c64, hr)))
        spread_macros[sp] = lst

    out = [f"// Generated by tools/gen_mont27_asm.py -- do not edit.  {LL} limbs of {LB} bits per lane.",
           "// No include guard: included once per section (RG_SECTION) by mont_engine.inc.",
           "#if RG_SECTION == 1"]
    for name, body in macros:
        out.append(f"#define {name} {body}")
    out.append("#ifndef FPHE_FUSED_SPREAD")
    out.append("#define FPHE_FUSED_SPREAD 1")
    out.append("#endif")
    for sp, lst in spread_macros.items():
        out.append(f"#if FPHE_FUSED_SPREAD == {sp}")
        for name, body in lst:
            out.append(f"#define {name} {body}")
        out.append("#endif")
    out.append("#elif RG_SECTION == 2")
    sig = "u64 (&T)[LL], const L27& A, u32 bf, u32 bm, u32 bl"
    out.append(f"template <int a> __device__ __forceinline__ void r27_sqrow({sig});")
    for a in range(LL):
        out.append(f"template <> __device__ __forceinline__ void r27_sqrow<{a}>({sig}) {{")
        bl_in = ', [bl] "v"(bl)' if LL % 2 == 0 else ''  # odd LL: no half-window column, bl unused
        out.append(f'  asm volatile(RG_SQROW_{a} : RG_T_OPS(T) : RG_A_INS(A), [bf] "v"(bf), [bm] "v"(bm){bl_in} : "vcc", "memory");')
        out.append("}")
    # TPI-1 top-zero dispatchers (rows whose window holds t_{LL-1} write it over the constant 0)
    out.append(f"template <int a> __device__ __forceinline__ void r27_sqrow_z({sig});")
    for a in range(LL):
        out.append(f"template <> __device__ __forceinline__ void r27_sqrow_z<{a}>({sig}) {{")
        bl_in = ', [bl] "v"(bl)' if LL % 2 == 0 else ''
        if any(k == LL - 1 for k, _ in window(a)):
            out.append(f'  asm volatile(RG_SQROZ_{a} : RG_T_OPS_LO(T), [t{LL - 1}] "=&v"(T[{LL - 1}]) : RG_A_INS(A), [bf] "v"(bf), [bm] "v"(bm){bl_in} : "vcc", "memory");')
        else:
            out.append(f'  asm volatile(RG_SQROW_{a} : RG_T_OPS_LO(T) : RG_A_INS(A), [bf] "v"(bf), [bm] "v"(bm){bl_in} : "vcc", "memory");')
        out.append("}")
    bl_in = ', [bl] "v"(bl)' if LL % 2 == 0 else ''
    out.append(f"__device__ __forceinline__ void r27_sqrow_f0({sig}) {{")
    out.append(f'  asm volatile(RG_SQROW_F0 : RG_T_SQ0_OUT(T) : RG_A_INS(A), [bf] "v"(bf), [bm] "v"(bm){bl_in} : "vcc", "memory");')
    out.append("}")
    out.append("#elif RG_SECTION == 3")
    out.append("template <int TPI, int a> __device__ __forceinline__ void r27f_sqrow(u64 (&T)[LL], const L27& A, u32 bf, u32 bm, u32 bl, const Mod<TPI>& N, u32 np, u32 mk);")
    # TPI 1 (one lane per element: p^2, q^2 and n of <= 1024-bit keys) runs the TPI-4 rows with
    # an identity DPP for m (the lane is its element's lane 0) and the modulus limbs in SGPRs
    # (wave-uniform); the X hand-off from the next lane is that element's lane-0 X, which is
    # 0 mod 2^LB, so no select is needed there either
    tpis = ((4, "quad_perm:[0,0,0,0]", "RGF", "v"), (2, "quad_perm:[0,0,2,2]", "RGF2", "v"),
            (8, "quad_perm:[0,0,0,0]", "RGF8", "v"), (1, "quad_perm:[0,1,2,3]", "RGF", "s"))
    for a in range(LL):
        for tpi, bc, fam, nc in tpis:
            out.append(f"template <> __device__ __forceinline__ void r27f_sqrow<{tpi}, {a}>(u64 (&T)[LL], const L27& A, u32 bf, u32 bm, u32 bl, const Mod<{tpi}>& N, u32 np, u32 mk) {{")
            bl_in = ' [bl] "v"(bl),' if LL % 2 == 0 else ''
            out.append(f'  asm volatile({fam}_SQROW_{a}("{bc}") : RGF_T_OPS(T) : RG_A_INS(A), RG_N_INS(N, "{nc}"), [bf] "v"(bf), [bm] "v"(bm),{bl_in} [np] "s"(np), [mk] "v"(mk) : RGF_CLOB);')
            out.append("}")
    out.append("template <int TPI> __device__ __forceinline__ void r27f_row(u64 (&T)[LL], const L27& A, u32 b, const Mod<TPI>& N, u32 np, u32 mk);")
    for tpi, bc, fam, nc in tpis:
        out.append(f"template <> __device__ __forceinline__ void r27f_row<{tpi}>(u64 (&T)[LL], const L27& A, u32 b, const Mod<{tpi}>& N, u32 np, u32 mk) {{")
        out.append(f'  asm volatile({fam}_ROW("{bc}") : RGF_T_OPS(T) : RG_A_INS(A), RG_N_INS(N, "{nc}"), [b] "v"(b), [np] "s"(np), [mk] "v"(mk) : RGF_CLOB);')
        out.append("}")
    out.append("#elif RG_SECTION == 4")
    names = {n.split("(")[0] for n, _ in macros} | {n.split("(")[0] for lst in spread_macros.values() for n, _ in lst}
    for n in sorted(names):
        out.append(f"#undef {n}")
    out.append("#endif")
    path = os.path.join(HERE, "..", "fate_amd", "csrc", f"mont_gen_ll{LL}.h")
    with open(path, "w") as f:
        f.write("\n".join(out) + "\n")


if __name__ == "__main__":
    gen(38, 27)
    gen(37, 28)
