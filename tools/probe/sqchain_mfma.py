"""Driver for tools/probe/sqchain_mfma.hip: S chained 4096-bit Montgomery squarings
(R = 2^4144) per element with the engine's VALU squaring (variant 0) and the MFMA-reduction
squaring (variant 1); checks both against Python integers and times them.

    python tools/probe/sqchain_mfma.py [nelem] [S]
"""
import ctypes
import json
import os
import random
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
LB, NL, D = 28, 148, 592
RBITS = LB * NL
R = 1 << RBITS


def limbs(x, n=NL):
    return [(x >> (LB * i)) & ((1 << LB) - 1) for i in range(n)]


def value(ls):
    return sum(int(v) << (LB * i) for i, v in enumerate(ls))


def digits(x, n):
    return [(x >> (7 * i)) & 127 for i in range(n)]


def tables(N):
    Np = (-pow(N, -1, R)) % R
    npd = digits(Np, D)
    nd = digits(N, D)
    W1 = np.zeros((640, 16), dtype=np.int8)
    for i in range(640):
        b = i - 48
        for j in range(16):
            k = b - j
            W1[i, j] = npd[k] if 0 <= k < D else 0
    W2 = np.zeros((668, 16), dtype=np.int8)
    for i in range(668):
        b = i - 12
        for j in range(16):
            k = b - 16 * (j >> 2) - (j & 3)
            W2[i, j] = nd[k] if 0 <= k < D else 0
    return np.concatenate([W1, W2]).reshape(-1)


def main():
    nelem = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 15
    S = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    rng = random.Random(11)
    N = rng.getrandbits(4096) | (1 << 4095) | 1
    np28 = (-pow(N, -1, 1 << LB)) % (1 << LB)
    nchk = 64
    xs = [rng.randrange(0, 2 * N) for _ in range(nchk - 4)] + [2 * N - 1, 0, 1, N]
    X = np.array([limbs(x) for x in xs], dtype=np.uint32)
    dev = torch.device("cuda", 0)
    Xd = torch.from_numpy(np.tile(X, (nelem // nchk, 1)).view(np.int32)).to(dev)
    Nd = torch.from_numpy(np.array(limbs(N), dtype=np.uint32).view(np.int32)).to(dev)
    Wd = torch.from_numpy(tables(N)).to(dev)
    lib = ctypes.CDLL(os.path.join(HERE, os.environ.get("SQ_LIB", "libsqchain.so")))
    lib.sqchain_launch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint,
                                   ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    stream = torch.cuda.current_stream().cuda_stream
    Rinv = pow(R, -1, N)
    out = {"nelem": nelem, "S": S}
    variants = [int(v) for v in os.environ.get("SQ_VARIANTS", "0,1").split(",")]
    for variant in variants:
        Y = torch.zeros_like(Xd)
        for s_chk in (1, S):
            assert lib.sqchain_launch(variant, Xd.data_ptr(), Y.data_ptr(), Nd.data_ptr(), np28, Wd.data_ptr(),
                                      nchk, s_chk, stream) == 0
            torch.cuda.synchronize()
            Yh = Y[:nchk].cpu().numpy().view(np.uint32)
            bad = big = 0
            for i, x in enumerate(xs):
                exp = x
                for _ in range(s_chk):
                    exp = exp * exp * Rinv % N
                y = value(Yh[i])
                if y % N != exp:
                    bad += 1
                if y >= 2 * N:
                    big += 1
            out[f"v{variant}_S{s_chk}_bad"] = bad
            out[f"v{variant}_S{s_chk}_ge2N"] = big
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        lib.sqchain_launch(variant, Xd.data_ptr(), Y.data_ptr(), Nd.data_ptr(), np28, Wd.data_ptr(), nelem, S, stream)
        e0.record()
        assert lib.sqchain_launch(variant, Xd.data_ptr(), Y.data_ptr(), Nd.data_ptr(), np28, Wd.data_ptr(), nelem,
                                  S, stream) == 0
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        out[f"v{variant}_ms"] = round(ms, 3)
        out[f"v{variant}_ns_per_sqr"] = round(ms * 1e6 / (nelem * S), 4)
    st = (ctypes.c_ulonglong * 5)()
    if lib.sqchain_stamps(st) == 0:
        # totals over every wave of every launch of variant 1 (checks + warm-up + timed)
        tot = sum(st)
        out["phase_share"] = {k: round(st[i] / tot, 3) for i, k in
                              enumerate(["A_rows", "tfrag_Hstore", "product1_q", "product2_U", "phaseC"])}
    if 4 in variants:
        ro = (ctypes.c_int * 16)()
        lib.sqchain_roles(ro)
        out["v4_roles_simd_k"] = [(r >> 4, r & 15) for r in ro[:12]]
    if "v0_ms" in out and "v1_ms" in out:
        out["speedup_mfma"] = round(out["v0_ms"] / out["v1_ms"], 3)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
