"""Driver for tools/probe/redc_mfma7.hip (base-128 digits, parallel carry-save normalisation
of q): checks q = T N' (mod R) and U = (T + qN)/R exactly on a sample against Python
integers and times `reps` reductions per element.

    [REDC_LIB=libredc_mfma7_w1.so] python tools/probe/redc_mfma7.py [nelem] [reps]
"""
import ctypes
import json
import os
import random
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
B, D, QT, TT, NA1, NA2 = 128, 608, 19, 38, 19, 20
R = B ** D


def bal(x, n):
    out = []
    for _ in range(n):
        d = x % B
        if d >= B // 2:
            d -= B
        out.append(d)
        x = (x - d) // B
    assert x == 0, "did not fit"
    return out


def value(ds):
    return sum(int(d) * B ** k for k, d in enumerate(ds))


def main():
    nelem = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 17
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    rng = random.Random(5)
    N = rng.getrandbits(4096) | (1 << 4095) | 1
    Np = (-pow(N, -1, R)) % R
    nd = bal(N, 640)
    npd = bal(Np if Np < R // 2 else Np - R, D)
    frag = np.zeros((NA1 + NA2, 64, 16), dtype=np.int8)
    for d in range(NA1):
        for l in range(64):
            r, h = l & 31, l >> 5
            for j in range(16):
                idx = 32 * d + r - (16 * h + j)
                frag[d, l, j] = npd[idx] if 0 <= idx < D else 0
    for d in range(NA2):
        for l in range(64):
            r, h = l & 31, l >> 5
            for j in range(16):
                pos = (j & 3) + 8 * (j >> 2) + 4 * h
                idx = 32 * d + r - pos
                frag[NA1 + d, l, j] = nd[idx] if 0 <= idx < len(nd) else 0
    nchk = 64
    Ts = [rng.randrange(0, 4 * N * N) for _ in range(nchk)]
    tdig = np.array([bal(t, TT * 32) for t in Ts], dtype=np.int8)

    def frag_order(block):
        x = block.reshape(32, TT, 2, 16)
        return np.ascontiguousarray(x.transpose(1, 2, 0, 3)).reshape(-1)

    one = np.concatenate([frag_order(tdig[0:32]), frag_order(tdig[32:64])])
    dev = torch.device("cuda", 0)
    A = torch.from_numpy(frag.reshape(-1)).to(dev)
    T = torch.from_numpy(np.tile(one, nelem // nchk)).to(dev)
    U = torch.zeros(nelem * QT * 32, dtype=torch.int32, device=dev)
    dbg = torch.zeros(nelem * D, dtype=torch.int32, device=dev)
    lib = ctypes.CDLL(os.path.join(HERE, os.environ.get("REDC_LIB", "libredc_mfma7.so")))
    lib.redc7_launch.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int] * 3 + [ctypes.c_void_p, ctypes.c_int,
                                                                             ctypes.c_void_p]
    grid = max(1, nelem // 32 // 4)
    stream = torch.cuda.current_stream().cuda_stream
    assert lib.redc7_launch(A.data_ptr(), T.data_ptr(), U.data_ptr(), nelem, 1, grid, dbg.data_ptr(), 0, stream) == 0
    torch.cuda.synchronize()
    Qh = dbg[: nchk * D].view(nchk, D).cpu().numpy().astype(np.int64)
    Ub = U[: nchk * QT * 32].view(nchk // 32, QT, 16, 2, 32).cpu().numpy().astype(np.int64)
    Uh = np.zeros((nchk, QT * 32), dtype=np.int64)
    for bb in range(nchk // 32):
        for t in range(QT):
            for r in range(16):
                for h in range(2):
                    Uh[bb * 32: bb * 32 + 32, 32 * t + (r & 3) + 8 * (r >> 2) + 4 * h] = Ub[bb, t, r, h]
    Uh += tdig[:, D:D + QT * 32].astype(np.int64)
    qbad = ubad = 0
    maxdig = int(np.abs(Qh).max())
    for i, t in enumerate(Ts):
        q = value(Qh[i])
        if (q - (t % R) * Np) % R:
            qbad += 1
        s = t + q * N
        if s % R or value(Uh[i]) != s // R:
            ubad += 1
    shared = int(os.environ.get("REDC_SHARED_T", "0"))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    lib.redc7_launch(A.data_ptr(), T.data_ptr(), U.data_ptr(), nelem, reps, grid, None, shared, stream)
    e0.record()
    assert lib.redc7_launch(A.data_ptr(), T.data_ptr(), U.data_ptr(), nelem, reps, grid, None, shared, stream) == 0
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    per = ms / 1e3 / (nelem * reps)
    print(json.dumps({"q_congruent": qbad == 0, "U_exact": ubad == 0, "max_q_digit": maxdig, "nelem": nelem,
                      "reps": reps, "ms": round(ms, 3), "ns_per_redc_elem": round(per * 1e9, 4),
                      "simd_cycles_per_elem_at_2.3GHz": round(per * 2.3e9 * 1024, 1), "mfma_per_32_elems": 380,
                      "shared_t": shared}))


if __name__ == "__main__":
    main()
