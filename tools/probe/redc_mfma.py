"""Driver for tools/probe/redc_mfma.hip (round-2 research spike): builds a random 4096-bit N,
products T < 4N^2, the balanced base-256 digits and the MFMA A fragments, runs the batched
reduction `reps` times per element, checks U = (T + qN)/R exactly on a sample against
Python integers, and prints the time per reduction (and per element in SIMD cycles).

    python tools/probe/redc_mfma.py [nelem] [reps]
"""
import ctypes
import json
import os
import random
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
D, TD, QT, NA1, NA2 = 544, 1088, 17, 17, 18
R = 1 << (8 * D)


def bal_digits(x, n):
    out = []
    for _ in range(n):
        d = x & 255
        if d >= 128:
            d -= 256
        out.append(d)
        x = (x - d) >> 8
    assert x == 0 or x == -1 and False, "did not fit"
    return out


def value(ds):
    return sum(d << (8 * k) for k, d in enumerate(ds))


def main():
    nelem = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 17
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    rng = random.Random(5)
    N = rng.getrandbits(4096) | (1 << 4095) | 1
    Np = (-pow(N, -1, R)) % R
    nd = bal_digits(N, 576)
    npd = bal_digits(Np if Np < R // 2 else Np - R, D) + [0] * 32
    # fragments: lane l = 32h + r holds A[row r][k = 16h + j] in byte j
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
                pos = (j & 3) + 8 * (j >> 2) + 4 * h  # q's position for B byte j of half h
                idx = 32 * d + r - pos
                frag[NA1 + d, l, j] = nd[idx] if 0 <= idx < len(nd) else 0
    # T values: a sample of exact ones, the rest copies (timing only)
    nchk = 64
    Ts = [rng.randrange(0, 4 * N * N) for _ in range(nchk)]
    tdig = np.array([bal_digits(t, TD) for t in Ts], dtype=np.int8)  # [64][1088]
    # fragment order per batch of 32 elements: [tile 34][lane 64][16], lane = 32h + e holds
    # positions 32*tile + 16h + j of element e
    def frag_order(block):  # block [32][1088]
        x = block.reshape(32, 34, 2, 16)          # e, tile, h, j
        return np.ascontiguousarray(x.transpose(1, 2, 0, 3)).reshape(-1)
    one = np.concatenate([frag_order(tdig[0:32]), frag_order(tdig[32:64])])
    tall = np.tile(one, nelem // nchk)
    dev = torch.device("cuda", 0)
    A = torch.from_numpy(frag.reshape(-1)).to(dev)
    T = torch.from_numpy(tall.reshape(-1)).to(dev)
    U = torch.zeros(nelem * 544, dtype=torch.int32, device=dev)
    lib = ctypes.CDLL(os.path.join(HERE, os.environ.get("REDC_LIB", "libredc_mfma.so")))
    lib.redc_launch.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                                         ctypes.c_void_p]
    grid = max(1, nelem // 32 // 4)
    stream = torch.cuda.current_stream().cuda_stream
    # correctness, one rep
    dbg = torch.zeros(nelem * 544, dtype=torch.int32, device=dev)
    assert lib.redc_launch(A.data_ptr(), T.data_ptr(), U.data_ptr(), nelem, 1, grid, dbg.data_ptr(), stream) == 0
    torch.cuda.synchronize()
    # U: [batch][tile 17][reg 16][lane 64] -> [elem][pos]: lane = 32h + e, pos = 32t + (r&3) + 8(r>>2) + 4h
    Ub = U[: nchk * 544].view(nchk // 32, 17, 16, 2, 32).cpu().numpy().astype(np.int64)
    Uh = np.zeros((nchk, 544), dtype=np.int64)
    for bb in range(nchk // 32):
        for t in range(17):
            for r in range(16):
                for h in range(2):
                    pos = 32 * t + (r & 3) + 8 * (r >> 2) + 4 * h
                    Uh[bb * 32: bb * 32 + 32, pos] = Ub[bb, t, r, h]
    Uh += tdig[:, 544:].astype(np.int64)  # T_high (the kernel leaves it to the caller)
    Qh = dbg[: nchk * 544].view(nchk, 544).cpu().numpy().astype(np.int64)
    qbad = 0
    for i, t in enumerate(Ts):
        q = ((t % R) * Np) % R
        qd = bal_digits(q if q < R // 2 else q - R, D)
        if list(Qh[i]) != qd:
            qbad += 1
            if qbad == 1:
                diff = [k for k in range(D) if Qh[i][k] != qd[k]]
                print("q mismatch elem", i, "first positions", diff[:10], [int(Qh[i][k]) for k in diff[:5]], [qd[k] for k in diff[:5]])
    print("q digit mismatches:", qbad, "of", nchk)
    bad = 0
    for i, t in enumerate(Ts):
        tv = value([int(x) for x in tdig[i]])
        assert tv == t
        q = ((t % R) * Np) % R
        if q >= R // 2:
            q -= R
        want = (t + q * N)
        assert want % R == 0
        want //= R
        got = value([int(x) for x in Uh[i]])
        if got != want:
            bad += 1
    ok = bad == 0
    # timing
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    lib.redc_launch(A.data_ptr(), T.data_ptr(), U.data_ptr(), nelem, reps, grid, None, stream)
    e0.record()
    assert lib.redc_launch(A.data_ptr(), T.data_ptr(), U.data_ptr(), nelem, reps, grid, None, stream) == 0
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    per = ms / 1e3 / (nelem * reps)
    print(json.dumps({"exact": ok, "mismatches": bad, "nelem": nelem, "reps": reps, "ms": round(ms, 3),
                      "ns_per_redc_elem": round(per * 1e9, 4),
                      "simd_cycles_per_elem_at_2.3GHz": round(per * 2.3e9 * 1024, 1),
                      "mfma_per_32_elems": 153 + 153}))


if __name__ == "__main__":
    main()
