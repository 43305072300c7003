"""Time the device wire codec (fate_amd/wire.py) on 2^20 2048-bit ciphertexts: encode to
the reference's bincode pickle bytes (incl. D2H) and parse back (incl. the host header walk
and H2D); checks the round trip."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from fate_amd import paillier as P, wire  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
fx = json.load(open(os.path.join(ROOT, "tests", "golden", "paillier_2048.json")))
sk, pk, coder = P.keypair_from_primes(int(fx["p"], 16), int(fx["q"], 16))
g = torch.Generator().manual_seed(20241218)
x = (torch.randn(N, generator=g) * 4).cuda()
a = pk.encrypt_encoded(coder.encode_f32_vec(x), True)
b = a  # obfuscated encryptions of negative floats are negative integers (sign 1)
for rep in range(3):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    buf = wire.ciphertext_vector_to_bincode(b, pk)
    t1 = time.perf_counter()
    back, used = wire.ciphertext_vector_from_bincode(buf, pk)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    same = torch.equal(back.C[: (N + 63) // 64], b.C[: (N + 63) // 64]) and torch.equal(back.sign[:N], b.sign[:N]) \
        and torch.equal(back.exp[:N], b.exp[:N])
    print(json.dumps({"rep": rep, "N": N, "bytes": len(buf), "encode_s": round(t1 - t0, 4),
                      "decode_s": round(t2 - t1, 4), "encode_MBps": round(len(buf) / (t1 - t0) / 1e6),
                      "decode_MBps": round(len(buf) / (t2 - t1) / 1e6), "round_trip_equal": bool(same),
                      "negatives": int(b.sign[:N].sum())}), flush=True)
