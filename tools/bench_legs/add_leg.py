"""Time bench.py's Hetero-LR-shaped ct-add (enc(x) + enc(0.25 * flip(x)), 2^20 elements,
2048-bit key) and print the histogram of exponent gaps |ea - eb| (each gap step costs the
higher-exponent operand 4 squarings, decrese_exp_to, lib.rs:250-258)."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from fate_amd import paillier as P  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
fx = json.load(open(os.path.join(ROOT, "tests", "golden", "paillier_2048.json")))
sk, pk, coder = P.keypair_from_primes(int(fx["p"], 16), int(fx["q"], 16))
dev = torch.device("cuda", 0)
g = torch.Generator().manual_seed(20241218)
x = (torch.randn(N, generator=g) * 4).to(dev)
a = pk.encrypt_encoded(coder.encode_f32_vec(x), True)
b = pk.encrypt_encoded(coder.encode_f32_vec(torch.flip(x, [0]) * 0.25), True)


def t(f, *args, **kw):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = f(*args, **kw)
    torch.cuda.synchronize()
    return r, time.perf_counter() - t0


for rep in range(2):
    _, t_plain = t(P._add, pk, a, b, False, N)
    d = (a.exp[:N] - b.exp[:N]).abs()
    print(json.dumps({"rep": rep, "add_s": round(t_plain, 4), "gap_hist": torch.bincount(d.cpu()).tolist()}), flush=True)
