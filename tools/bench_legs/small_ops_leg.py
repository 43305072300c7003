"""Latency of the element-wise ops on few elements (2048-bit key): ct-add, ct x pt (float
weights of both signs: the invert branch), neg, sub, and a small iupdate -- the shapes of a
Hetero-LR gradient (features-long vectors) and of per-node histogram work.  One JSON line;
each figure is the best of 3 synchronised calls after a warm-up call."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from fate_amd import paillier as P  # noqa: E402

fx = json.load(open(os.path.join(ROOT, "tests", "golden", "paillier_2048.json")))
sk, pk, coder = P.keypair_from_primes(int(fx["p"], 16), int(fx["q"], 16), keyholder=False)
dev = torch.device("cuda", 0)
g = torch.Generator().manual_seed(9)


def best(f):
    f()
    torch.cuda.synchronize(dev)
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        f()
        torch.cuda.synchronize(dev)
        ts.append(time.perf_counter() - t0)
    return round(min(ts) * 1e3, 3)


out = {}
for n in (16, 256, 4096):
    a = pk.encrypt_encoded(coder.encode_f64_vec(torch.randn(n, generator=g, dtype=torch.float64).to(dev)), True)
    b = pk.encrypt_encoded(coder.encode_f64_vec((torch.randn(n, generator=g, dtype=torch.float64) * 1e-3).to(dev)), True)
    w = coder.encode_f64_vec(torch.randn(n, generator=g, dtype=torch.float64).to(dev))
    out[f"add_{n}_ms"] = best(lambda: a.add(pk, b))
    out[f"mul_{n}_ms"] = best(lambda: a.mul(pk, w))
    out[f"neg_{n}_ms"] = best(lambda: a.neg(pk))
    out[f"sub_{n}_ms"] = best(lambda: a.sub(pk, b))
    hist = P.CiphertextVector.zeros(64, pk._key.L2, dev)
    pos = torch.randint(0, 32, (n // 2, 1), generator=g).to(dev, torch.int32)
    out[f"iupdate_{n}_terms_ms"] = best(lambda: hist.iupdate(a, pos, 2, pk))
print(json.dumps(out), flush=True)
