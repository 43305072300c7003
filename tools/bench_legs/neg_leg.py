"""Time neg and sub (Ciphertext::neg / sub, fixedpoint_paillier/src/lib.rs:259-285) on
2^20 2048-bit ciphertexts.  FPHE_NEG_BATCH_MIN picks the path (read once per process):
unset -> batch inversion from 4096 elements, a huge value -> one safegcd inverse + Hensel
lift per element.  Checks c * neg(c) == 1 (mod n^2) on every element."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from fate_amd import paillier as P  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
bits = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
fx = json.load(open(os.path.join(ROOT, "tests", "golden", f"paillier_{bits}.json")))
sk, pk, coder = P.keypair_from_primes(int(fx["p"], 16), int(fx["q"], 16))
dev = torch.device("cuda", 0)
g = torch.Generator().manual_seed(20241218)
x = (torch.randn(N, generator=g) * 4).to(dev)
a = pk.encrypt_encoded(coder.encode_f32_vec(x), True)
b = pk.encrypt_encoded(coder.encode_f32_vec(torch.flip(x, [0]) * 0.25), True)


def t(f, *args):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = f(*args)
    torch.cuda.synchronize()
    return r, time.perf_counter() - t0


for rep in range(3):
    ng, t_neg = t(P._neg, pk, a)
    sb, t_sub = t(a.sub, pk, b)
    one = P._add(pk, a, ng, False).C.transpose(1, 2).reshape(-1, a.L2)[:N]
    ok = bool((one == pk._key.mont_one(one.device)).all())  # M(1), the stored integer 1
    print(json.dumps({"rep": rep, "N": N, "bits": bits, "batch_min": os.environ.get("FPHE_NEG_BATCH_MIN", "4096"),
                      "neg_s": round(t_neg, 4), "neg_per_s": round(N / t_neg), "sub_s": round(t_sub, 4),
                      "c_times_neg_c_is_1": ok}), flush=True)
