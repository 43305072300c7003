"""One decrypt (2^18 elements) and one Hetero-LR-shaped ct-add (2^20 elements), 2048-bit key,
for SQ / GRBM counter passes over k_pow_half27 and k_add27 (tools/gpu_job_ops_pmc.sh).
Operands come from key-holder encryptions (the fast CRT path) so the setup stays short."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from fate_amd import paillier as P  # noqa: E402

fx = json.load(open(os.path.join(ROOT, "tests", "golden", "paillier_2048.json")))
sk, pk, coder = P.keypair_from_primes(int(fx["p"], 16), int(fx["q"], 16))
dev = torch.device("cuda", 0)
N = 1 << 20
g = torch.Generator().manual_seed(20241218)
x = (torch.randn(N, generator=g) * 4).to(dev)
a = pk.encrypt_encoded(coder.encode_f32_vec(x), True)
b = pk.encrypt_encoded(coder.encode_f32_vec(torch.flip(x, [0]) * 0.25), True)
torch.cuda.synchronize()
t0 = time.perf_counter()
d = sk.decrypt_to_encoded(a.slice(0, 1 << 18))
torch.cuda.synchronize()
t1 = time.perf_counter()
s = a.add(pk, b)
torch.cuda.synchronize()
t2 = time.perf_counter()
print(json.dumps({"decrypt_2^18_s": round(t1 - t0, 4), "add_2^20_s": round(t2 - t1, 4)}))
