"""The op kernels once each, 2048-bit key, for rocprofv3 counter passes (tools/gpu_job.sh pmc):
a decrypt of 2^18 elements, a Hetero-LR-shaped ct-add of 2^20, a ct x pt of 2^18 by float32
weights in [-1, 2) (a third negative: the batch inverse runs), and the bench's histogram
iupdate (1M samples x 4 features x (g, h) = 8.4M terms into 256 slots).  Operands come from
key-holder encryptions (the fast CRT path) so the setup stays short.  Each kernel of these ops
is dispatched once in this order (tools/pmc_ops_summary.py relies on it)."""
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
w = coder.encode_f32_vec((torch.rand(1 << 18, generator=g) * 3.0 - 1.0).to(dev))
HF, NB = 4, 32
positions = (torch.randint(0, NB, (N, HF), generator=g) + torch.arange(HF) * NB).to(dev, torch.int32)
t = {}


def timed(name, f):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = f()
    torch.cuda.synchronize()
    t[name] = round(time.perf_counter() - t0, 4)
    return r


timed("decrypt_2^18_s", lambda: sk.decrypt_to_encoded(a.slice(0, 1 << 18)))
timed("add_2^20_s", lambda: a.add(pk, b))
timed("mul_2^18_s", lambda: a.slice(0, 1 << 18).mul(pk, w))
gh = P.Evaluator.cat([a, b])._gather(torch.stack([torch.arange(N), N + torch.arange(N)], 1).reshape(-1))
hist = P.CiphertextVector.zeros(HF * NB * 2, pk._key.L2, dev)
timed("iupdate_8.4M_terms_s", lambda: hist.iupdate(gh, positions, 2, pk))
print(json.dumps(t))
