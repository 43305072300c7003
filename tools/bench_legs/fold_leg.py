"""The SecureBoost iupdate of bench.py on synthetic ciphertexts (no encryption first): the
source vector holds random residues below n^2 with random signs and the exponents float32
encodes of randn*4 give (the fold's arithmetic does not depend on the values being
encryptions).  N samples x HF features x 32 bins x stride 2 (the (g, h) pair).  Prints one
JSON line per repetition.  For A/B runs and PMC passes of the fold kernels.

    python tools/bench_legs/fold_leg.py [N] [HF] [REPS]"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from fate_amd import paillier as P  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
HF = int(sys.argv[2]) if len(sys.argv) > 2 else 4
REPS = int(sys.argv[3]) if len(sys.argv) > 3 else 3
NB = 32
fx = json.load(open(os.path.join(ROOT, "tests", "golden", "paillier_2048.json")))
sk, pk, coder = P.keypair_from_primes(int(fx["p"], 16), int(fx["q"], 16))
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(1)
M = 2 * N
x = torch.randn(M, generator=g, device=dev) * 4
x[:8] = torch.tensor([0.0, -0.0, 1e-30, -1e-30, 3.4e38, -3.4e38, 1.0, -1.0], device=dev)
gh = P.CiphertextVector.empty(M, pk._key.L2, dev)
gh.C.copy_(torch.randint(-2 ** 31, 2 ** 31 - 1, gh.C.shape, generator=g, device=dev, dtype=torch.int32))
gh.C[:, -1, :] = 0  # below 2^4064 < n^2
gh.sign.copy_(torch.randint(0, 2, gh.sign.shape, generator=g, device=dev, dtype=torch.uint8))
gh.exp[:M] = coder.encode_f32_vec(x).exp[:M]
gh.n = pk.n
bins = torch.randint(0, NB, (N, HF), generator=g, device=dev)
positions = bins + torch.arange(HF, device=dev) * NB
for rep in range(REPS):
    hist = P.CiphertextVector.zeros(HF * NB * 2, pk._key.L2, dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    hist.iupdate(gh, positions, 2, pk)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(json.dumps({"rep": rep, "samples": N, "features": HF, "terms": N * HF * 2, "iupdate_s": round(dt, 5),
                      "scatter_adds_per_s": round(N * HF * 2 / dt)}), flush=True)
