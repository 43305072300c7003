"""Time bench.py's ct x pt leg (Ciphertext::mul, fixedpoint_paillier/src/lib.rs:334-349):
2^20 2048-bit ciphertexts times float32 weights in [-1, 2), so a third of the elements take
the invert branch.  FPHE_NEG_BATCH_MIN picks the inverse (read once per process): unset ->
masked batch inversion, a huge value -> one inverse per element.  Checks the decrypted
products against x * w."""
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
w = (torch.rand(N, generator=g) * 3.0 - 1.0).to(dev)
a = pk.encrypt_encoded(coder.encode_f32_vec(x), True)
pw = coder.encode_f32_vec(w)

for rep in range(3):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    m = a.mul(pk, pw)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    d = coder.decode_f64_vec(sk.decrypt_to_encoded(m))
    want = x.double() * w.double()
    ok = bool(torch.allclose(d, want, rtol=1e-12, atol=1e-12))
    print(json.dumps({"rep": rep, "N": N, "batch_min": os.environ.get("FPHE_NEG_BATCH_MIN", "4096"),
                      "mul_s": round(dt, 4), "mul_per_s": round(N / dt), "allclose": ok}), flush=True)
