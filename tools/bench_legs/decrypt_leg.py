"""2048-bit CRT decryption of 2^20 ciphertexts: 3 timed launches after a warm-up (HIP events on
the current stream), one JSON line.  For same-box A/B of library builds (FPHE_LIB_PATH,
tools/gpu_job_ab.sh with LEG=decrypt_leg.py)."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from fate_amd import paillier as P  # noqa: E402

fx = json.load(open(os.path.join(ROOT, "tests", "golden", "paillier_2048.json")))
sk, pk, coder = P.keypair_from_primes(int(fx["p"], 16), int(fx["q"], 16), keyholder=True)
x = torch.randn(1 << 20, generator=torch.Generator().manual_seed(4)).cuda()
c = pk.encrypt_encoded(coder.encode_f32_vec(x), True)
sk.decrypt_to_encoded(c)
ms = []
for _ in range(3):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    d = sk.decrypt_to_encoded(c)
    e1.record()
    torch.cuda.synchronize()
    ms.append(e0.elapsed_time(e1))
print(json.dumps({"decrypt_ms": [round(v, 2) for v in ms], "per_s": round((1 << 20) / min(ms) * 1e3),
                  "ok": bool(torch.equal(coder.decode_f32_vec(d), x))}))
