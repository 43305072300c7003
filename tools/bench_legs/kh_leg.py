"""Key-holder (CRT) encryption rate at 2048 and 1024 bits over 2^20 float32 (untimed pass
first, the timed one queued behind it), and its identity with the public-key path on the
first 4096 elements for the same injected r: one JSON line.  Same-box A/B of library builds
(FPHE_LIB_PATH, tools/gpu_job_ab.sh with LEG=kh_leg.py)."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from fate_amd import paillier as P  # noqa: E402

N = 1 << 20
dev = torch.device("cuda", 0)
stream = torch.cuda.current_stream(dev)
out = {}
for bits in (2048, 1024):
    fx = json.load(open(os.path.join(ROOT, "tests", "golden", f"paillier_{bits}.json")))
    p, q = int(fx["p"], 16), int(fx["q"], 16)
    _, pk_pub, coder = P.keypair_from_primes(p, q, keyholder=False)
    _, pk_kh, _ = P.keypair_from_primes(p, q)
    x = (torch.randn(N, generator=torch.Generator().manual_seed(bits), dtype=torch.float32) * 4).to(dev)
    pv = coder.encode_f32_vec(x)
    pk_kh.encrypt_encoded(pv, True)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    pk_kh.encrypt_encoded(pv, True)
    e1.record(stream)
    torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1)
    g = torch.Generator().manual_seed(7)
    r = [1 + int.from_bytes(bytes(torch.randint(0, 256, (bits // 8,), generator=g).tolist()), "little") % (pk_pub.n - 1)
         for _ in range(4096)]
    sub = coder.encode_f32_vec(x[:4096])
    a = pk_kh.encrypt_encoded(sub, True, r=r).to_signed_ints(pk_pub.ns)
    b = pk_pub.encrypt_encoded(sub, True, r=r).to_signed_ints(pk_pub.ns)
    out[f"keyholder_{bits}_per_s"] = round(N / ms * 1e3)
    out[f"keyholder_{bits}_equals_public_4096"] = a == b
print(json.dumps(out))
