"""1024-bit keys (TPI 2 for n^2, TPI 1 for p^2 / q^2): public-key encrypt, CRT decrypt and the
key-holder encrypt over 2^20 float32 elements, timed as bench.py's key_1024 leg (untimed
passes first, the timed ones queued behind them), rates and roofline fractions as one JSON
line.  For same-box A/B of library builds (FPHE_LIB_PATH, tools/gpu_job_ab.sh LEG=...)."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from fate_amd import paillier as P  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
dev = torch.device("cuda", 0)
stream = torch.cuda.current_stream(dev)
fx = json.load(open(os.path.join(ROOT, "tests", "golden", "paillier_1024.json")))
sk, pk, coder = P.keypair_from_primes(int(fx["p"], 16), int(fx["q"], 16), keyholder=False)
_, pk_kh, _ = P.keypair_from_primes(int(fx["p"], 16), int(fx["q"], 16))
x = (torch.randn(N, generator=torch.Generator().manual_seed(5), dtype=torch.float32) * 4).to(dev)
pv = coder.encode_f32_vec(x)
sk.decrypt_to_encoded(pk.encrypt_encoded(pv, True))
pk_kh.encrypt_encoded(pv, True)
ev = [torch.cuda.Event(enable_timing=True) for _ in range(6)]
ev[0].record(stream)
c = pk.encrypt_encoded(pv, True)
ev[1].record(stream)
ev[2].record(stream)
d = sk.decrypt_to_encoded(c)
ev[3].record(stream)
ev[4].record(stream)
ck = pk_kh.encrypt_encoded(pv, True)
ev[5].record(stream)
torch.cuda.synchronize(dev)
enc, dec, kh = (ev[i].elapsed_time(ev[i + 1]) for i in (0, 2, 4))
ok = bool(torch.equal(coder.decode_f32_vec(d).cpu(), x.cpu()))
frac = lambda mac, ms: round(N * mac / (ms / 1e3) / 1e12 / bench.PEAK_TMAC32, 4)
print(json.dumps({"encrypt_per_s": round(N / enc * 1e3), "encrypt_frac": frac(bench.enc_mac32_per_elem(1024), enc),
                  "decrypt_per_s": round(N / dec * 1e3), "decrypt_frac": frac(bench.dec_mac32_per_elem(1024), dec),
                  "keyholder_encrypt_per_s": round(N / kh * 1e3), "roundtrip": ok}))
