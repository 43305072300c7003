"""Same-box A/B of an fphe_fold_segments variant switched by an env variable read per call:
the bench's iupdate (1M SecureBoost-shaped (g, h) samples x 4 features x 32 bins, device
positions), cold calls alternating A and B with a host sync and a short idle between, as the
bench's leg runs it.
    python tools/bench_legs/iupdate_ab_leg.py ENVVAR VALUE_A VALUE_B [REPS]"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from fate_amd import paillier as P  # noqa: E402

var, va, vb = sys.argv[1], sys.argv[2], sys.argv[3]
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 12
N, HF, NB = 1 << 20, 4, 32
fx = json.load(open(os.path.join(ROOT, "tests", "golden", "paillier_2048.json")))
sk, pk, coder = P.keypair_from_primes(int(fx["p"], 16), int(fx["q"], 16))
dev = torch.device("cuda", 0)
g = torch.Generator().manual_seed(99)
psig = torch.sigmoid(torch.randn(N, generator=g, dtype=torch.float64))
ylab = (torch.rand(N, generator=g, dtype=torch.float64) < 0.5).double()
x = torch.stack([(psig - ylab).float(), (psig * (1 - psig)).float()], 1).reshape(-1).to(dev)
gh = pk.encrypt_encoded(coder.encode_f32_vec(x), True)
positions = (torch.randint(0, NB, (N, HF), generator=g) + torch.arange(HF) * NB).to(dev, torch.int32)
times = {va: [], vb: []}
ref = None
for i in range(reps):
    for v in ((va, vb) if i % 2 == 0 else (vb, va)):
        os.environ[var] = v
        h = P.CiphertextVector.zeros(HF * NB * 2, pk._key.L2, dev)
        torch.cuda.synchronize()
        time.sleep(0.05)
        t0 = time.perf_counter()
        h.iupdate(gh, positions, 2, pk)
        torch.cuda.synchronize()
        times[v].append(time.perf_counter() - t0)
        st = h.to_signed_ints(pk.ns)
        if ref is None:
            ref = st
        assert st == ref, "variants disagree"
    print(f"rep {i}: " + " ".join(f"{k}={times[k][-1] * 1e3:.3f}ms" for k in times), flush=True)
out = {k: {"median_ms": round(sorted(t)[len(t) // 2] * 1e3, 3), "min_ms": round(min(t) * 1e3, 3)} for k, t in times.items()}
print(json.dumps({"var": var, "reps": reps, **out, "identical_results": True}))
