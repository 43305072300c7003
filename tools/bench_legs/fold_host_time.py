"""Host-side duration of one fphe_fold_segments call (the ctypes call returns when every launch
is queued, unless something in it blocks on the device) against its device time, on the bench's
histogram shape.  Prints {"host_ms", "device_ms"}."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from fate_amd import paillier as P  # noqa: E402

N = 1 << 20
fx = json.load(open(os.path.join(ROOT, "tests", "golden", "paillier_2048.json")))
sk, pk, coder = P.keypair_from_primes(int(fx["p"], 16), int(fx["q"], 16))
dev = torch.device("cuda", 0)
g = torch.Generator().manual_seed(1)
psig = torch.sigmoid(torch.randn(N, generator=g, dtype=torch.float64))
ylab = (torch.rand(N, generator=g, dtype=torch.float64) < 0.5).double()
x = torch.stack([(psig - ylab).float(), (psig * (1 - psig)).float()], 1).reshape(-1).to(dev)
gh = pk.encrypt_encoded(coder.encode_f32_vec(x), True)
HF, NB = 4, 32
pos = (torch.randint(0, NB, (N, HF), generator=g) + torch.arange(HF) * NB).to(dev, torch.int32).reshape(-1)
ii = torch.arange(N * HF, device=dev, dtype=torch.int32) // HF
t = torch.arange(2, device=dev, dtype=torch.int32)
src = (ii[:, None] * 2 + t).reshape(-1)
slot = (pos[:, None] * 2 + t).reshape(-1)
for rep in range(3):
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    h0 = time.perf_counter()
    out = P._fold_to_segments(pk, gh, slot, HF * NB * 2, index=src, deferred=[])
    h1 = time.perf_counter()
    e1.record()
    torch.cuda.synchronize()
    print(json.dumps({"rep": rep, "host_ms": round((h1 - h0) * 1e3, 3), "device_ms": round(e0.elapsed_time(e1), 3)}),
          flush=True)
