"""pack_squeeze latency, one chunk per wave (fphe_pack_squeeze, fate_amd/csrc/wide_dev.h)
against the step launches of the throughput kernel (fphe_sqmul; FPHE_WIDE_SQUEEZE_MAX=0),
at the bench's packed-histogram shape (4 x 32 slots, 13 per chunk, shift 2 x 74 bits) and
config 4's (10 x 32 slots, shift 2 x 77 bits), 2048-bit key; results compared bit for bit.

    python tools/bench_legs/squeeze_leg.py
"""
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
for slots, shift, num in ((128, 148, 13), (320, 154, 13), (4096, 148, 13)):
    x = torch.randn(slots, generator=torch.Generator().manual_seed(slots), dtype=torch.float64).to(dev)
    v = pk.encrypt_encoded(coder.encode_f64_vec(x), True)
    out = {}
    res = {}
    for mode, cap in (("wide", 1 << 30), ("stepwise", 0)):
        P.WIDE_SQUEEZE_MAX_CHUNKS = cap
        v.pack_squeeze(num, shift, pk)  # warm
        torch.cuda.synchronize(dev)
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            r = v.pack_squeeze(num, shift, pk)
            torch.cuda.synchronize(dev)
            ts.append(time.perf_counter() - t0)
        out[mode + "_ms"] = round(min(ts) * 1e3, 3)
        res[mode] = r.to_signed_ints(pk.ns)
    out.update({"slots": slots, "shift": shift, "pack_num": num, "chunks": -(-slots // num),
                "same": res["wide"] == res["stepwise"], "speedup": round(out["stepwise_ms"] / out["wide_ms"], 2)})
    print(json.dumps(out), flush=True)
