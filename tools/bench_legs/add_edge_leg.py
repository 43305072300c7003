"""bench.py's ct-add kernel leg (rooflines.ct_add: k_add27 over enc(x) + enc(0.25 flip(x)),
2^20 elements, 2048-bit key, warm clock) on the bench's x -- whose first 8 entries are the
edge values 0, -0, +-1e-30, +-3.4e38, +-1, putting exponent gaps up to 31 (124 squarings of
one element) into the launch -- and on the same x with those 8 entries replaced by ordinary
values: does the lone 124-squaring chain bound the launch?"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from fate_amd import paillier as P  # noqa: E402

N = 1 << 20
fx = json.load(open(os.path.join(ROOT, "tests", "golden", "paillier_2048.json")))
sk, pk, coder = P.keypair_from_primes(int(fx["p"], 16), int(fx["q"], 16))
dev = torch.device("cuda", 0)
stream = torch.cuda.current_stream(dev)
x = torch.randn(N, generator=torch.Generator().manual_seed(20241218), dtype=torch.float32) * 4
x[:8] = torch.tensor([0.0, -0.0, 1e-30, -1e-30, 3.4e38, -3.4e38, 1.0, -1.0])
for name, xv in (("edge", x), ("no_edge", torch.cat([x[8:16], x[8:]]))):
    xd = xv.to(dev)
    a = pk.encrypt_encoded(coder.encode_f32_vec(xd), True)
    b = pk.encrypt_encoded(coder.encode_f32_vec(torch.flip(xd, [0]) * 0.25), True)
    blk = bench.add_kernel_leg(P, pk, a, b, N, stream, dev)
    print(json.dumps({"data": name, "kernel_ms": blk["kernel_ms"], "cold_kernel_ms": blk["cold_kernel_ms"],
                      "frac": blk["frac"], "issue": blk["issue"]["frac"],
                      "max_gap": len(blk["gap_histogram"]) - 1}), flush=True)
