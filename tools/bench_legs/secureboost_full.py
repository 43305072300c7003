"""BASELINE config 4 at its full size on one MI355X: the SecureBoost histogram over 10M
samples, 10 features x 32 bins, 1 node (320 slots), 2048-bit key.

  (i)  unpacked (the reference's gh_pack=False, guest.py:245-246): g and h encrypted as
       separate float32 ciphertexts (20M, key holder, timed apart), then timed: ct x pt by a
       per-sample weight w ~ U(0.5, 1.5) (GOSS-style stand-in, float significands, so the
       exponents change) and the per-bin iupdate fold (10M x 10 x 2 = 200M scatter-adds,
       with 16^d exponent alignment).  The 640 slots are decrypted and compared (allclose)
       with the float64 histogram.
  (ii) packed (the reference default): (g + 1, h) packed at precision 52 with shift_bit from
       compute_offset_bit(10M, 2, 1), 10M key-holder encryptions, the per-bin fold (100M
       adds, exponent 0), per-feature cumsum, pack_squeeze, decrypt + unpack, allclose.

One JSON line per phase (progress) and a summary line.  On 8 GPUs each rank would take 1/8
of the samples and the partial histograms are all-gathered and folded (bench.py --gpus N,
histogram_multi_gpu).

    python tools/bench_legs/secureboost_full.py [samples]
"""
import json
import math
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from fate_amd import paillier as P  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
HF, NB = 10, 32
fx = json.load(open(os.path.join(ROOT, "tests", "golden", "paillier_2048.json")))
sk, pk, coder = P.keypair_from_primes(int(fx["p"], 16), int(fx["q"], 16), keyholder=True)
dev = torch.device("cuda", 0)
out = {"samples": N, "features": HF, "bins": NB}


def timed(name, f):
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    r = f()
    torch.cuda.synchronize(dev)
    out[name] = round(time.perf_counter() - t0, 3)
    print(json.dumps({"phase": name, "s": out[name]}), flush=True)
    return r


g0 = torch.Generator().manual_seed(20241218)
p = torch.sigmoid(torch.randn(N, generator=g0, dtype=torch.float64))
y = (torch.rand(N, generator=g0, dtype=torch.float64) < 0.5).double()
g, h = (p - y).float(), (p * (1 - p)).float()
w = (torch.rand(N, generator=g0) + 0.5).float()
bins = torch.randint(0, NB, (N, HF), generator=g0)
positions = bins + torch.arange(HF) * NB

# (i) unpacked
gh = torch.stack([g, h], 1).reshape(-1).to(dev)
egh = timed("unpacked_encrypt_20M_s", lambda: pk.encrypt_encoded(coder.encode_f32_vec(gh), True))
wrep = w.repeat_interleave(2).to(dev)
ew = timed("unpacked_ct_x_pt_20M_s", lambda: egh.mul(pk, coder.encode_f32_vec(wrep)))
del egh
# the bin indexes live in HBM like the ciphertexts (bench.py); one untimed full-size pass
# first maps the call's stream-ordered scratch into the device pool
positions_d = positions.to(dev, torch.int32)
P.CiphertextVector.zeros(HF * NB * 2, pk._key.L2, dev).iupdate(ew, positions_d, 2, pk)
hist = P.CiphertextVector.zeros(HF * NB * 2, pk._key.L2, dev)
timed("unpacked_iupdate_200M_s", lambda: hist.iupdate(ew, positions_d, 2, pk))
del ew
dec = coder.decode_f64_vec(sk.decrypt_to_encoded(hist)).cpu().reshape(HF * NB, 2)
want = torch.zeros(HF * NB, 2, dtype=torch.float64)
for f in range(HF):
    want[:, 0].index_add_(0, positions[:, f], g.double() * w.double())
    want[:, 1].index_add_(0, positions[:, f], h.double() * w.double())
out["unpacked_allclose"] = bool(torch.allclose(dec, want, rtol=1e-9, atol=1e-6))
out["unpacked_scatter_adds_per_s"] = round(N * HF * 2 / out["unpacked_iupdate_200M_s"], 1)
del hist

# (ii) packed
shift = int(math.log2(2 ** 52 * N * 2) + 1)
squeeze_num = (2048 - 2) // (shift * 2)
vals = torch.stack([g.double() + 1.0, h.double()], 1).reshape(-1).to(dev)
pv = timed("packed_pack_s", lambda: coder.pack_floats(vals, shift, 2, 52))
en = timed("packed_encrypt_10M_s", lambda: pk.encrypt_encoded(pv, True))
P.CiphertextVector.zeros(HF * NB, pk._key.L2, dev).iupdate(en, positions_d, 1, pk)
hp = P.CiphertextVector.zeros(HF * NB, pk._key.L2, dev)
timed("packed_iupdate_100M_s", lambda: hp.iupdate(en, positions_d, 1, pk))
del en
timed("packed_cumsum_s", lambda: hp.chunking_cumsum_with_step(pk, [NB] * HF, 1))
sq = timed("packed_squeeze_s", lambda: hp.pack_squeeze(squeeze_num, shift * 2, pk))
dq = sk.decrypt_to_encoded(sq)
got = torch.tensor(coder.unpack_floats(dq, shift, 2 * squeeze_num, 52, HF * NB * 2), dtype=torch.float64)
wantp = torch.zeros(HF * NB, 2, dtype=torch.float64)
for f in range(HF):
    wantp[:, 0].index_add_(0, positions[:, f], g.double() + 1.0)
    wantp[:, 1].index_add_(0, positions[:, f], h.double())
wantp = wantp.view(HF, NB, 2).cumsum(1).reshape(-1)
out.update({"packed_shift_bit": shift, "packed_squeeze_num": squeeze_num, "packed_squeezed_ciphertexts": sq.count,
            "packed_scatter_adds_per_s": round(N * HF / out["packed_iupdate_100M_s"], 1),
            "packed_allclose": bool(torch.allclose(got, wantp, rtol=1e-12, atol=1e-9))})
print(json.dumps(out), flush=True)
