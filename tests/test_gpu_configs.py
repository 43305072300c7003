"""BASELINE config 1 at its exact workload: "1024-bit Paillier
encrypt -> decrypt round-trip on 1k-element float32 vector ... bit-exact identity check".

SURVEY.md §8 "Configs as concrete synthetic inputs": x = randn(1000) * 4 from
torch.manual_seed(20241218), x[:8] = [0, -0, 1e-30, -1e-30, 3.4e38, -3.4e38, 1, -1];
obfuscated encryption with r from a seeded RNG (the reference draws r from OS entropy,
math/src/rug/random.rs:15-25, so parity means: the same integers for the same r); decrypt;
decode; decoded.view(int32) == x.view(int32) with -0.0 decoding as +0.0 (its significand is 0,
the reference's behaviour).  The ciphertext integers are checked against the oracle's
(crates/paillier/src/lib.rs:104-121 via fixedpoint_paillier::PK::encrypt_encoded,
lib.rs:370-381), as the reference's own test of this path does (paillier/src/lib.rs:190-197)."""
import json
import os
import random

import pytest
import torch

from fate_amd import paillier as P
from oracle import paillier_oracle as O

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _config1_inputs():
    g = torch.Generator().manual_seed(20241218)
    x = torch.randn(1000, generator=g, dtype=torch.float32) * 4
    x[:8] = torch.tensor([0.0, -0.0, 1e-30, -1e-30, 3.4e38, -3.4e38, 1.0, -1.0])
    return x


@pytest.mark.parametrize("keyholder", [False, True], ids=["public", "keyholder_crt"])
def test_config1_roundtrip_bit_exact(keyholder, kernel_path):
    with open(os.path.join(HERE, "golden", "paillier_1024.json")) as f:
        fx = json.load(f)
    p, q = int(fx["p"], 16), int(fx["q"], 16)
    sk, pk, coder = P.keypair_from_primes(p, q, keyholder=keyholder)
    osk, opk = O.keypair_from_primes(p, q)
    assert opk.n.bit_length() == 1024
    x = _config1_inputs()
    rng = random.Random(20241218)
    r = [1 + rng.randrange(opk.n - 1) for _ in range(x.numel())]
    pv = coder.encode_f32_vec(x.cuda())
    ct = pk.encrypt_encoded(pv, True, r=r)
    got_c, got_e = ct.to_signed_ints(pk.ns)
    want = [O.fp_encrypt(opk, O.encode_f32(opk.n, v), True, rv) for v, rv in zip(x.tolist(), r)]
    assert got_e == [w.exp for w in want]
    assert got_c == [w.c for w in want]
    # decrypt -> decode on the device, against the inputs' bit patterns
    out = coder.decode_f32_vec(sk.decrypt_to_encoded(ct)).cpu()
    xb = x.view(torch.int32).clone()
    xb[xb == -2147483648] = 0  # -0.0 decodes as +0.0
    assert torch.equal(out.view(torch.int32), xb)
    # and the oracle's own round trip lands on the same floats
    dec = [O.fp_decrypt(osk, w) for w in want[:64]]
    assert [float(O.decode_f32(opk.n, d.significant, d.exp)) for d in dec] == out[:64].tolist()
