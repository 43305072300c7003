"""GPU parity: libfatephe (through the fate_amd Python surface and the C ABI) against the
golden fixtures produced by the oracle (tests/golden/make_fixtures.py), bit-exact.

Integer work => bit-exact equality of signed ciphertext integers, exponents and decoded
float bits (no tolerance)."""
import json
import os
import struct

import numpy as np
import pytest
import torch

from fate_amd import paillier as P

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def load(bits):
    with open(os.path.join(HERE, "golden", f"paillier_{bits}.json")) as f:
        fx = json.load(f)
    p, q = int(fx["p"], 16), int(fx["q"], 16)
    sk, pk, coder = P.keypair_from_primes(p, q)
    return fx, sk, pk, coder


def ct_vec(pk, pairs):
    cs = [int(c, 16) for c, _ in pairs]
    es = [e for _, e in pairs]
    return P.CiphertextVector.from_signed_ints(cs, es, pk.ns, pk._key.L2)


def ct_list(pk, v):
    cs, es = v.to_signed_ints(pk.ns)
    return [[hex(c), e] for c, e in zip(cs, es)]


@pytest.fixture(params=[1024, 2048])
def fx(request):
    return load(request.param)


def test_encode_f32(fx):
    f, sk, pk, coder = fx
    x = torch.tensor(f["encrypt"]["x_f32"], dtype=torch.float32)
    pv = coder.encode_f32_vec(x.cuda())
    sig, exp = pv.to_ints()
    assert sig == [int(s, 16) for s in f["encrypt"]["sig"]]
    assert exp == f["encrypt"]["exp"]


@pytest.mark.parametrize("keyholder", [False, True], ids=["public", "keyholder_crt"])
def test_encrypt_injected_r(fx, keyholder):
    """Public-key path (fphe_encrypt) and key-holder CRT path (fphe_encrypt_crt): both must
    give the reference's ciphertext integers for the same r."""
    f, sk, pk, coder = fx
    if not keyholder:
        pk = P.PK(pk.n)
    assert pk.keyholder == keyholder
    e = f["encrypt"]
    pv = P.PlaintextVector.from_ints([int(s, 16) for s in e["sig"]], e["exp"])
    ct = pk.encrypt_encoded(pv, True, r=[int(r, 16) for r in e["r"]])
    cs, es = ct.to_signed_ints(pk.ns)
    assert [hex(c) for c in cs] == e["ct"]
    assert es == e["exp"]


def test_encrypt_nude(fx):
    f, sk, pk, coder = fx
    e = f["encrypt"]
    pv = P.PlaintextVector.from_ints([int(s, 16) for s in e["sig"]], e["exp"])
    ct = pk.encrypt_encoded(pv, False)
    cs, _ = ct.to_signed_ints(pk.ns)
    assert [hex(c) for c in cs] == e["nude"]


def test_decrypt_and_decode(fx):
    f, sk, pk, coder = fx
    e = f["encrypt"]
    ct = P.CiphertextVector.from_signed_ints([int(c, 16) for c in e["ct"]], e["exp"], pk.ns, pk._key.L2)
    pt = sk.decrypt_to_encoded(ct)
    sig, exp = pt.to_ints()
    assert [hex(s) for s in sig] == e["dec"]
    out = coder.decode_f32_vec(pt).cpu().numpy()
    want = np.array(e["dec_f32"], dtype=np.float32)
    assert out.view(np.uint32).tolist() == want.view(np.uint32).tolist()


def test_add(fx):
    f, sk, pk, coder = fx
    a = ct_vec(pk, f["add"]["a"])
    b = ct_vec(pk, f["add"]["b"])
    assert ct_list(pk, a.add(pk, b)) == [[c, e] for c, e in f["add"]["out"]]


def test_mul(fx):
    f, sk, pk, coder = fx
    c = ct_vec(pk, f["mul"]["c"])
    pv = P.PlaintextVector.from_ints([int(s, 16) for s, _ in f["mul"]["p"]], [e for _, e in f["mul"]["p"]])
    assert ct_list(pk, c.mul(pk, pv)) == [[x, e] for x, e in f["mul"]["out"]]


@pytest.mark.parametrize("keyholder", [False, True], ids=["public", "keyholder_crt"])
def test_roundtrip_device_rng(fx, keyholder):
    """decrypt(encrypt(x)) == x with device-drawn r (reference test crates/paillier/src/lib.rs:190-197)."""
    f, sk, pk, coder = fx
    if not keyholder:
        pk = P.PK(pk.n)
    x = torch.tensor(f["encrypt"]["x_f32"], dtype=torch.float32).cuda()
    ct = pk.encrypt_encoded(coder.encode_f32_vec(x), True)
    y = coder.decode_f32_vec(sk.decrypt_to_encoded(ct))
    xb = x.cpu().numpy().view(np.uint32)
    yb = y.cpu().numpy().view(np.uint32)
    # -0.0 encodes to significand 0 and decodes as +0.0 (reference behaviour)
    xb = np.where(xb == 0x80000000, 0, xb)
    assert yb.tolist() == xb.tolist()
    # two encryptions of the same plaintext differ (fresh r per element and per call)
    ct2 = pk.encrypt_encoded(coder.encode_f32_vec(x), True)
    assert not torch.equal(ct.C, ct2.C)
