"""GPU parity: libfatephe (through the fate_amd Python surface and the C ABI) against the
golden fixtures produced by the oracle (tests/golden/make_fixtures.py), bit-exact.

Integer work => bit-exact equality of signed ciphertext integers, exponents and decoded
float bits (no tolerance)."""
import ctypes
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
def test_encrypt_injected_r(fx, kernel_path, keyholder):
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


def test_decrypt_and_decode(fx, kernel_path):
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
def test_roundtrip_device_rng(fx, kernel_path, keyholder):
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


def test_keyholder_obfuscation_is_uniform_nth_residue(fx, kernel_path):
    """The key holder's device-drawn obfuscation (k_draw_z: (z_p, z_q) drawn directly in CRT
    coordinates instead of r) is an n-th residue, x = c / (1 + m n) mod n^2 with x^lambda = 1
    mod n^2, as the reference's r^n (paillier/src/lib.rs:94-98), and since x mod p = z_p
    (Fermat), z_p / p and z_q / q over 4096 elements pass a Kolmogorov-Smirnov test against
    U(0, 1) (D < 0.04, p ~ 1e-5) and are pairwise distinct."""
    f, sk, pk, coder = fx
    p, q = sk.p, sk.q
    n, ns = pk.n, pk.ns
    lam = (p - 1) * (q - 1)
    x = (torch.randn(4096, generator=torch.Generator().manual_seed(3)) * 4).cuda()
    pv = coder.encode_f32_vec(x)
    sig, _ = pv.to_ints()
    cs, _ = pk.encrypt_encoded(pv, True).to_signed_ints(ns)
    zs = {p: [], q: []}
    for i, (c, m) in enumerate(zip(cs, sig)):
        xo = (c % ns) * pow((1 + (m % n) * n) % ns, -1, ns) % ns
        if i < 64:
            assert pow(xo, lam, ns) == 1, f"element {i}: obfuscation is not an n-th residue"
        for s in (p, q):
            zs[s].append(xo % s)
    for s, z in zs.items():
        assert len(set(z)) == len(z)
        u = np.sort(np.array([v / s for v in z]))
        k = np.arange(1, len(u) + 1) / len(u)
        d = max(np.max(k - u), np.max(u - (k - 1 / len(u))))
        assert d < 0.04, f"z mod {'p' if s == p else 'q'} fails KS against U(0,1): D = {d:.4f}"


F64_EDGES = [
    0.0, -0.0, 1.0, -1.0, 0.5, 1.5, -2.5, 0.1, 1.0 / 3.0, -7.0 / 3.0,
    5e-324, -5e-324, 1e-323, 3 * 2.0 ** -1074, 2.2250738585072009e-308, -2.2250738585072009e-308,  # subnormals
    2.2250738585072014e-308, -2.2250738585072014e-308, 2.0 ** -1022 * 1.5,                          # smallest normals
    1.7976931348623157e308, -1.7976931348623157e308, 2.0 ** 1023, 8.98846567431158e307,             # largest
    2.0 ** 52, 2.0 ** 52 + 1, 2.0 ** 53, 2.0 ** 53 - 1, 2.0 ** 53 + 2, -(2.0 ** 63), 2.0 ** 64 - 2048,
    float.fromhex("0x1.fffffffffffffp-1"), float.fromhex("0x1.0000000000001p+0"),                    # ulp around 1
    float.fromhex("0x1.8p-1070"), float.fromhex("-0x1.000001p+100"), 3.4028234663852886e38, 1e-30,
]


def test_encode_f64_bit_exact(fx):
    """Device k_encode_f64 against the oracle's Coder::encode_f64 (fixedpoint_paillier/src/
    lib.rs:148-168: frexp, exp = floor((e - 53) / 4), significand = round_half_away(x 16^-exp),
    zero -> (0, -14)) on subnormals down to 4.9e-324, the largest normals, ulp neighbours and
    a seeded random sweep over the whole exponent range."""
    from oracle import paillier_oracle as O
    f, sk, pk, coder = fx
    n = int(f["p"], 16) * int(f["q"], 16)
    rng = np.random.default_rng(17)
    bits = rng.integers(0, 2 ** 63, 2000, dtype=np.uint64) | (rng.integers(0, 2, 2000, dtype=np.uint64) << np.uint64(63))
    rand = [float(v) for v in bits.view(np.float64) if np.isfinite(v)]
    xs = F64_EDGES + rand
    pv = coder.encode_f64_vec(torch.tensor(xs, dtype=torch.float64).cuda())
    sig, exp = pv.to_ints()
    want = [O.encode_f64(n, x) for x in xs]
    assert exp == [w.exp for w in want]
    assert sig == [w.significant for w in want]


@pytest.mark.parametrize("bad", [float("inf"), float("-inf"), float("nan")])
def test_encode_f64_nonfinite_panics(fx, bad):
    """Non-finite floats: the reference's to_integer().unwrap() panics (lib.rs:152-157)."""
    f, sk, pk, coder = fx
    with pytest.raises(P.PanicException):
        coder.encode_f64_vec(torch.tensor([1.0, bad, 2.0], dtype=torch.float64).cuda())


def test_chacha20_rfc8439_block():
    """Device ChaCha20 block function (the CSPRNG of the obfuscation nonces, chacha_dev.h)
    against RFC 8439 §2.3.2's test vector and the same restatement the CPU suite pins
    (tests/test_host.py), over many counters and nonces."""
    from fate_amd import _lib
    from tests.chacha_ref import RFC8439_232, chacha20_block
    lib = _lib.load()
    key, counter, nonce, want = RFC8439_232
    kk = (ctypes.c_uint32 * 8)(*key)
    nn = (ctypes.c_uint32 * 3)(*nonce)
    out = torch.zeros(16 * 300, dtype=torch.int32, device="cuda")
    _lib.check(lib.fphe_chacha20_blocks(kk, counter, nn, 300, ctypes.c_void_p(out.data_ptr()), None),
               "fphe_chacha20_blocks")
    torch.cuda.synchronize()
    got = [v & 0xffffffff for v in out.cpu().tolist()]
    assert got[:16] == want
    for i in (1, 2, 77, 299):
        assert got[16 * i:16 * i + 16] == chacha20_block(key, counter + i, nonce)
    # the stream selector of draw_r for an element index above 2^32 (bits 32..47 in the counter)
    e = (3 << 32) + 12345
    nn2 = (ctypes.c_uint32 * 3)(e & 0xffffffff, 0xdeadbeef, 0x01234567)
    _lib.check(lib.fphe_chacha20_blocks(kk, (e >> 32) << 16, nn2, 2, ctypes.c_void_p(out.data_ptr()), None),
               "fphe_chacha20_blocks")
    torch.cuda.synchronize()
    got = [v & 0xffffffff for v in out[:32].cpu().tolist()]
    assert got[:16] == chacha20_block(key, 3 << 16, [e & 0xffffffff, 0xdeadbeef, 0x01234567])
