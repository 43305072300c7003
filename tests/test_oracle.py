"""CPU tests of the parity oracle (no GPU): the pure-Python restatement of rust/fate_utils is
pinned against (1) libgmp -- the library the reference's rug wraps -- through the
independent C restatement oracle/gmp_ref.c, (2) the reference's own tests (round trips,
pack/unpack, pack_squeeze, matmul/rmatmul), and (3) the committed golden fixtures."""
import json
import math
import os
import random
import struct

import numpy as np
import pytest

from oracle import paillier_oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))


def fixture(bits):
    with open(os.path.join(HERE, "golden", f"paillier_{bits}.json")) as f:
        return json.load(f)


def keys(bits):
    fx = fixture(bits)
    p, q = int(fx["p"], 16), int(fx["q"], 16)
    sk, pk = O.keypair_from_primes(p, q)
    return fx, sk, pk


@pytest.fixture(scope="module")
def gmp():
    from oracle import gmp_ref
    gmp_ref.load()
    return gmp_ref


# ---- rug / GMP integer semantics ---------------------------------
def test_truncating_semantics_match_gmp(gmp):
    rng = random.Random(1)
    for _ in range(300):
        a = rng.randrange(-(1 << 300), 1 << 300)
        m = rng.randrange(1, 1 << 200)
        assert O.tdiv_r(a, m) == gmp.tdiv_r(a, m)
        assert O.tdiv_r(a, m) == a - m * int(a / m) if abs(a) < (1 << 50) else True
    assert gmp.powm(-5, 3, 7) == O.powm(-5, 3, 7) == 1
    assert gmp.powm(3, -1, 7) == O.powm(3, -1, 7) == 5
    assert gmp.tdiv_r(-10, 7) == O.tdiv_r(-10, 7) == -3


@pytest.mark.parametrize("bits", [1024, 2048])
def test_fixtures_vs_gmp(gmp, bits):
    """Every golden ciphertext / decryption is reproduced by libgmp (rug's backend)."""
    fx, sk, pk = keys(bits)
    g = gmp.GmpKey(pk.n, sk.p, sk.q)
    e = fx["encrypt"]
    k = 24 if bits == 2048 else len(e["sig"])
    for s, r, c, nude, d in list(zip(e["sig"], e["r"], e["ct"], e["nude"], e["dec"]))[:k]:
        s, r, c = int(s, 16), int(r, 16), int(c, 16)
        assert g.encrypt(s, r, True) == c
        assert g.encrypt(s, None, False) == int(nude, 16)
        assert g.decrypt(c) == int(d, 16)
    for (a, ea), (b, eb), (o, eo) in zip(fx["add"]["a"], fx["add"]["b"], fx["add"]["out"]):
        a, b = int(a, 16), int(b, 16)
        if a == 1 or b == 1 or ea != eb:
            continue  # literal-1 shortcut / exponent alignment is L1 logic, not a GMP call
        assert g.add_ct(a, b) == int(o, 16)


@pytest.mark.parametrize("bits", [1024, 2048])
def test_ops_fixtures_vs_gmp(gmp, bits):
    """The ops fixtures' neg and ct x pt outputs are what libgmp computes: mpz_invert (powm by
    -1) for neg, mpz_powm over every branch of Ciphertext::mul, a negative exponent meaning
    an inverse first (fixedpoint_paillier/src/lib.rs:259-263, 334-349)."""
    fx, sk, pk = keys(bits)
    with open(os.path.join(HERE, "golden", f"paillier_{bits}_ops.json")) as f:
        ops = json.load(f)
    ns, mx = pk.ns, pk.max_int
    for (a, ea), (o, eo) in zip(ops["neg"]["a"], ops["neg"]["out"]):
        assert gmp.powm(int(a, 16), -1, ns) == int(o, 16) and eo == ea
    kinds = set()
    for (c, ec), (s, es), (o, eo), kind in zip(ops["mul"]["c"], ops["mul"]["p"], ops["mul"]["out"],
                                               ops["mul"]["kind"]):
        c, s = int(c, 16), int(s, 16)
        if s >= pk.n - mx:  # encoded negative int: invert, then powm by n - s
            want = gmp.powm(gmp.powm(c, -1, ns), pk.n - s, ns)
            kinds.add("invert")
        else:
            assert s <= mx
            want = gmp.powm(c, s, ns)
            kinds.add("negative_exponent" if s < 0 else "powm")
        assert want == int(o, 16) and eo == ec + es, kind
    assert kinds == {"invert", "negative_exponent", "powm"}
    # sub = add(a, neg(b)) and rsub = add(neg(a), b), re-derived with the oracle's add on
    # the libgmp inverse
    for (a, ea), (b, eb), (o, eo), (r, er) in zip(ops["sub"]["a"], ops["sub"]["b"], ops["sub"]["out"],
                                                  ops["sub"]["rsub"]):
        A, B = O.Ciphertext(int(a, 16), ea), O.Ciphertext(int(b, 16), eb)
        nb = O.Ciphertext(gmp.powm(B.c, -1, ns), eb)
        na = O.Ciphertext(gmp.powm(A.c, -1, ns), ea)
        assert O.ct_add(pk, A, nb) == O.Ciphertext(int(o, 16), eo)
        assert O.ct_add(pk, na, B) == O.Ciphertext(int(r, 16), er)


def test_invert_branch_and_negative_significands(gmp):
    """encrypt's m > n/4 branch (invert) and negative m (negative ciphertext integer)."""
    fx, sk, pk = keys(1024)
    g = gmp.GmpKey(pk.n, sk.p, sk.q)
    rng = random.Random(7)
    for m in [pk.n // 4 + 1, pk.n - 5, pk.n // 2, -1, -(1 << 55), 0, 1, 25519]:
        r = 1 + rng.randrange(pk.n - 1)
        c = O.encrypt(pk, m, True, r)
        assert c == g.encrypt(m, r, True)
        if m < 0:
            assert c < 0  # truncating remainder keeps the sign (paillier/src/lib.rs:111-116)
        assert O.decrypt(sk, c) == g.decrypt(c) == (m % pk.n)


# ---- the reference's own tests ---------------------------------------------------------
def test_reference_decrypt_roundtrip_25519():
    """crates/paillier/src/lib.rs:190-197 (keygen(1024); decrypt(encrypt(25519, true)))."""
    from fate_amd._keygen import keygen_primes
    p, q = keygen_primes(1024)
    sk, pk = O.keypair_from_primes(p, q)
    c = O.encrypt(pk, 25519, True, r=12345)
    assert O.decrypt(sk, c) == 25519


def test_reference_keygen_odd_size_panics():
    """crates/paillier/src/lib.rs:184-188 (keygen(1023) panics)."""
    from fate_amd._keygen import keygen_primes
    with pytest.raises(AssertionError):
        keygen_primes(1023)


def test_reference_pack_float():
    """python/fate/test/test_paillier.py:5-12."""
    n = keys(1024)[2].n
    vec = [0.1, 0.2, 0.3, 0.4, 0.5]
    packed = O.pack_floats([float(np.float32(v)) for v in vec], 32, 2, 16)
    unpacked = O.unpack_floats(packed, 32, 2, 16, 5)
    assert np.allclose(np.array(vec, dtype=np.float32), np.array(unpacked), rtol=1e-3, atol=1e-3)


def test_reference_pack_squeeze():
    """python/fate/test/test_paillier.py:15-33 (encrypt packed, add, pack_squeeze, unpack)."""
    fx, sk, pk = keys(1024)
    vec1 = [float(np.float32(v)) for v in [0.1, 0.2, 0.3, 0.4, 0.5]]
    vec2 = [float(np.float32(v)) for v in [0.6, 0.7, 0.8, 0.9, 1.0]]
    a = [O.fp_encrypt(pk, p, False) for p in O.pack_floats(vec1, 32, 2, 16)]
    b = [O.fp_encrypt(pk, p, False) for p in O.pack_floats(vec2, 32, 2, 16)]
    c = O.vec_add(pk, a, b)
    packed = O.pack_squeeze(pk, c, 2, 64)
    dec = [O.fp_decrypt(sk, x) for x in packed]
    out = O.unpack_floats(dec, 32, 4, 16, 5)
    assert np.allclose(np.array(vec1) + np.array(vec2), np.array(out), rtol=1e-3, atol=1e-3)


def test_reference_matmul_rmatmul():
    """python/fate/test/test_vertor_paillier.py:48-63 (allclose of decrypted products)."""
    fx, sk, pk = keys(1024)
    rng = np.random.default_rng(3)
    x = rng.random((5, 2)).astype(np.float32)
    y = rng.random((2, 4)).astype(np.float32)
    ex = [O.fp_encrypt(pk, O.encode_f32(pk.n, v), True, r=1 + i) for i, v in enumerate(x.flatten())]
    z = O.matmul(pk, ex, [O.encode_f32(pk.n, v) for v in y.flatten()], [5, 2], [2, 4])
    zd = np.array([float(O.decode_f32(pk.n, d.significant, d.exp)) for d in (O.fp_decrypt(sk, c) for c in z)])
    assert np.allclose(zd.reshape(5, 4), x @ y)
    x2 = rng.random((2, 5)).astype(np.float32)
    y2 = rng.random((4, 2)).astype(np.float32)
    ex2 = [O.fp_encrypt(pk, O.encode_f32(pk.n, v), True, r=3 + i) for i, v in enumerate(x2.flatten())]
    z2 = O.rmatmul(pk, ex2, [O.encode_f32(pk.n, v) for v in y2.flatten()], [2, 5], [4, 2])
    zd2 = np.array([float(O.decode_f32(pk.n, d.significant, d.exp)) for d in (O.fp_decrypt(sk, c) for c in z2)])
    assert np.allclose(zd2.reshape(4, 5), y2 @ x2)


# ---- fixed-point encode / decode (fixedpoint_paillier/src/lib.rs:148-192) ---------------
def test_encode_exact_and_roundtrip():
    n = keys(1024)[2].n
    rng = random.Random(5)
    vals = [0.0, -0.0, 1.0, -1.0, 3.4e38, -3.4e38, 1e-30, 1.4e-45, 2.0 ** -149, 65504.0]
    vals += [struct.unpack("<f", struct.pack("<f", rng.gauss(0, 10)))[0] for _ in range(500)]
    for v in vals:
        v = struct.unpack("<f", struct.pack("<f", v))[0]  # encode_f32 sees the f32 value
        pt = O.encode_f32(n, v)
        if v == 0.0:
            assert (pt.significant, pt.exp) == (0, -14)
            continue
        # exactness: sig * 16^exp == v, |sig| < 2^56
        from fractions import Fraction
        assert Fraction(pt.significant) * Fraction(16) ** pt.exp == Fraction(v)
        assert abs(pt.significant) < (1 << 57)
        back = O.decode_f32(n, pt.significant % n if pt.significant < 0 else pt.significant, pt.exp)
        assert struct.pack("<f", back) == struct.pack("<f", v)


def test_decode_rules():
    n = keys(1024)[2].n
    # exp >= 0 truncates toward zero (rug Integer::to_f64 / mpz_get_d)
    assert O.decode_f64(n, (1 << 57) + 31, 0) == float(1 << 57)
    # exp < 0 rounds to nearest even at 53 bits (MPFR), e.g. 2^53+1 scaled down
    assert O.decode_f64(n, (1 << 53) + 1, -1) == float((1 << 53)) / 16
    assert O.decode_f64(n, (1 << 53) + 3, -1) == float((1 << 53) + 4) / 16
    # negative mantissa: sig >= n - max_int decodes as sig - n
    assert O.decode_f64(n, n - 3, 0) == -3.0
    # for odd n, max_int + 1 == n - max_int: the "Overflow" branch of decode (:177-179)
    # is unreachable and (n+1)/2 is the most negative mantissa
    assert O.decode_f64(n, n // 2 + 1, 0) == -O._int_to_f64_trunc(n // 2)
    with pytest.raises(ValueError):
        O.decode_f64(n, n + 1, 0)


def test_ct_add_literal_one_and_alignment():
    fx, sk, pk = keys(1024)
    a = O.fp_encrypt(pk, O.encode_f32(pk.n, 1.5), True, r=77)
    b = O.fp_encrypt(pk, O.encode_f32(pk.n, -1234.25), True, r=99)
    z = O.ct_zero()
    assert O.ct_add(pk, z, b).c == b.c and O.ct_add(pk, z, b).exp == b.exp
    assert O.ct_add(pk, a, z).c == a.c
    s = O.ct_add(pk, a, b)
    d = O.fp_decrypt(sk, s)
    assert float(O.decode_f32(pk.n, d.significant, d.exp)) == np.float32(1.5 - 1234.25)
    # order independence of folds
    xs = [O.fp_encrypt(pk, O.encode_f32(pk.n, v), True, r=i + 2) for i, v in
          enumerate([0.5, -2.0, 1e-3, 7.0, -0.125, 3.0, 0.0, -9.5])]
    f1 = O.ct_zero()
    for x in xs:
        f1 = O.ct_add(pk, f1, x)
    f2 = O.ct_zero()
    for x in reversed(xs):
        f2 = O.ct_add(pk, f2, x)
    assert (f1.c, f1.exp) == (f2.c, f2.exp)


def test_fixtures_reproducible():
    """The committed fixtures are what the oracle computes (spot check, 1024-bit)."""
    fx, sk, pk = keys(1024)
    e = fx["encrypt"]
    for i in range(0, len(e["sig"]), 17):
        pt = O.encode_f32(pk.n, e["x_f32"][i])
        assert hex(pt.significant) == e["sig"][i] and pt.exp == e["exp"][i]
        c = O.fp_encrypt(pk, pt, True, int(e["r"][i], 16))
        assert hex(c.c) == e["ct"][i]


# ---- the bulk libgmp checkers (oracle/gmp_ref.c gref_fold / gref_mul / gref_squeeze /
# gref_cumsum) that the large -m gpu parity tests use, pinned against the Python restatement
def _signed_sources(pk, k, seed):
    """k signed ciphertext integers with spread exponents and literal 1s (the fold's traps)."""
    rng = random.Random(seed)
    out = []
    for _ in range(k):
        r = rng.random()
        if r < 0.08:
            out.append(O.Ciphertext(1, rng.choice([0, -14, -3])))
        else:
            c = rng.randrange(1, pk.ns)
            out.append(O.Ciphertext(-c if rng.random() < 0.4 else c, rng.choice([-16, -14, -13, -13, -12, -9, 2])))
    return out


@pytest.mark.parametrize("bits", [1024, 2048])
def test_bulk_fold_matches_oracle(gmp, bits):
    fx, sk, pk = keys(bits)
    g = gmp.GmpKey(pk.n)
    L = pk.ns.bit_length() // 32 + 1
    src = _signed_sources(pk, 90, bits)
    rng = random.Random(bits + 1)
    nslots = 13
    acc = [O.ct_zero() for _ in range(nslots)]
    acc[3] = src[5]  # a slot that starts from a real ciphertext
    terms = [rng.randrange(len(src)) for _ in range(600)]
    slots = [rng.randrange(nslots - 2) for _ in range(600)]  # two slots see no term
    want = list(acc)
    for t, s in zip(terms, slots):
        want[s] = O.ct_add(pk, want[s], src[t])
    sv = gmp.to_vec([c.c for c in src], [c.exp for c in src], L)
    av = gmp.to_vec([c.c for c in acc], [c.exp for c in acc], L)
    for threads in (1, 3):
        got = gmp.from_vec(g.fold(sv, terms, slots, av, threads=threads))
        assert got == ([c.c for c in want], [c.exp for c in want])


@pytest.mark.parametrize("bits", [1024, 2048])
def test_bulk_mul_squeeze_cumsum_match_oracle(gmp, bits):
    fx, sk, pk = keys(bits)
    g = gmp.GmpKey(pk.n)
    L = pk.ns.bit_length() // 32 + 1
    src = [c for c in _signed_sources(pk, 40, bits + 7)]
    rng = random.Random(bits + 3)
    # ct x pt: float significands of both signs, encoded negative ints (the invert branch)
    pts = []
    for i in range(len(src)):
        if i % 4 == 3:
            pts.append(O.encode_i64(pk.n, -rng.randrange(1, 1 << 40)))
        else:
            pts.append(O.encode_f32(pk.n, float(np.float32(rng.uniform(-2, 2)))))
    want = [O.ct_mul(pk, c, p) for c, p in zip(src, pts)]
    Lp = max(1, max(abs(p.significant).bit_length() for p in pts) // 32 + 1)
    pv = gmp.to_vec([p.significant for p in pts], [p.exp for p in pts], Lp)
    got = gmp.from_vec(g.mul(gmp.to_vec([c.c for c in src], [c.exp for c in src], L), pv, threads=2))
    assert got == ([c.c for c in want], [c.exp for c in want])
    # pack_squeeze over a ragged last chunk
    want = O.pack_squeeze(pk, src[:23], 3, 140)
    got = gmp.from_vec(g.squeeze(gmp.to_vec([c.c for c in src[:23]], [c.exp for c in src[:23]], L), 3, 140))
    assert got == ([c.c for c in want], [c.exp for c in want])
    # chunking_cumsum_with_step
    data = list(src[:30])
    O.chunking_cumsum_with_step(pk, data, [8, 12, 10], 2)
    got = gmp.from_vec(g.cumsum(gmp.to_vec([c.c for c in src[:30]], [c.exp for c in src[:30]], L), [8, 12, 10], 2))
    assert got == ([c.c for c in data], [c.exp for c in data])
