#!/usr/bin/env python3
"""Generate the golden parity fixtures under tests/golden/ from the CPU oracle.

The reference (rust/fate_utils) cannot be built or imported in this environment
(no cargo/rustc, no fate_utils wheel), and it ships no known-answer
vectors, so these fixtures are produced by the oracle (oracle/paillier_oracle.py), which
is itself cross-checked against libgmp -- the library the reference's rug wraps -- by
tests/test_oracle.py.  Keys and obfuscation nonces r are derived from a fixed seed so the
fixtures are reproducible:  python3 tests/golden/make_fixtures.py
"""
from __future__ import annotations

import json
import os
import random
import struct
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import paillier_oracle as O  # noqa: E402

SEED = 20241218


def _is_prime(n: int, rng: random.Random) -> bool:
    if n < 2:
        return False
    for p in (2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37):
        if n % p == 0:
            return n == p
    d, s = n - 1, 0
    while d % 2 == 0:
        d //= 2
        s += 1
    for _ in range(40):
        a = 2 + rng.randrange(n - 3)
        x = pow(a, d, n)
        if x in (1, n - 1):
            continue
        for _ in range(s - 1):
            x = x * x % n
            if x == n - 1:
                break
        else:
            return False
    return True


def _gen_prime(bits: int, rng: random.Random) -> int:
    # BInt::gen_prime (math/src/rug/random.rs:27-32): random bits, top bit set, next_prime
    x = rng.getrandbits(bits) | (1 << (bits - 1))
    c = x + 1 if x % 2 == 0 else x + 2
    while not _is_prime(c, rng):
        c += 2
    return c


def keypair(bits: int, rng: random.Random):
    while True:
        p, q = _gen_prime(bits // 2, rng), _gen_prime(bits // 2, rng)
        if p != q and (p * q).bit_length() == bits:
            return (p, q) if p < q else (q, p)


def f32(x: float) -> float:
    return struct.unpack("<f", struct.pack("<f", x))[0]


def float_inputs(rng: random.Random, count: int):
    specials = [0.0, -0.0, 1e-30, -1e-30, 3.4e38, -3.4e38, 1.0, -1.0, 0.5, -2.75, 1.5e-45, 123456.789]
    xs = [f32(v) for v in specials]
    while len(xs) < count:
        xs.append(f32(rng.gauss(0.0, 1.0) * 4.0))
    return xs[:count]


def build(bits: int, n_enc: int, n_add: int, n_mul: int, rng: random.Random) -> dict:
    p, q = keypair(bits, rng)
    sk, pk = O.keypair_from_primes(p, q)
    n = pk.n
    xs = float_inputs(rng, n_enc)
    pts = [O.encode_f32(n, x) for x in xs]
    rs = [1 + rng.randrange(n - 1) for _ in xs]
    cts = [O.fp_encrypt(pk, pt, True, r) for pt, r in zip(pts, rs)]
    nude = [O.fp_encrypt(pk, pt, False) for pt in pts]
    dec = [O.fp_decrypt(sk, c) for c in cts]
    dec_f32 = [float(O.decode_f32(n, d.significant, d.exp)) for d in dec]
    # ct-add: pairs with differing exponents, plus literal-1 zeros (:303-308)
    add_a, add_b, add_out = [], [], []
    zero = O.ct_zero()
    for i in range(n_add):
        a = cts[i % n_enc]
        b = cts[(3 * i + 1) % n_enc]
        if i % 11 == 5:
            a = zero
        if i % 13 == 7:
            b = zero
        add_a.append(a)
        add_b.append(b)
        add_out.append(O.ct_add(pk, a, b))
    # ct x pt (non-negative float significands and small non-negative ints)
    mul_c, mul_p, mul_out = [], [], []
    for i in range(n_mul):
        c = cts[(5 * i + 2) % n_enc]
        if i % 2 == 0:
            pt = O.encode_f32(n, abs(f32(rng.uniform(0.5, 1.5))))
        else:
            pt = O.encode_i64(n, rng.randrange(0, 1 << 40))
        if i == 3:
            pt = O.encode_f32(n, 0.0)
        mul_c.append(c)
        mul_p.append(pt)
        mul_out.append(O.ct_mul(pk, c, pt))
    hx = lambda v: hex(v)  # noqa: E731
    ct_j = lambda c: [hx(c.c), c.exp]  # noqa: E731
    return {
        "bits": bits, "p": hx(p), "q": hx(q),
        "encrypt": {
            "x_f32": xs,
            "sig": [hx(pt.significant) for pt in pts], "exp": [pt.exp for pt in pts],
            "r": [hx(r) for r in rs],
            "ct": [hx(c.c) for c in cts],
            "nude": [hx(c.c) for c in nude],
            "dec": [hx(d.significant) for d in dec],
            "dec_f32": dec_f32,
        },
        "add": {"a": [ct_j(c) for c in add_a], "b": [ct_j(c) for c in add_b], "out": [ct_j(c) for c in add_out]},
        "mul": {"c": [ct_j(c) for c in mul_c], "p": [[hx(pt.significant), pt.exp] for pt in mul_p],
                "out": [ct_j(c) for c in mul_out]},
    }


def build_ops(fx: dict, rng: random.Random) -> dict:
    """The vector algebra beyond encrypt/add/mul on the same key and ciphertexts as `fx`:
    neg / sub / rsub (mpz_invert), ct x pt over every branch of Ciphertext::mul (negative
    float significands = GMP's negative exponent, encoded negative ints = the invert branch,
    big ints up to max_int, the branch limits themselves), matmul / rmatmul, iupdate and
    pack_squeeze (fixedpoint_paillier/src/lib.rs:259-285, 334-349, 439-450, 724-735, 852-908)."""
    p, q = int(fx["p"], 16), int(fx["q"], 16)
    sk, pk = O.keypair_from_primes(p, q)
    n = pk.n
    e = fx["encrypt"]
    obf = [O.Ciphertext(int(c, 16), x) for c, x in zip(e["ct"], e["exp"])]
    nude = [O.Ciphertext(int(c, 16), x) for c, x in zip(e["nude"], e["exp"])]
    # real encryptions, signed ones among them (negative significands encrypt to negative
    # integers: tdiv keeps the sign), and the literal-1 zero
    pool = obf[:12] + [c for c in nude if c.c < 0][:4] + [O.ct_zero()]
    hx = lambda v: hex(v)  # noqa: E731
    ctj = lambda c: [hx(c.c), c.exp]  # noqa: E731
    ptj = lambda t: [hx(t.significant), t.exp]  # noqa: E731
    out: dict = {}
    negs = [c for c in pool if c.c != 1]
    out["neg"] = {"a": [ctj(c) for c in negs], "out": [ctj(O.ct_neg(pk, c)) for c in negs]}
    sa = [pool[i % len(pool)] for i in range(12)]
    sb = [pool[(5 * i + 3) % len(pool)] for i in range(12)]
    out["sub"] = {"a": [ctj(c) for c in sa], "b": [ctj(c) for c in sb],
                  "out": [ctj(O.ct_sub(pk, a, b)) for a, b in zip(sa, sb)],
                  "rsub": [ctj(O.ct_rsub(pk, a, b)) for a, b in zip(sa, sb)]}
    mx = pk.max_int
    pts = [
        ("neg_f32", O.encode_f32(n, -0.75)), ("neg_f32", O.encode_f32(n, f32(-rng.uniform(0.5, 1.5)))),
        ("neg_f64_tiny", O.encode_f64(n, -5e-324)), ("pos_f64_big", O.encode_f64(n, 1.7976931348623157e308)),
        ("neg_i64", O.encode_i64(n, -1)), ("neg_i64", O.encode_i64(n, -(1 << 40) - 12345)),
        ("neg_i64_min", O.encode_i64(n, -(1 << 63))),
        ("zero", O.encode_i64(n, 0)), ("one", O.encode_i64(n, 1)),
        ("big", O.Plaintext(rng.getrandbits(n.bit_length() - 3), 0)),
        ("max_int", O.Plaintext(mx, 0)), ("n_minus_max_int", O.Plaintext(n - mx, 0)),
        ("n_minus_1", O.Plaintext(n - 1, 0)),
    ]
    mc = [obf[(3 * i + 1) % len(obf)] if i % 4 != 3 else nude[i % len(nude)] for i in range(len(pts))]
    out["mul"] = {"kind": [k for k, _ in pts], "c": [ctj(c) for c in mc], "p": [ptj(t) for _, t in pts],
                  "out": [ctj(O.ct_mul(pk, c, t)) for c, (_, t) in zip(mc, pts)]}
    # matmul (3x4) @ (4x2) plaintexts, and rmatmul (4x3) x (2x4) with signed int features
    a = obf[:12]
    bs = [O.encode_f32(n, f32(rng.gauss(0.0, 1.0))) for _ in range(8)]
    bi = [O.encode_i64(n, rng.randrange(-50, 50)) for _ in range(8)]
    out["matmul"] = {"a": [ctj(c) for c in a], "b": [ptj(t) for t in bs], "lshape": [3, 4], "rshape": [4, 2],
                     "out": [ctj(c) for c in O.matmul(pk, a, bs, [3, 4], [4, 2])]}
    out["rmatmul"] = {"a": [ctj(c) for c in a], "b": [ptj(t) for t in bi], "lshape": [4, 3], "rshape": [2, 4],
                      "out": [ctj(c) for c in O.rmatmul(pk, a, bi, [4, 3], [2, 4])]}
    # iupdate: 4 slots x stride 2, 6 samples each added into 1-3 slots (exponents differ)
    data = [O.ct_zero() for _ in range(8)]
    other = [obf[(7 * i) % len(obf)] for i in range(12)]
    indexes = [sorted(rng.sample(range(4), rng.randint(1, 3))) for _ in range(6)]
    want = list(data)
    O.iupdate(pk, want, other, indexes, 2)
    out["iupdate"] = {"data": [ctj(c) for c in data], "other": [ctj(c) for c in other], "indexes": indexes,
                      "stride": 2, "out": [ctj(c) for c in want]}
    sq = [O.Ciphertext(c.c if c.c > 0 else -c.c, 0) for c in obf[:9]]
    out["pack_squeeze"] = {"data": [ctj(c) for c in sq], "pack_num": 3, "shift_bit": 77,
                           "out": [ctj(c) for c in O.pack_squeeze(pk, sq, 3, 77)]}
    return out


def main() -> None:
    rng = random.Random(SEED)
    built = {}
    for bits, ne, na, nm in ((1024, 96, 48, 32), (2048, 48, 24, 16)):
        fx = build(bits, ne, na, nm, rng)
        built[bits] = fx
        path = os.path.join(HERE, f"paillier_{bits}.json")
        with open(path, "w") as f:
            json.dump(fx, f, separators=(",", ":"))
        print(path, os.path.getsize(path))
    # the ops fixtures draw from their own seed, so adding them left the files above unchanged
    rng_ops = random.Random(SEED + 1)
    for bits in (1024, 2048):
        path = os.path.join(HERE, f"paillier_{bits}_ops.json")
        with open(path, "w") as f:
            json.dump(build_ops(built[bits], rng_ops), f, separators=(",", ":"))
        print(path, os.path.getsize(path))


if __name__ == "__main__":
    main()
