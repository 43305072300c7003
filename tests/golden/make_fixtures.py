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


def main() -> None:
    rng = random.Random(SEED)
    for bits, ne, na, nm in ((1024, 96, 48, 32), (2048, 48, 24, 16)):
        fx = build(bits, ne, na, nm, rng)
        path = os.path.join(HERE, f"paillier_{bits}.json")
        with open(path, "w") as f:
            json.dump(fx, f, separators=(",", ":"))
        print(path, os.path.getsize(path))


if __name__ == "__main__":
    main()
