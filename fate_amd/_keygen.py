"""Paillier key generation (host side, once per job -- not on the hot path).

Follows ``paillier::keygen`` (rust/fate_utils/crates/paillier/src/lib.rs:72-87) and
``BInt::gen_prime`` (rust/fate_utils/crates/math/src/rug/random.rs:27-32): each prime is
``next_prime(random k/2-bit integer with its top bit set)``, retried until ``p != q`` and
``n = p*q`` has exactly ``k`` bits.  Primality: Miller-Rabin with 40 random bases after
trial division (GMP's ``mpz_nextprime`` is a probabilistic test as well).
"""
from __future__ import annotations

import secrets
from typing import Tuple

_SMALL_PRIMES = []


def _small_primes(limit: int = 2000):
    if not _SMALL_PRIMES:
        sieve = bytearray([1]) * limit
        sieve[0:2] = b"\x00\x00"
        for i in range(2, int(limit ** 0.5) + 1):
            if sieve[i]:
                sieve[i * i::i] = bytearray(len(sieve[i * i::i]))
        _SMALL_PRIMES.extend(i for i in range(limit) if sieve[i])
    return _SMALL_PRIMES


def is_probable_prime(n: int, rounds: int = 40) -> bool:
    if n < 2:
        return False
    for p in _small_primes():
        if n == p:
            return True
        if n % p == 0:
            return False
    d, s = n - 1, 0
    while d % 2 == 0:
        d //= 2
        s += 1
    for _ in range(rounds):
        a = 2 + secrets.randbelow(n - 3)
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


def next_prime(x: int) -> int:
    """Smallest probable prime > x (``Integer::next_prime_mut``)."""
    c = x + 1
    if c <= 2:
        return 2
    if c % 2 == 0:
        c += 1
    while not is_probable_prime(c):
        c += 2
    return c


def gen_prime(bit_size: int) -> int:
    x = secrets.randbits(bit_size) | (1 << (bit_size - 1))
    return next_prime(x)


def keygen_primes(bit_length: int) -> Tuple[int, int]:
    """Return (p, q) with p < q, p != q, bits(p*q) == bit_length."""
    if bit_length % 2 != 0:
        # paillier/src/lib.rs:73 `assert_eq!(bit_lenght % 2, 0)` panics
        raise AssertionError("assertion failed: bit_length % 2 == 0")
    half = bit_length // 2
    while True:
        p = gen_prime(half)
        q = gen_prime(half)
        if p != q and (p * q).bit_length() == bit_length:
            return (p, q) if p < q else (q, p)
