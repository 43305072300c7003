"""CPU restatement of the reference Paillier hot path -- TEST INFRASTRUCTURE ONLY.

This module is the parity oracle.  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import it, and only as the checker.  The
product path (``fate_amd``) never imports anything under ``oracle/``.

It restates, line by line, the semantics of the Rust crates the reference ships:

* ``rust/fate_utils/crates/paillier/src/lib.rs``          (L0: keygen/encrypt/decrypt/add_ct/mul_pt)
* ``rust/fate_utils/crates/fixedpoint_paillier/src/lib.rs``(L1: fixed-point coder, Ciphertext, vectors)
* ``rust/fate_utils/crates/math/src/rug/{mod,ops}.rs``     (BInt = rug::Integer semantics)

Integers are Python ints, which are exact and signed like ``rug::Integer``.  The
reference's big-integer library is rug 1.20.1 (``rust/fate_utils/Cargo.toml:8``)
over GMP; the GMP semantics we depend on are:

* ``%`` / ``/`` on ``rug::Integer`` truncate toward zero (``mpz_tdiv_r`` /
  ``mpz_tdiv_q``; ``math/src/rug/ops.rs:91-97`` maps ``Rem``/``Div`` straight
  onto rug).  Python's ``%`` floors, so :func:`tdiv_r` / :func:`tdiv_q` restate
  truncation explicitly.
* ``pow_mod`` (``mpz_powm``) and ``invert`` (``mpz_invert``) return canonical
  residues in ``[0, m)``; a negative exponent means "invert the base first"
  (``math/src/rug/mod.rs:22-35``).  Python's three-argument ``pow`` has the
  same contract.

Parity status: the reference holds no known-answer ciphertext vectors
 and its Rust cannot be built here (no cargo/rustc), so this
restatement is pinned by (1) the reference's own round-trip tests
(``crates/paillier/src/lib.rs:190-197``, ``python/fate/test/test_paillier.py``,
``python/fate/test/test_vertor_paillier.py``), replayed in ``tests/``, and (2)
an independent cross-check against libgmp 6.2.1 -- the library rug wraps -- via
``oracle/gmp_ref.c``.  Ciphertext-integer known-answer parity against the
reference binary itself is therefore "parity unpinned" (see DESIGN.md §Oracle).
"""
from __future__ import annotations

import math
import struct
from dataclasses import dataclass
from fractions import Fraction
from typing import List, Optional, Sequence, Tuple

BASE = 16                      # fixedpoint_paillier/src/lib.rs:13
MAX_INT_FRACTION = 2           # :14
FLOAT_MANTISSA_BITS = 53       # :15
LOG2_BASE = 4                  # :16


# --------------------------------------------------------------------------------------
# rug / GMP integer semantics (math/src/rug/{mod,ops}.rs)
# --------------------------------------------------------------------------------------
def tdiv_q(a: int, m: int) -> int:
    """Truncating quotient, ``mpz_tdiv_q`` (rug ``Div``, math/src/rug/ops.rs:91-97)."""
    q = abs(a) // abs(m)
    return q if (a >= 0) == (m > 0) else -q


def tdiv_r(a: int, m: int) -> int:
    """Truncating remainder, sign of the dividend (rug ``Rem``, math/src/rug/ops.rs:91-97)."""
    r = abs(a) % abs(m)
    return r if a >= 0 else -r


def powm(b: int, e: int, m: int) -> int:
    """``BInt::pow_mod_ref`` -> ``mpz_powm`` (math/src/rug/mod.rs:22-29).

    Canonical result; negative ``e`` inverts the base (panics via ``unwrap`` in the
    reference if not invertible -> ``ValueError`` here)."""
    return pow(b, e, m)


def invert(a: int, m: int) -> int:
    """``BInt::invert`` -> ``mpz_invert`` (math/src/rug/mod.rs:30-35), canonical."""
    return pow(a, -1, m)


# --------------------------------------------------------------------------------------
# L0: crates/paillier/src/lib.rs
# --------------------------------------------------------------------------------------
@dataclass(frozen=True)
class PK:
    n: int
    ns: int  # n*n  (paillier/src/lib.rs:50-53, 90-93)

    @property
    def max_int(self) -> int:
        # fixedpoint_paillier/src/lib.rs:408-413: max_int = n / MAX_INT_FRACTION (truncating)
        return self.n // MAX_INT_FRACTION


@dataclass(frozen=True)
class SK:
    p: int
    q: int
    n: int
    p_minus_one: int
    q_minus_one: int
    ps: int
    qs: int
    p_invert: int
    hp: int
    hq: int


def sk_new(p: int, q: int) -> SK:
    """``SK::new`` (paillier/src/lib.rs:125-150): swap so p<q, precompute CRT constants."""
    assert p != q, "p == q"
    if not p < q:
        p, q = q, p
    n = p * q
    ps, qs = p * p, q * q
    p_invert = invert(p, q)
    g = p * q + 1
    hp = invert(tdiv_q(powm(g, p - 1, ps) - 1, p), p)
    hq = invert(tdiv_q(powm(g, q - 1, qs) - 1, q), q)
    return SK(p, q, n, p - 1, q - 1, ps, qs, p_invert, hp, hq)


def keypair_from_primes(p: int, q: int) -> Tuple[SK, PK]:
    """``paillier::keygen`` tail (paillier/src/lib.rs:72-87) for given primes."""
    sk = sk_new(p, q)
    n = p * q
    return sk, PK(n, n * n)


def encrypt(pk: PK, m: int, obfuscate: bool, r: Optional[int] = None) -> int:
    """``PK::encrypt`` (paillier/src/lib.rs:104-121) with ``random_rn`` (:94-98).

    ``r`` is the draw of ``gen_positive_integer(n)`` (math/src/rug/random.rs:22-25),
    injected because the reference draws it from fresh OS entropy per element."""
    if m > (pk.n >> 2):
        neg_plaintext = pk.n - m
        neg_ciphertext = tdiv_r(pk.n * neg_plaintext + 1, pk.ns)
        nude = invert(neg_ciphertext, pk.ns)
    else:
        nude = tdiv_r(m * pk.n + 1, pk.ns)
    if obfuscate:
        if r is None:
            raise ValueError("oracle needs an injected r for obfuscated encryption")
        if not 1 <= r <= pk.n - 1:
            raise ValueError("r must lie in [1, n-1] (random.rs:22-25)")
        rn = powm(r, pk.n, pk.ns)
        return tdiv_r(nude * rn, pk.ns)
    return nude


def decrypt(sk: SK, c: int) -> int:
    """``SK::decrypt`` + ``h_function`` (paillier/src/lib.rs:163-176)."""
    dp = _h(c, sk.p, sk.p_minus_one, sk.ps, sk.hp)
    dq = _h(c, sk.q, sk.q_minus_one, sk.qs, sk.hq)
    o = tdiv_r((dq - dp) * sk.p_invert, sk.q) * sk.p + dp
    if o < 0:
        o += sk.n
    return o


def _h(c: int, p: int, p_1: int, ps: int, hp: int) -> int:
    return tdiv_r(tdiv_q(powm(c, p_1, ps) - 1, p) * hp, p)


def add_ct(pk: PK, a: int, b: int) -> int:
    """``CT::add_ct`` (paillier/src/lib.rs:35-37): product, truncating remainder."""
    return tdiv_r(a * b, pk.ns)


def mul_pt(pk: PK, c: int, b: int) -> int:
    """``CT::mul_pt`` (paillier/src/lib.rs:41-43): ``c.pow_mod_ref(b, ns)``."""
    return powm(c, b, pk.ns)


# --------------------------------------------------------------------------------------
# L1: crates/fixedpoint_paillier/src/lib.rs
# --------------------------------------------------------------------------------------
@dataclass
class Plaintext:
    significant: int
    exp: int


@dataclass
class Ciphertext:
    c: int          # signed ciphertext integer (rug::Integer)
    exp: int

    def copy(self) -> "Ciphertext":
        return Ciphertext(self.c, self.exp)


def frexp_exponent(x: float) -> int:
    """libc ``frexp`` exponent (fixedpoint_paillier/src/frexp.rs:12-17)."""
    if x == 0.0 or math.isnan(x) or math.isinf(x):
        return 0  # glibc: frexp(0)=0, frexp(inf/nan) leaves exp=0
    return math.frexp(x)[1]


def _round_half_away(fr: Fraction) -> int:
    # rug Float::round (mpfr_round): ties away from zero
    neg = fr < 0
    a = -fr if neg else fr
    fl = a.numerator // a.denominator
    rem = a - fl
    if rem * 2 >= 1:
        fl += 1
    return -fl if neg else fl


def encode_f64(n: int, x: float) -> Plaintext:
    """``Coder::encode_f64`` (fixedpoint_paillier/src/lib.rs:148-168)."""
    if math.isnan(x) or math.isinf(x):
        # `.to_integer().unwrap()` on a non-finite Float panics (:152-157)
        raise OverflowError("cannot encode non-finite float")
    e = frexp_exponent(x)
    lsb = e - FLOAT_MANTISSA_BITS
    exp = math.floor(lsb / LOG2_BASE)
    sig = _round_half_away(Fraction(x) * Fraction(BASE) ** (-exp))
    max_int = n // MAX_INT_FRACTION
    if abs(sig) > max_int:
        raise OverflowError(f"Integer needs to be within +/- {max_int} but got {sig}")
    return Plaintext(sig, exp)


def encode_f32(n: int, x) -> Plaintext:
    """``Coder::encode_f32`` (:187-189): widen to f64 first."""
    return encode_f64(n, float(struct.unpack("<f", struct.pack("<f", float(x)))[0]))


def encode_i64(n: int, v: int) -> Plaintext:
    """``Coder::encode_i64`` / ``encode_i32`` (:68-78, :119-129)."""
    return Plaintext(n + v if v < 0 else v, 0)


def _mantissa(n: int, sig: int) -> int:
    # decode_f64 / decode_i64 guard (:130-142, :169-180)
    max_int = n // MAX_INT_FRACTION
    if sig > n:
        raise ValueError("Attempted to decode corrupted number")
    if sig <= max_int:
        return sig
    if sig >= n - max_int:
        return sig - n
    raise OverflowError("Overflow detected in decrypted number")


def _int_to_f64_trunc(v: int) -> float:
    """``rug::Integer::to_f64``: round toward zero (mpz_get_d).  Unverified vs real rug
    (SURVEY.md §8c); fixtures avoid depending on it for >53-bit values."""
    if v == 0:
        return 0.0
    neg = v < 0
    a = -v if neg else v
    bl = a.bit_length()
    if bl > 53:
        a = (a >> (bl - 53)) << (bl - 53)
    if bl > 1024:
        return -math.inf if neg else math.inf
    f = float(a)  # exact now (<=53 significant bits)
    return -f if neg else f


def _round_rne_bits(num: int, den_log2: int, prec: int) -> Fraction:
    """Round num * 2^-den_log2 (num != 0) to ``prec`` significant bits, ties-to-even,
    with an unbounded exponent (MPFR)."""
    neg = num < 0
    a = -num if neg else num
    bl = a.bit_length()
    shift = bl - prec
    if shift > 0:
        q, rem = a >> shift, a & ((1 << shift) - 1)
        half = 1 << (shift - 1)
        if rem > half or (rem == half and (q & 1)):
            q += 1
        a = q << shift
    val = Fraction(a, 1 << den_log2) if den_log2 >= 0 else Fraction(a * (1 << -den_log2))
    return -val if neg else val


def decode_f64(n: int, sig: int, exp: int) -> float:
    """``Coder::decode_f64`` (fixedpoint_paillier/src/lib.rs:169-186)."""
    m = _mantissa(n, sig)
    if exp >= 0:
        return _int_to_f64_trunc(m << (LOG2_BASE * exp))
    if m == 0:
        return 0.0
    # mantissa * Float(53, 16)^exp : MPFR product rounded to 53 bits (RNE), then
    # mpfr_get_d (RNE, may round again into the subnormal range).
    v = _round_rne_bits(m, -LOG2_BASE * exp, FLOAT_MANTISSA_BITS)
    return float(v)  # Fraction->float is correctly rounded (RNE)


def decode_f32(n: int, sig: int, exp: int):
    """``Coder::decode_f32`` (:190-192): ``decode_f64 as f32`` (RNE)."""
    import numpy as np
    return np.float32(decode_f64(n, sig, exp))


def decode_i64(n: int, sig: int, exp: int) -> int:
    """``Coder::decode_i64`` (:130-142): (mantissa << 4*exp) -> i128 -> wraps to i64."""
    m = _mantissa(n, sig)
    v = m << (LOG2_BASE * exp) if exp >= 0 else m >> (-LOG2_BASE * exp)
    if not -(1 << 127) <= v < (1 << 127):
        raise OverflowError("cant't convert to i128")
    v &= (1 << 64) - 1
    return v - (1 << 64) if v >= (1 << 63) else v


def pack_floats(floats: Sequence[float], offset_bit: int, pack_num: int, precision: int) -> List[Plaintext]:
    """``Coder::pack_floats`` (:79-93)."""
    out = []
    for i in range(0, len(floats), pack_num):
        acc = 0
        for v in floats[i:i + pack_num]:
            acc <<= offset_bit
            acc += _round_half_away(Fraction(float(v)) * (1 << precision))
        out.append(Plaintext(acc, 0))
    return out


def unpack_floats(encoded: Sequence[Plaintext], offset_bit: int, pack_num: int, precision: int,
                  total_num: int) -> List[float]:
    """``Coder::unpack_floats`` (:94-118); Rational::to_f64 truncates (SURVEY §8c caveat)."""
    mask = (1 << offset_bit) - 1
    res: List[float] = []
    remaining = total_num
    for x in encoded:
        k = min(remaining, pack_num)
        sig = x.significant
        tmp = []
        for _ in range(k):
            fr = Fraction(sig & mask, 1 << precision)
            tmp.append(_fraction_to_f64_trunc(fr))
            sig >>= offset_bit
        tmp.reverse()
        res.extend(tmp)
        remaining -= k
    return res


def _fraction_to_f64_trunc(fr: Fraction) -> float:
    if fr == 0:
        return 0.0
    f = float(fr)
    if abs(Fraction(f)) > abs(fr):
        f = math.nextafter(f, 0.0)
    return f


# ---- Ciphertext (fixedpoint_paillier/src/lib.rs:237-350) ------------------------------
def ct_zero() -> Ciphertext:
    """``Ciphertext::zero`` (:244-249): literal 1, exp 0."""
    return Ciphertext(1, 0)


def fp_encrypt(pk: PK, pt: Plaintext, obfuscate: bool, r: Optional[int] = None) -> Ciphertext:
    """``PK::encrypt`` / ``encrypt_encoded`` (:24-34, :370-387)."""
    return Ciphertext(encrypt(pk, pt.significant, obfuscate, r), pt.exp)


def fp_decrypt(sk: SK, ct: Ciphertext) -> Plaintext:
    """``SK::decrypt`` / ``decrypt_to_encoded`` (:41-50, :391-406)."""
    return Plaintext(decrypt(sk, ct.c), ct.exp)


def decrese_exp_to(pk: PK, a: Ciphertext, exp: int) -> Ciphertext:
    """``Ciphertext::decrese_exp_to`` (:250-258)."""
    assert exp < a.exp
    factor = BASE ** (a.exp - exp)
    return Ciphertext(mul_pt(pk, a.c, factor), exp)


def ct_add(pk: PK, a: Ciphertext, b: Ciphertext) -> Ciphertext:
    """``Ciphertext::add`` (:301-333)."""
    if a.c == 1:
        return b.copy()
    if b.c == 1:
        return a.copy()
    if a.exp > b.exp:
        a = decrese_exp_to(pk, a, b.exp)
        return Ciphertext(add_ct(pk, a.c, b.c), b.exp)
    if a.exp < b.exp:
        b = decrese_exp_to(pk, b, a.exp)
        return Ciphertext(add_ct(pk, a.c, b.c), a.exp)
    return Ciphertext(add_ct(pk, a.c, b.c), a.exp)


def ct_neg(pk: PK, a: Ciphertext) -> Ciphertext:
    """``Ciphertext::neg`` (:259-264)."""
    return Ciphertext(invert(a.c, pk.ns), a.exp)


def ct_sub(pk: PK, a: Ciphertext, b: Ciphertext) -> Ciphertext:
    """``Ciphertext::sub`` (:280-282)."""
    return ct_add(pk, a, ct_neg(pk, b))


def ct_rsub(pk: PK, a: Ciphertext, b: Ciphertext) -> Ciphertext:
    """``Ciphertext::rsub`` (:283-285): neg(a) + b."""
    return ct_add(pk, ct_neg(pk, a), b)


def ct_add_pt(pk: PK, a: Ciphertext, b: Plaintext) -> Ciphertext:
    """``Ciphertext::add_pt`` (:265-268)."""
    return ct_add(pk, a, fp_encrypt(pk, b, False))


def ct_sub_pt(pk: PK, a: Ciphertext, b: Plaintext) -> Ciphertext:
    """``Ciphertext::sub_pt`` (:269-272)."""
    return ct_sub(pk, a, fp_encrypt(pk, b, False))


def ct_rsub_pt(pk: PK, a: Ciphertext, b: Plaintext) -> Ciphertext:
    """``Ciphertext::rsub_pt`` (:276-279): b - a."""
    return ct_sub(pk, fp_encrypt(pk, b, False), a)


def ct_mul(pk: PK, a: Ciphertext, b: Plaintext) -> Ciphertext:
    """``Ciphertext::mul`` (:334-349)."""
    max_int = pk.max_int
    if pk.n - max_int <= b.significant:
        neg_c = invert(a.c, pk.ns)
        inside = powm(neg_c, pk.n - b.significant, pk.ns)
    elif b.significant <= max_int:
        inside = powm(a.c, b.significant, pk.ns)
    else:
        raise ValueError(f"invalid plaintext: {b}")
    return Ciphertext(inside, a.exp + b.exp)


def ct_i_double(pk: PK, a: Ciphertext) -> Ciphertext:
    """``Ciphertext::i_double`` (:294-299)."""
    return Ciphertext(powm(a.c, 2, pk.ns), a.exp)


# ---- CiphertextVector (fixedpoint_paillier/src/lib.rs:415-909) -------------------------
def vec_add(pk, a, b):             # :797-805
    return [ct_add(pk, x, y) for x, y in zip(a, b)]


def vec_sub(pk, a, b):             # :812-820
    return [ct_sub(pk, x, y) for x, y in zip(a, b)]


def vec_rsub(pk, a, b):            # :827-835 (y.sub(x))
    return [ct_sub(pk, y, x) for x, y in zip(a, b)]


def vec_mul(pk, a, pts):           # :842-850
    return [ct_mul(pk, x, y) for x, y in zip(a, pts)]


def vec_idouble(pk, a):            # :753-758  x.add_assign(&x.clone())
    return [ct_add(pk, x, x.copy()) for x in a]


def pack_squeeze(pk: PK, data: List[Ciphertext], pack_num: int, shift_bit: int) -> List[Ciphertext]:
    """``CiphertextVector::pack_squeeze`` (:439-450)."""
    base = 1 << shift_bit
    out = []
    for i in range(0, len(data), pack_num):
        chunk = data[i:i + pack_num]
        res = chunk[0].c
        for y in chunk[1:]:
            res = powm(res, base, pk.ns)
            res = tdiv_r(res * y.c, pk.ns)
        out.append(Ciphertext(res, 0))
    return out


def iupdate(pk: PK, data: List[Ciphertext], other: List[Ciphertext], indexes: List[List[int]],
            stride: int) -> None:
    """``CiphertextVector::iupdate`` (:724-735), in place."""
    for i, x in enumerate(indexes):
        sb = i * stride
        for pos in x:
            sa = pos * stride
            for t in range(stride):
                data[sa + t] = ct_add(pk, data[sa + t], other[sb + t])


def iupdate_with_masks(pk, data, other, indexes, masks, stride):
    """``CiphertextVector::iupdate_with_masks`` (:736-747)."""
    value_positions = [i for i, m in enumerate(masks) if m]
    for value_pos, x in zip(value_positions, indexes):
        sb = value_pos * stride
        for pos in x:
            sa = pos * stride
            for t in range(stride):
                data[sa + t] = ct_add(pk, data[sa + t], other[sb + t])


def chunking_cumsum_with_step(pk: PK, data: List[Ciphertext], chunk_sizes: List[int], step: int) -> None:
    """``CiphertextVector::chunking_cumsum_with_step`` (:763-774), in place, with its two
    mem::replace swaps: for step > 0 that is data[i+j] = add(data[i+j], data[i+j-step]); for
    step 0 the element is added to the swapped-in literal 1, so it stays as it was."""
    placeholder = ct_zero()
    i = 0
    for cs in chunk_sizes:
        for j in range(step, cs):
            x = i + j
            placeholder, data[x] = data[x], placeholder
            placeholder = ct_add(pk, placeholder, data[x - step])
            placeholder, data[x] = data[x], placeholder
        i += cs


def intervals_sum_with_step(pk: PK, data: List[Ciphertext], intervals, step: int) -> List[Ciphertext]:
    """``CiphertextVector::intervals_sum_with_step`` (:776-791)."""
    out = [ct_zero() for _ in range(len(intervals) * step)]
    for i, (s, e) in enumerate(intervals):
        for k, val in enumerate(data[s:e]):
            c = k % step
            out[i * step + c] = ct_add(pk, out[i * step + c], val)
    return out


def matmul(pk: PK, a: List[Ciphertext], b: List[Plaintext], lshape, rshape) -> List[Ciphertext]:
    """``CiphertextVector::matmul`` (:852-880)."""
    out = [ct_zero() for _ in range(lshape[0] * rshape[1])]
    for i in range(lshape[0]):
        for j in range(rshape[1]):
            for k in range(lshape[1]):
                t = ct_mul(pk, a[i * lshape[1] + k], b[k * rshape[1] + j])
                out[i * rshape[1] + j] = ct_add(pk, out[i * rshape[1] + j], t)
    return out


def rmatmul(pk: PK, a: List[Ciphertext], b: List[Plaintext], lshape, rshape) -> List[Ciphertext]:
    """``CiphertextVector::rmatmul`` (:882-908)."""
    out = [ct_zero() for _ in range(lshape[1] * rshape[0])]
    for i in range(rshape[0]):
        for j in range(lshape[1]):
            for k in range(rshape[1]):
                t = ct_mul(pk, a[k * lshape[1] + j], b[i * rshape[1] + k])
                out[i * lshape[1] + j] = ct_add(pk, out[i * lshape[1] + j], t)
    return out


def i_shuffle(data: list, indexes: List[int]) -> None:
    """``CiphertextVector::i_shuffle`` (:473-490): cycle-walk swap, in place."""
    visited = [False] * len(data)
    for i in range(len(data)):
        if visited[i] or indexes[i] == i:
            continue
        current = i
        nxt = indexes[current]
        while not visited[nxt] and nxt != i:
            data[current], data[nxt] = data[nxt], data[current]
            visited[current] = True
            current = nxt
            nxt = indexes[current]
        visited[current] = True


# --------------------------------------------------------------------------------------
# Device representation helpers (SURVEY.md Appendix A "Device mapping")
# --------------------------------------------------------------------------------------
def to_device_repr(pk: PK, c: int) -> Tuple[int, int]:
    """signed ciphertext -> (canonical residue C in [0, n^2), sign bit)."""
    if c < 0:
        return c + pk.ns, 1
    return c, 0


def from_device_repr(pk: PK, C: int, s: int) -> int:
    return C - pk.ns if (s and C != 0) else C
