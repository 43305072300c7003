"""Exponent gaps beyond the add kernel's exact range.

The reference aligns exponents with ``decrese_exp_to`` -- c^(16^gap) mod n^2, for any i32 gap
(fixedpoint_paillier/src/lib.rs:250-258, used by Ciphertext::add :301-333).  k_add27 squares
exactly up to kMaxGap = 65536 steps; beyond that fate_amd.paillier splits the alignment into
fphe_align steps of at most 65536 (``_prealign``), up to MAX_EXACT_GAP = 2^20, and raises
ValueError past it.  Such exponents come only from crafted or corrupt states: the vectors here
are unpickled from the reference's bincode with crafted exponents.  Each gap near 65536 costs
~262k squarings on one wave (~8 s at 1024 bits) and as many in the oracle's pow."""
import json
import os
import pickle

import pytest
import torch

from fate_amd import paillier as P
from fate_amd import wire
from oracle import paillier_oracle as O

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def k1024():
    with open(os.path.join(HERE, "golden", "paillier_1024.json")) as f:
        fx = json.load(f)
    p, q = int(fx["p"], 16), int(fx["q"], 16)
    sk, pk, coder = P.keypair_from_primes(p, q)
    osk, opk = O.keypair_from_primes(p, q)
    return sk, pk, coder, osk, opk, None


def _unpickled(pk, cs, exps):
    """A device vector unpickled from the reference's state (bincode of signed integers,
    paillier.rs:219-226) with the given exponents: key-less until an op hands it the key."""
    v = P.CiphertextVector.from_signed_ints(cs, exps, pk.ns, pk._key.L2)
    buf = pickle.dumps(v)
    back = pickle.loads(buf)
    assert back.raw and back.to_signed_ints() == (cs, exps)
    return back


def _cts(opk, k, seed):
    return [O.fp_encrypt(opk, O.encode_f64(opk.n, 0.5 + i * 1.25 * (-1) ** i), True, 3 + 7 * i + seed).c
            for i in range(k)]


def test_add_exact_across_kernel_gap_limit(k1024):
    """gaps 65,535 / 65,536 / 65,537 either way, small gaps, a literal 1 facing a 300,000 gap
    (add's identity: returned untouched), and negative signed integers: bit-exact with
    oracle.ct_add."""
    sk, pk, coder, osk, opk, _ = k1024
    ca = _cts(opk, 8, 1)
    cb = _cts(opk, 8, 2)
    ca[5] = -ca[5]  # a negative signed ciphertext (truncating %: the reference keeps its sign)
    ea = [0, 0, 0, -65537, 5, -14, 0, 0]
    eb = [-65535, -65536, -65537, 0, 3, -14, -300000, -2]
    ca[6] = 1  # literal 1 against a far lower exponent
    a = _unpickled(pk, ca, ea)
    b = _unpickled(pk, cb, eb)
    s = a.add(pk, b)
    got = s.to_signed_ints(pk.ns)
    want = [O.ct_add(opk, O.Ciphertext(x, ex), O.Ciphertext(y, ey)) for x, ex, y, ey in zip(ca, ea, cb, eb)]
    assert got == ([w.c for w in want], [w.exp for w in want])
    # and their decryptions (CRT decrypt of the Montgomery-resident sums)
    dec = sk.decrypt_to_encoded(s)
    sig, exp = dec.to_ints()
    ow = [O.fp_decrypt(osk, w) for w in want]
    assert (sig, exp) == ([d.significant for d in ow], [d.exp for d in ow])


def test_add_scalar_broadcast_beyond_kernel_gap(k1024):
    """The broadcast form (add_scalar, paillier.rs:346) with one element 65,540 steps above."""
    sk, pk, coder, osk, opk, _ = k1024
    ca = _cts(opk, 3, 5)
    cb = _cts(opk, 1, 6)
    ea, eb = [0, -65540, 3], [-65540]
    a = _unpickled(pk, ca, ea)
    b = _unpickled(pk, cb, eb)
    got = a.add_scalar(pk, P.Ciphertext(b)).to_signed_ints(pk.ns)
    want = [O.ct_add(opk, O.Ciphertext(x, ex), O.Ciphertext(cb[0], eb[0])) for x, ex in zip(ca, ea)]
    assert got == ([w.c for w in want], [w.exp for w in want])


def test_add_gap_beyond_exact_limit_raises(k1024):
    """Past MAX_EXACT_GAP (2^20 steps, 4 x 2^20 squarings per element) the add raises
    ValueError instead of running for hours; a literal 1 at that gap is still add's identity."""
    sk, pk, coder, osk, opk, _ = k1024
    ca, cb = _cts(opk, 2, 7), _cts(opk, 2, 8)
    g = P.MAX_EXACT_GAP + 1
    a = _unpickled(pk, ca, [0, 0])
    b = _unpickled(pk, cb, [-g, -1])
    with pytest.raises(ValueError, match="exponent gap"):
        a.add(pk, b)
    lit = _unpickled(pk, [1, ca[1]], [0, 0])
    got = lit.add(pk, b).to_signed_ints(pk.ns)
    want = [O.ct_add(opk, O.Ciphertext(1, 0), O.Ciphertext(cb[0], -g)),
            O.ct_add(opk, O.Ciphertext(ca[1], 0), O.Ciphertext(cb[1], -1))]
    assert got == ([w.c for w in want], [w.exp for w in want])


def test_iupdate_exact_beyond_kernel_gap(k1024):
    """The device-grouped fold (fphe_fold_segments) flags a per-slot exponent gap beyond its
    alignment range; iupdate then folds by the exact path (torch grouping, pairwise ct-add
    with the split alignment): bit-exact with the reference's sequential iupdate
    (fixedpoint_paillier/src/lib.rs:724-735)."""
    sk, pk, coder, osk, opk, _ = k1024
    cs = _cts(opk, 5, 9)
    exps = [0, -65537, -3, -3, 2]
    src = _unpickled(pk, cs, exps)
    hist = P.CiphertextVector.zeros(3, pk._key.L2)
    positions = [[0], [0], [1], [0, 2], [2]]
    hist.iupdate(src, positions, 1, pk)
    want = [O.ct_zero() for _ in range(3)]
    O.iupdate(opk, want, [O.Ciphertext(c, e) for c, e in zip(cs, exps)], positions, 1)
    assert hist.to_signed_ints(pk.ns) == ([w.c for w in want], [w.exp for w in want])


def test_wire_state_carries_extreme_exponents(k1024):
    """i32 extremes survive the reference's pickle state unchanged (bincode i32)."""
    sk, pk, coder, osk, opk, _ = k1024
    cs = _cts(opk, 2, 10)
    v = _unpickled(pk, cs, [2 ** 31 - 1, -2 ** 31])
    state = wire.ciphertext_vector_to_bincode(v)
    back, used = wire.ciphertext_vector_from_bincode(state)
    assert used == len(state) and back.to_signed_ints() == (cs, [2 ** 31 - 1, -2 ** 31])


def test_iupdate_exact_gap_between_histogram_and_terms(k1024):
    """The histogram's own values sit 70,000 exponents away from the folded terms: iupdate's
    final ct-add (queued without a gap read-back) flags it, and the add is redone pre-aligned
    -- bit-exact with the reference's sequential iupdate."""
    sk, pk, coder, osk, opk, _ = k1024
    cs = _cts(opk, 4, 11)
    hc = _cts(opk, 3, 12)
    hexps = [70000, -70000, 1]
    exps = [0, 0, 2, -1]
    hist = _unpickled(pk, hc, hexps)
    src = _unpickled(pk, cs, exps)
    positions = [[0], [1], [2, 0], [1]]
    hist.iupdate(src, positions, 1, pk)
    want = [O.Ciphertext(c, e) for c, e in zip(hc, hexps)]
    O.iupdate(opk, want, [O.Ciphertext(c, e) for c, e in zip(cs, exps)], positions, 1)
    assert hist.to_signed_ints(pk.ns) == ([w.c for w in want], [w.exp for w in want])


def test_forced_raise_skips_gap_beyond_kernel_limit(k1024, monkeypatch):
    """FPHE_FOLD_RAISE=force makes every key above its segment's least exponent a raise
    candidate; a key 65,537 steps up is beyond what k_segfold27 squares (4 kMaxGap) and must
    stay out of the slot plan: the fold then takes the exact path and matches the
    reference's sequential iupdate.  The segment also holds a key 2 steps up, which is raised."""
    sk, pk, coder, osk, opk, _ = k1024
    cs = _cts(opk, 6, 13)
    exps = [-65537, 0, -65535, -65535, -65537, 1]
    monkeypatch.setenv("FPHE_FOLD_RAISE", "force")
    src = _unpickled(pk, cs, exps)
    hist = P.CiphertextVector.zeros(2, pk._key.L2)
    positions = [[0], [0], [0, 1], [0], [1], [1]]
    hist.iupdate(src, positions, 1, pk)
    want = [O.ct_zero() for _ in range(2)]
    O.iupdate(opk, want, [O.Ciphertext(c, e) for c, e in zip(cs, exps)], positions, 1)
    assert hist.to_signed_ints(pk.ns) == ([w.c for w in want], [w.exp for w in want])


def test_stale_exponent_bound_is_caught(k1024):
    """ct-add skips the gap read-back when the host-side bounds (ebound) keep every
    gap within the kernel's exact range.  With FPHE_CHECK_EBOUND=1 (set for the test suite,
    tests/conftest.py) a bound that no longer covers the exponents fails loudly instead of
    giving a silently wrong sum."""
    sk, pk, coder, osk, opk, _ = k1024
    assert P.CHECK_EBOUND
    x = torch.tensor([1.5, -2.25, 1e-20, 3e10], dtype=torch.float64).cuda()
    a = pk.encrypt_encoded(coder.encode_f64_vec(x), True)
    b = pk.encrypt_encoded(coder.encode_f64_vec(x * 0.5), True)
    a.add(pk, b)  # sound bounds: passes
    lo, hi = a.ebound
    a.ebound = (hi, hi)  # stale: the exponents span [lo, hi] with lo < hi
    assert lo < hi
    with pytest.raises(AssertionError, match="stale exponent bound"):
        a.add(pk, b)
