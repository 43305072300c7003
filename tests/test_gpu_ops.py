"""GPU parity of the vector algebra beyond encrypt/decrypt/add/mul: the modular inverse
(neg, sub, rsub, the invert branches of ct x pt) and the SecureBoost / Hetero-LR vector
ops (iupdate, chunking_cumsum_with_step, intervals_sum_with_step, pack_squeeze, matmul,
rmatmul, iadd/isub_vec_self).  Expected values come from the CPU oracle
(oracle/paillier_oracle.py, pinned against libgmp in tests/test_oracle.py) evaluated on
the same inputs; comparison is bit-exact on signed ciphertext integers and exponents."""
import json
import os
import random

import pytest
import torch

from fate_amd import paillier as P
from oracle import paillier_oracle as O

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def load(bits):
    with open(os.path.join(HERE, "golden", f"paillier_{bits}.json")) as f:
        fx = json.load(f)
    p, q = int(fx["p"], 16), int(fx["q"], 16)
    sk, pk, coder = P.keypair_from_primes(p, q)
    osk, opk = O.keypair_from_primes(p, q)
    cts = [O.Ciphertext(int(c, 16), e) for c, e in zip(fx["encrypt"]["ct"], fx["encrypt"]["exp"])]
    return fx, sk, pk, coder, opk, cts


@pytest.fixture(params=[1024, 2048], scope="module")
def env(request):
    return load(request.param)


def more(opk, cts, k, seed=0):
    """cts extended to k ciphertexts with random signed integers in (-n^2, n^2) and small
    exponents: the vector algebra is exact integer arithmetic on any such values (they need
    not be encryptions), and the oracle at 2048 bits costs ~0.14 s per real encryption."""
    rng = random.Random(1000 + seed)
    out = list(cts)
    while len(out) < k:
        c = rng.randrange(2, opk.ns)
        out.append(O.Ciphertext(-c if rng.random() < 0.3 else c, rng.choice([0, -13, -14, -12])))
    return out


def dev_vec(pk, cts):
    return P.CiphertextVector.from_signed_ints([c.c for c in cts], [c.exp for c in cts], pk.ns, pk._key.L2)


def host(pk, v):
    cs, es = v.to_signed_ints(pk.ns)
    return list(zip(cs, es))


def ref(cts):
    return [(c.c, c.exp) for c in cts]


def test_neg(env):
    fx, sk, pk, coder, opk, cts = env
    cts = cts + [O.ct_zero()]  # inv(1) = 1
    out = dev_vec(pk, cts).neg(pk)
    assert host(pk, out) == ref([O.ct_neg(opk, c) for c in cts])


@pytest.mark.parametrize("count", [4096, 8192 + 37, 3 * 4096 + 64 * 5 + 1])
def test_neg_batch_inversion(env, count):
    """Vectors of >= 4096 elements take the batch-inversion path (k_binv_pre27, one safegcd
    inverse per group of 16/8 elements, k_binv_post27): ragged tails, literal 1s and
    negative (sign 1) ciphertexts mixed in, bit-exact against the oracle's invert."""
    fx, sk, pk, coder, opk, cts = env
    rng = random.Random(count)
    pool = cts + [O.ct_zero()] + [O.Ciphertext(c.c - opk.ns if c.c > 0 else c.c + opk.ns, c.exp) for c in cts[:8]]
    want = {i: O.ct_neg(opk, c) for i, c in enumerate(pool)}
    pick = [rng.randrange(len(pool)) for _ in range(count)]
    out = dev_vec(pk, [pool[i] for i in pick]).neg(pk)
    assert host(pk, out) == ref([want[i] for i in pick])


@pytest.mark.parametrize("count", [100, 5000])
def test_neg_not_invertible_panics(env, count):
    """invert().unwrap() panics on a non-unit (math/src/rug/mod.rs:30-35); the batch path
    raises it through the group total's inverse."""
    fx, sk, pk, coder, opk, cts = env
    bad = [cts[i % len(cts)] for i in range(count)]
    bad[count // 3] = O.Ciphertext(int(fx["p"], 16), 0)  # shares the factor p with n^2
    with pytest.raises(P.PanicException):
        dev_vec(pk, bad).neg(pk)


def test_sub_rsub(env):
    fx, sk, pk, coder, opk, cts = env
    a, b = cts[:40], cts[40:80]
    va, vb = dev_vec(pk, a), dev_vec(pk, b)
    assert host(pk, va.sub(pk, vb)) == ref(O.vec_sub(opk, a, b))
    assert host(pk, va.rsub(pk, vb)) == ref(O.vec_rsub(opk, a, b))
    s = P.Ciphertext(dev_vec(pk, [b[3]]))
    assert host(pk, va.sub_scalar(pk, s)) == ref([O.ct_sub(opk, x, b[3]) for x in a])
    assert host(pk, va.rsub_scalar(pk, s)) == ref([O.ct_sub(opk, b[3], x) for x in a])


def test_decrypt_of_sub(env):
    """dec(enc(x) - enc(y)) == x - y (reference round-trip style, crates/paillier/src/lib.rs:190-197)."""
    fx, sk, pk, coder, opk, cts = env
    xs = fx["encrypt"]["x_f32"]
    h = len(xs) // 2
    x = torch.tensor(xs[:h], dtype=torch.float64)
    y = torch.tensor(xs[h:2 * h], dtype=torch.float64)
    ex = pk.encrypt_encoded(coder.encode_f64_vec(x.cuda()), True)
    ey = pk.encrypt_encoded(coder.encode_f64_vec(y.cuda()), True)
    d = coder.decode_f64_vec(sk.decrypt_to_encoded(ex.sub(pk, ey))).cpu()
    assert torch.allclose(d, x - y, rtol=0, atol=1e-9 * float((x.abs() + y.abs()).max()))


def test_mul_negative_and_big_plaintexts(env):
    fx, sk, pk, coder, opk, cts = env
    rng = random.Random(5)
    c = cts[:32]
    sigs, exps = [], []
    for i in range(32):
        k = i % 4
        if k == 0:
            sigs.append(-rng.randrange(1, 1 << 53))          # negative float significand
        elif k == 1:
            sigs.append(opk.n - rng.randrange(1, 1 << 40))   # encoded negative int ("big")
        elif k == 2:
            sigs.append(rng.randrange(0, 1 << 56))           # ordinary
        else:
            sigs.append(-1)
        exps.append(rng.randrange(-20, 3))
    pv = P.PlaintextVector.from_ints(sigs, exps)
    want = [O.ct_mul(opk, x, O.Plaintext(s, e)) for x, s, e in zip(c, sigs, exps)]
    assert host(pk, dev_vec(pk, c).mul(pk, pv)) == ref(want)


@pytest.mark.parametrize("count", [4096 + 3, 9000])
def test_mul_invert_branches_batch(env, count):
    """ct x pt over >= 4096 elements: the invert branches (negative significands, encoded
    negative ints) take the masked batch inversion; elements that need no inverse act as 1
    in their group.  Bit-exact against the oracle on a pool of (ct, pt) pairs."""
    fx, sk, pk, coder, opk, cts = env
    rng = random.Random(count)
    pool = []
    for i in range(64):
        k = i % 4
        sig = (-rng.randrange(1, 1 << 53) if k == 0 else opk.n - rng.randrange(1, 1 << 20) if k == 1
               else rng.randrange(0, 1 << 56) if k == 2 else -1)
        pool.append((cts[i % len(cts)], sig, rng.randrange(-20, 3)))
    want = [O.ct_mul(opk, c, O.Plaintext(s_, e_)) for c, s_, e_ in pool]
    pick = [rng.randrange(len(pool)) for _ in range(count)]
    pv = P.PlaintextVector.from_ints([pool[i][1] for i in pick], [pool[i][2] for i in pick])
    got = dev_vec(pk, [pool[i][0] for i in pick]).mul(pk, pv)
    assert host(pk, got) == ref([want[i] for i in pick])


def test_mul_plaintext_edges(env):
    """Edges of Ciphertext::mul's classification (lib.rs:334-349).  For odd n,
    max_int + 1 == n - max_int, so no significand below n is "invalid"; P > n takes the
    inverse branch with a negative exponent, which GMP turns back into c^(P - n)."""
    fx, sk, pk, coder, opk, cts = env
    sigs = [opk.max_int, opk.max_int + 1, opk.n - 1, opk.n, opk.n + 5, 0]
    c = cts[:len(sigs)]
    pv = P.PlaintextVector.from_ints(sigs, [0] * len(sigs))
    want = [O.ct_mul(opk, x, O.Plaintext(s, 0)) for x, s in zip(c, sigs)]
    assert host(pk, dev_vec(pk, c).mul(pk, pv)) == ref(want)


def test_pack_squeeze(env):
    fx, sk, pk, coder, opk, cts = env
    data = cts[:23]  # ragged last chunk
    for pack_num, shift in ((2, 77), (3, 20), (1, 5)):
        got = dev_vec(pk, data).pack_squeeze(pack_num, shift, pk)
        assert host(pk, got) == ref(O.pack_squeeze(opk, data, pack_num, shift))


@pytest.mark.parametrize("wide_max", [4096, 0])
def test_pack_squeeze_wide_and_stepwise(env, monkeypatch, wide_max):
    """pack_squeeze (lib.rs:439-450) on both device paths -- fphe_pack_squeeze, one chunk per
    wave (wide_dev.h: WIDE_SQUEEZE_MAX_CHUNKS = 4096), and the fphe_sqmul step launches (0) --
    on negative signed ciphertexts (the result takes the last multiplied y's sign, or x_0's in
    a one-element chunk), config 4's 13-way squeeze at 148 bits, shift 0 and 1."""
    monkeypatch.setattr(P, "WIDE_SQUEEZE_MAX_CHUNKS", wide_max)
    fx, sk, pk, coder, opk, cts = env
    data = more(opk, cts, 61, 7)
    for pack_num, shift in ((13, 148), (4, 1), (2, 0), (5, 37)):
        got = dev_vec(pk, data).pack_squeeze(pack_num, shift, pk)
        assert host(pk, got) == ref(O.pack_squeeze(opk, data, pack_num, shift)), (pack_num, shift)


def test_iupdate_and_masks(env):
    fx, sk, pk, coder, opk, cts = env
    rng = random.Random(7)
    stride = 2
    data = [O.ct_zero() for _ in range(10 * stride)]
    cts = more(opk, cts, 91)
    data[3] = cts[90]  # a non-zero slot that also receives contributions
    other = cts[:20 * stride]
    indexes = [[rng.randrange(10) for _ in range(rng.randrange(0, 4))] for _ in range(20)]
    v = dev_vec(pk, data)
    v.iupdate(dev_vec(pk, other), indexes, stride, pk)
    want = list(data)
    O.iupdate(opk, want, other, indexes, stride)
    assert host(pk, v) == ref(want)
    masks = [rng.random() < 0.5 for _ in range(20)]
    idx2 = [[rng.randrange(10)] for _ in range(sum(masks))]
    v2 = dev_vec(pk, data)
    v2.iupdate_with_masks(dev_vec(pk, other), idx2, masks, stride, pk)
    want2 = list(data)
    O.iupdate_with_masks(opk, want2, other, idx2, masks, stride)
    assert host(pk, v2) == ref(want2)


def test_iupdate_fresh_zeros_target_edges(env):
    """The zeros() target stays key-less until the fold hands it the key (_keyed leaves it so
    for iupdate / iupdate_with_masks): a panicking call, a call with no terms and a [samples,
    positions] tensor call must leave it exactly the reference's value, and a zeros() vector
    folded into itself reads literal-1 terms (lib.rs:301-308, 724-747)."""
    fx, sk, pk, coder, opk, cts = env
    stride = 2
    cts = more(opk, cts, 40, seed=3)
    other = cts[:12 * stride]
    v = P.CiphertextVector.zeros(6 * stride, pk._key.L2)
    with pytest.raises(P.PanicException):  # position 6 is past 12 / 2 slots
        v.iupdate(dev_vec(pk, other), [[0], [6]] + [[] for _ in range(10)], stride, pk)
    v.iupdate(dev_vec(pk, other), [[] for _ in range(12)], stride, pk)  # no terms at all
    want = [O.ct_zero() for _ in range(6 * stride)]
    assert host(pk, v) == ref(want)
    pos = torch.tensor([[(3 * i) % 6, (i + 1) % 6] for i in range(12)], dtype=torch.int64)
    v.iupdate(dev_vec(pk, other), pos.to(v.device), stride, pk)
    O.iupdate(opk, want, other, pos.tolist(), stride)
    assert host(pk, v) == ref(want)
    # the same positions as rectangular lists (one per sample: the tensor path) and as a numpy
    # matrix, into a zeros() target and into a vector that already holds sums
    for form in (pos.tolist(), pos.numpy()):
        w = P.CiphertextVector.zeros(6 * stride, pk._key.L2)
        w.iupdate(dev_vec(pk, other), form, stride, pk)
        w.iupdate(dev_vec(pk, other), form, stride, pk)
        w2 = [O.ct_zero() for _ in range(6 * stride)]
        O.iupdate(opk, w2, other, pos.tolist(), stride)
        O.iupdate(opk, w2, other, pos.tolist(), stride)
        assert host(pk, w) == ref(w2)
    # a zeros() vector as its own source: every term is the literal 1
    z = P.CiphertextVector.zeros(4 * stride, pk._key.L2)
    z.iupdate(z, [[1], [1, 3]], stride, pk)
    wz = [O.ct_zero() for _ in range(4 * stride)]
    O.iupdate(opk, wz, [O.ct_zero() for _ in range(4 * stride)], [[1], [1, 3]], stride)
    assert host(pk, z) == ref(wz)


def _fold_terms(opk, count, seed):
    """Terms for the segmented fold: long equal-exponent runs (> 64, several fphe_fold
    rounds), negative ciphertext integers (sign 1), other exponents, literal 1s with
    exponent 0 and -14 (the nude encryption of 0.0 is the integer 1, which add() treats as
    zero)."""
    rng = random.Random(seed)
    terms = []
    for i in range(count):
        exp = rng.choice([0, 0, 0, 0, -3, 2, -1])
        c = rng.randrange(2, opk.ns)  # any integer works for the fold's algebra (see more())
        terms.append(O.Ciphertext(-c if rng.random() < 0.5 else c, exp))  # signed, as encryptions of negatives
    terms[5] = O.fp_encrypt(opk, O.encode_f64(opk.n, 0.0), False)  # integer 1, exp -14
    terms[9] = O.ct_zero()
    return terms


def test_iupdate_long_segments(env):
    """iupdate with hundreds of terms per slot: exercises fphe_fold's multi-round chunking
    and the per-exponent merge against the reference's sequential fold."""
    fx, sk, pk, coder, opk, cts = env
    rng = random.Random(11)
    stride = 1
    other = _fold_terms(opk, 420, 3)
    data = [O.ct_zero() for _ in range(4)]
    data[2] = cts[7]
    indexes = [[0] if rng.random() < 0.8 else [rng.randrange(4)] for _ in range(len(other))]
    indexes[5] = [3]   # slot 3: only the exp -14 literal 1 (stays the literal 1 of exp 0)
    indexes[9] = [1]
    v = dev_vec(pk, data)
    v.iupdate(dev_vec(pk, other), indexes, stride, pk)
    want = list(data)
    O.iupdate(opk, want, other, indexes, stride)
    assert host(pk, v) == ref(want)


def test_align_many_gaps(env):
    """fphe_align (the per-exponent merge of the folds): c^(16^gap) mod n^2, canonical with
    sign 0 for gap > 0 (decrese_exp_to, lib.rs:250-258), the element unchanged for gap 0;
    gaps 0..31 mixed within waves, signed inputs, the literal 1, a ragged tail."""
    fx, sk, pk, coder, opk, cts = env
    rng = random.Random(21)
    terms = more(opk, cts, 131, seed=4)
    terms[7] = O.ct_zero()
    gaps = [rng.choice([0, 0, 1, 2, 3, 5, 9, 17, 31]) for _ in terms]
    got = P._align(pk, dev_vec(pk, terms), torch.tensor(gaps))
    want = []
    for t, g in zip(terms, gaps):
        if g == 0:
            want.append((t.c, t.exp))
        else:
            want.append((pow(t.c % opk.ns, 16 ** g, opk.ns), t.exp))
    assert host(pk, got) == want


def test_iupdate_wide_exponents(env):
    """Slots whose terms span exponents -40..4 (gaps up to 44, 176 squarings), with literal
    1s whose exponent is below every other term of their slot (a literal 1 is add's
    identity and must not set the slot's exponent), against the sequential fold."""
    fx, sk, pk, coder, opk, cts = env
    rng = random.Random(23)
    other = []
    for i in range(300):
        c = rng.randrange(2, opk.ns)
        other.append(O.Ciphertext(-c if rng.random() < 0.4 else c, rng.randrange(-40, 5)))
    for i in (3, 50, 77):
        other[i] = O.Ciphertext(1, -60)  # literal 1, lowest exponent of any term
    data = [O.ct_zero() for _ in range(6)]
    data[4] = cts[3]
    indexes = [[rng.randrange(6)] for _ in range(len(other))]
    indexes[3] = [5]
    indexes[50] = [5]  # slot 5: literal 1s and what else lands there
    v = dev_vec(pk, data)
    v.iupdate(dev_vec(pk, other), indexes, 1, pk)
    want = list(data)
    O.iupdate(opk, want, other, indexes, 1)
    assert host(pk, v) == ref(want)


def test_chunking_cumsum_with_step(env):
    fx, sk, pk, coder, opk, cts = env
    data = cts[:24]
    for sizes, step in (([4, 2, 6], 2), ([12, 12], 1), ([24], 3)):
        v = dev_vec(pk, data)
        v.chunking_cumsum_with_step(pk, sizes, step)
        want = list(data)
        O.chunking_cumsum_with_step(opk, want, sizes, step)
        assert host(pk, v) == ref(want)


def test_intervals_sum_with_step(env):
    fx, sk, pk, coder, opk, cts = env
    data = cts[:30]
    intervals, step = [(0, 7), (7, 7), (10, 30)], 3
    got = dev_vec(pk, data).intervals_sum_with_step(pk, intervals, step)
    assert host(pk, got) == ref(O.intervals_sum_with_step(opk, data, intervals, step))
    # many overlapping intervals (a histogram's node x feature ranges), and intervals_slice
    rng = random.Random(4)
    many = []
    for _ in range(300):
        a = rng.randrange(30)
        many.append((a, rng.randrange(a, 31)))
    got = dev_vec(pk, data).intervals_sum_with_step(pk, many, 2)
    assert host(pk, got) == ref(O.intervals_sum_with_step(opk, data, many, 2))
    got = dev_vec(pk, data).intervals_slice(many)
    assert host(pk, got) == ref([x for a, b in many for x in data[a:b]])
    # step 0: empty chunks (the reference's (0..0).cycle() adds nothing), the ranges still checked
    assert host(pk, dev_vec(pk, data).intervals_sum_with_step(pk, intervals, 0)) == []
    with pytest.raises(P.PanicException, match="slice index starts at 9 but ends at 8"):
        dev_vec(pk, data).intervals_sum_with_step(pk, [(0, 3), (9, 8), (0, 31)], 2)
    with pytest.raises(P.PanicException, match="range end index 31 out of range for slice of length 30"):
        dev_vec(pk, data).intervals_sum_with_step(pk, [(0, 3), (0, 31), (9, 8)], 0)


def test_matmul_rmatmul(env):
    fx, sk, pk, coder, opk, cts = env
    rng = random.Random(3)
    # a: 3x4 ciphertexts; b: 4x2 plaintexts with negative entries (invert branch)
    a = cts[:12]
    bs = [O.encode_f64(opk.n, rng.uniform(-3, 3)) for _ in range(8)]
    pv = P.PlaintextVector.from_ints([b.significant for b in bs], [b.exp for b in bs])
    got = dev_vec(pk, a).matmul(pk, pv, [3, 4], [4, 2])
    assert host(pk, got) == ref(O.matmul(opk, a, bs, [3, 4], [4, 2]))
    # rmatmul: self (lshape) 4x3 ciphertexts, other (rshape) 2x4 plaintexts
    got = dev_vec(pk, a).rmatmul(pk, pv, [4, 3], [2, 4])
    assert host(pk, got) == ref(O.rmatmul(opk, a, bs, [4, 3], [2, 4]))


def _self_op_ref(opk, data, sa, sb, size, sub):
    data = list(data)
    if sa == sb:
        end = len(data) if size is None else sa + size
        for k in range(sa, end):
            data[k] = O.ct_zero() if sub else O.ct_i_double(opk, data[k])
        return data
    w0, r0 = max(sa, sb), min(sa, sb)
    s = len(data) - w0 if size is None else size
    for k in range(s):  # iadd_i_j / isub_i_j (lib.rs:417-433)
        data[w0 + k] = (O.ct_sub if sub else O.ct_add)(opk, data[w0 + k], data[r0 + k])
    return data


def test_iadd_isub_vec_self(env):
    fx, sk, pk, coder, opk, cts = env
    data = cts[:20]
    for sa, sb, size in ((0, 3, 10), (5, 1, None), (4, 4, 6), (0, 10, 10)):
        for sub in (False, True):
            v = dev_vec(pk, data)
            (v.isub_vec_self if sub else v.iadd_vec_self)(sa, sb, size, pk)
            assert host(pk, v) == ref(_self_op_ref(opk, data, sa, sb, size, sub)), (sa, sb, size, sub)


def test_int_codec(env):
    """encode_i64 / decode_i64 / decode_i32 on the device vs the oracle (lib.rs:68-146)."""
    fx, sk, pk, coder, opk, cts = env
    vals = [0, 1, -1, 2**63 - 1, -2**63, 123456789012345, -987654321, 2**31, -2**31 - 5]
    pv = coder.encode_i64_vec(torch.tensor(vals, dtype=torch.int64).cuda())
    sig, exp = pv.to_ints()
    assert sig == [O.encode_i64(opk.n, v).significant % opk.n for v in vals] and exp == [0] * len(vals)
    assert coder.decode_i64_vec(pv) == [O.decode_i64(opk.n, s, 0) for s in sig]
    # decode with exponents (the floor shift for negative mantissas, and i64 wrap of i128)
    rng = random.Random(11)
    ms = [rng.randrange(-(1 << 80), 1 << 80) for _ in range(40)] + [-7, 7, -(1 << 100), 5, 1 << 100, -(1 << 127)]
    es = [rng.randrange(-8, 6) for _ in range(40)] + [-1, -1, -6, 30, 8, 0]
    sigs = [m % opk.n for m in ms]
    pv2 = P.PlaintextVector.from_ints(sigs, es)
    want = []
    for s_, e_ in zip(sigs, es):
        try:
            want.append(O.decode_i64(opk.n, s_, e_))
        except OverflowError:
            want.append(None)
    ok = [i for i, w in enumerate(want) if w is not None]
    pv_ok = P.PlaintextVector.from_ints([sigs[i] for i in ok], [es[i] for i in ok])
    assert coder.decode_i64_vec(pv_ok) == [want[i] for i in ok]
    bad = [i for i, w in enumerate(want) if w is None]
    assert bad, "expected at least one out-of-range case"
    with pytest.raises(P.PanicException):
        coder.decode_i64_vec(P.PlaintextVector.from_ints([sigs[bad[0]]], [es[bad[0]]]))
    # decode_i32: decode_f64 as i32 (saturating)
    want32 = []
    for s_, e_ in zip([sigs[i] for i in ok], [es[i] for i in ok]):
        f = O.decode_f64(opk.n, s_, e_)
        want32.append(0 if f != f else max(-2**31, min(2**31 - 1, int(f))) if abs(f) < 2**63 else
                      (2**31 - 1 if f > 0 else -2**31))
    assert coder.decode_i32_vec(pv_ok) == want32


def test_pack_unpack_floats(env):
    """pack_floats / unpack_floats on the device vs the oracle (lib.rs:79-118), SecureBoost
    shape: g+1 and h packed at precision 52 with offset 77 (guest.py:203-206)."""
    fx, sk, pk, coder, opk, cts = env
    rng = random.Random(4)
    vals = []
    for _ in range(37):
        g = rng.uniform(-1, 1)
        vals += [g + 1.0, rng.uniform(0, 0.25)]
    vals += [0.0, 2.0 ** -60, 1.5]  # ragged last chunk, a value that rounds to 0
    off, pn, prec = 77, 2, 52
    pv = coder.pack_floats(torch.tensor(vals, dtype=torch.float64).cuda(), off, pn, prec)
    sig, exp = pv.to_ints()
    want = O.pack_floats(vals, off, pn, prec)
    assert sig == [w.significant for w in want] and exp == [0] * len(want)
    got = coder.unpack_floats(pv, off, pn, prec, len(vals))
    assert got == O.unpack_floats(want, off, pn, prec, len(vals))
    # through encryption, ciphertext adds and pack_squeeze-free decryption
    ct = pk.encrypt_encoded(pv, True)
    back = coder.unpack_floats(sk.decrypt_to_encoded(ct), off, pn, prec, len(vals))
    assert back == O.unpack_floats(want, off, pn, prec, len(vals))


def test_neg_batch_inversion_full_grid(env):
    """c * neg(c) == 1 (mod n^2) for every element of a 600k-element vector: enough wave
    tiles that the batch-inversion kernels' grid-stride loops take several rounds (a
    size-independent property; the element-level oracle comparison is above)."""
    fx, sk, pk, coder, opk, cts = env
    n = 600_000 + 17
    g = torch.Generator().manual_seed(11)
    x = (torch.randn(n, generator=g) * 4).cuda()
    a = pk.encrypt_encoded(coder.encode_f32_vec(x), True)
    prod = P._add(pk, a, P._neg(pk, a), False)
    C = prod.C.transpose(1, 2).reshape(-1, prod.L2)[:n]  # tile-major [tiles][L2][64] -> rows
    assert bool((C == pk._key.mont_one(C.device)).all())  # M(1): the integer 1 in Montgomery form
    assert torch.equal(prod.exp[:n], a.exp[:n])


def test_empty_and_degenerate_vector_ops(env):
    """Empty and degenerate inputs through the vector algebra, against the oracle's loops on
    the same inputs (lib.rs:439-450, :724-791, :852-908): iupdate with no terms and with
    every sample's index list empty, a zero-size chunk and a step past its chunk in
    chunking_cumsum_with_step, empty intervals, pack_squeeze of nothing, matmul / rmatmul
    with a zero inner or outer dimension (the literal-1 zeros), decrypt of nothing."""
    fx, sk, pk, coder, opk, cts = env
    data = more(opk, cts, 12, 5)
    empty = dev_vec(pk, [])
    v = dev_vec(pk, data)
    v.iupdate(empty, [], 1, pk)
    assert host(pk, v) == ref(data)
    v.iupdate(dev_vec(pk, data[:6]), [[]] * 6, 2, pk)
    want = list(data)
    O.iupdate(opk, want, data[:6], [[]] * 6, 2)
    assert host(pk, v) == ref(want)
    for sizes, step in (([0, 5, 0, 7], 2), ([3, 9], 4), ([12], 12), ([], 1), ([10, 2, 1], 2), ([5, 7], 0)):
        v = dev_vec(pk, data)
        v.chunking_cumsum_with_step(pk, sizes, step)
        want = list(data)
        O.chunking_cumsum_with_step(opk, want, sizes, step)
        assert host(pk, v) == ref(want), (sizes, step)
    got = dev_vec(pk, data).intervals_sum_with_step(pk, [(4, 4), (0, 0)], 2)
    assert host(pk, got) == ref(O.intervals_sum_with_step(opk, data, [(4, 4), (0, 0)], 2))
    assert host(pk, empty.pack_squeeze(3, 20, pk)) == []
    pv0 = P.PlaintextVector.from_ints([], [])
    got = dev_vec(pk, []).matmul(pk, pv0, [3, 0], [0, 2])
    assert host(pk, got) == ref(O.matmul(opk, [], [], [3, 0], [0, 2]))
    bs = [O.encode_f64(opk.n, 1.5 - k) for k in range(8)]
    pv = P.PlaintextVector.from_ints([b.significant for b in bs], [b.exp for b in bs])
    assert host(pk, empty.matmul(pk, pv, [0, 4], [4, 2])) == []
    got = dev_vec(pk, []).rmatmul(pk, pv0, [0, 3], [2, 0])
    assert host(pk, got) == ref(O.rmatmul(opk, [], [], [0, 3], [2, 0]))
    assert sk.decrypt_to_encoded(empty).to_ints() == ([], [])


def test_iupdate_into_fresh_zeros(env):
    """iupdate / iupdate_with_masks into a zeros() histogram take the literal-1 fast path (the
    folded slots replace the literal 1s, add(1, x) = x, lib.rs:301-308); the result equals the
    reference's sequential loop from zeros, untouched slots keep the literal 1 with exp 0, and
    a second iupdate into the same (now non-zero) vector adds as usual."""
    fx, sk, pk, coder, opk, cts = env
    rng = random.Random(11)
    stride = 2
    cts = more(opk, cts, 60)
    other = cts[:20 * stride]
    other[5] = O.ct_zero()  # a literal-1 term
    indexes = [[rng.randrange(7) for _ in range(rng.randrange(0, 3))] for _ in range(20)]
    v = P.CiphertextVector.zeros(10 * stride, pk._key.L2)  # slots 7..9 get no terms
    v.iupdate(dev_vec(pk, other), indexes, stride, pk)
    want = [O.ct_zero() for _ in range(10 * stride)]
    O.iupdate(opk, want, other, indexes, stride)
    assert host(pk, v) == ref(want)
    v.iupdate(dev_vec(pk, other), indexes, stride, pk)  # no longer zeros: the ct-add path
    O.iupdate(opk, want, other, indexes, stride)
    assert host(pk, v) == ref(want)
    masks = [rng.random() < 0.6 for _ in range(20)]
    idx2 = [[rng.randrange(10)] for _ in range(sum(masks))]
    v2 = P.CiphertextVector.zeros(10 * stride, pk._key.L2)
    v2.iupdate_with_masks(dev_vec(pk, other), idx2, masks, stride, pk)
    want2 = [O.ct_zero() for _ in range(10 * stride)]
    O.iupdate_with_masks(opk, want2, other, idx2, masks, stride)
    assert host(pk, v2) == ref(want2)


def test_shuffles_and_index_slices(env):
    """i_shuffle / shuffle (lib.rs:473-497) against the oracle's cycle walk, for a permutation
    and for index lists that are not one (duplicates, a longer list), with the indexes as a
    list and as a tensor (the protocol's Shuffler hands over tensors); slice_indexes
    (lib.rs:457-463) with repeats and its index panic."""
    fx, sk, pk, coder, opk, cts = env
    rng = random.Random(21)
    data = cts[:40]
    perm = list(range(40))
    rng.shuffle(perm)
    dup = [rng.randrange(40) for _ in range(43)]
    for ix in (perm, dup):
        want = list(data)
        O.i_shuffle(want, ix)
        v = dev_vec(pk, data)
        got = v.shuffle(torch.tensor(ix))
        assert host(pk, got) == ref(want)
        assert host(pk, v) == ref(data)  # shuffle leaves its source alone
        v.i_shuffle(ix)
        assert host(pk, v) == ref(want)
    with pytest.raises(P.PanicException, match="index out of bounds"):
        dev_vec(pk, data).i_shuffle(perm[:30])
    sel = [3, 3, 0, 39, 17]
    assert host(pk, dev_vec(pk, data).slice_indexes(sel)) == ref([data[i] for i in sel])
    with pytest.raises(P.PanicException, match="the len is 40 but the index is 40"):
        dev_vec(pk, data).slice_indexes([1, 40, 41])
