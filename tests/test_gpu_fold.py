"""The device-grouped segmented fold (fphe_fold_segments, fate_amd.paillier._fold_to_segments):
the engine under iupdate / iupdate_with_masks / intervals_sum_with_step / matmul and the
cross-rank histogram fold.  Bit-exact against the oracle's sequential Ciphertext::add folds
(fixedpoint_paillier/src/lib.rs:301-333, 724-791) and against the torch grouping it replaces,
on: wide and outlier exponents (alignment by up to tens of base-16 steps), negative signed
ciphertexts, literal-1 terms (all-literal segments end on their last term's exponent), empty
segments, several fold levels (runs longer than 64 x 64 terms), the fallback when the
(segment, exponent) key space is too large, and out-of-range indexes (the reference panics)."""
import random

import pytest
import torch

from fate_amd import paillier as P
from oracle import paillier_oracle as O

from test_gpu_ops import dev_vec, host, load, more  # noqa: E402

import numpy as np  # noqa: E402

from oracle import gmp_ref  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(params=[1024, 2048], scope="module")
def env(request):
    return load(request.param)


def oracle_fold(opk, src, idx, seg, nseg):
    out = [O.ct_zero() for _ in range(nseg)]
    for i, s in zip(idx, seg):
        out[s] = O.ct_add(opk, out[s], src[i])
    return [(c.c, c.exp) for c in out]


def gmp_spot_check(pk, src, idx, seg, got, segs):
    """libgmp's sequential fold (oracle/gmp_ref.c gref_fold: the reference's add_assign loop,
    term order kept) of the segments `segs`, against the device's result `got` (host pairs):
    the large folds' slot plans are pinned to libgmp, not only to another device mode."""
    L = pk._key.L2
    segs = sorted(segs)
    sv = gmp_ref.to_vec([c.c for c in src], [c.exp for c in src], L)
    idx_np = np.asarray(idx.cpu() if isinstance(idx, torch.Tensor) else idx, dtype=np.int64)
    seg_np = np.asarray(seg.cpu() if isinstance(seg, torch.Tensor) else seg, dtype=np.int64)
    keep = np.isin(seg_np, segs)
    slots = np.searchsorted(np.array(segs), seg_np[keep])
    want = gmp_ref.from_vec(gmp_ref.GmpKey(pk.n).fold(sv, idx_np[keep], slots,
                                                       gmp_ref.to_vec([1] * len(segs), [0] * len(segs), L),
                                                       threads=len(segs)))
    assert [got[s] for s in segs] == list(zip(*want))


def mixed_sources(opk, cts, k, seed):
    """k signed ciphertexts: random integers with exponents spread over -40..18 (the bench's
    outliers), a sprinkling of literal 1s with their own exponents."""
    rng = random.Random(seed)
    src = more(opk, cts, k, seed)
    out = []
    for c in src:
        r = rng.random()
        if r < 0.06:
            out.append(O.Ciphertext(1, rng.choice([0, -14, -3, 5])))  # the reference's zero
        elif r < 0.10:
            out.append(O.Ciphertext(c.c, rng.choice([-40, -38, 18, 17])))
        else:
            out.append(O.Ciphertext(c.c, rng.choice([-14, -13, -13, -12, -15, -16])))
    return out


def test_fold_segments_vs_oracle(env):
    fx, sk, pk, coder, opk, cts = env
    rng = random.Random(5)
    src = mixed_sources(opk, cts, 160, 5)
    nseg = 23
    T = 700
    idx = [rng.randrange(len(src)) for _ in range(T)]
    seg = [rng.randrange(nseg - 3) for _ in range(T)]  # the last 3 segments stay empty
    # an all-literal segment: its fold is 1 with the exponent of its last term
    lits = [i for i, c in enumerate(src) if c.c == 1]
    for k, i in enumerate(lits[:4]):
        idx.append(i)
        seg.append(nseg - 4)
    got = P._fold_to_segments(pk, dev_vec(pk, src), torch.tensor(seg), nseg, index=torch.tensor(idx))
    assert host(pk, got) == oracle_fold(opk, src, idx, seg, nseg)


def test_fold_segments_many_levels_and_torch_grouping(env):
    """Runs of ~9K terms (three fold levels) on few segments, against the torch grouping."""
    fx, sk, pk, coder, opk, cts = env
    src = mixed_sources(opk, cts, 300, 9)
    v = dev_vec(pk, src)
    g = torch.Generator().manual_seed(3)
    T = 40000
    idx = torch.randint(0, len(src), (T,), generator=g)
    seg = torch.randint(0, 5, (T,), generator=g)
    got = P._fold_to_segments(pk, v, seg, 6, index=idx)
    res, ids = P._fold_segments(pk, v, seg, index=idx)
    want = P._literal_ones(pk, 6, v.device)
    res.n = pk.n
    want._assign(ids, res)
    assert host(pk, got) == host(pk, want)
    # and segment 0 against the oracle (a strided subset of its terms keeps this quick)
    sel = torch.nonzero(seg == 0).squeeze(1)[::17]
    got0 = P._fold_to_segments(pk, v, torch.zeros(sel.numel(), dtype=torch.long), 1, index=idx[sel])
    assert host(pk, got0) == oracle_fold(opk, src, idx[sel].tolist(), [0] * sel.numel(), 1)


def test_fold_segments_identity_index_and_fallback(env):
    """index=None (term t is element t: the cross-rank fold), and a key space beyond the
    device grouping's 2^25 buckets (exponents far apart in different segments) that takes the
    torch grouping instead -- same integers."""
    fx, sk, pk, coder, opk, cts = env
    src = mixed_sources(opk, cts, 200, 11)
    m = 40
    seg = [t % m for t in range(len(src))]
    got = P._fold_to_segments(pk, dev_vec(pk, src), torch.tensor(seg), m)
    assert host(pk, got) == oracle_fold(opk, src, list(range(len(src))), seg, m)
    far = [O.Ciphertext(c.c, (-30000 if i % 2 else 30000) + (i % 3)) for i, c in enumerate(src)]
    segf = [i % 2 + 2 * (i % 700) for i in range(len(far))]  # 1400 segments x 60003 exponents
    got = P._fold_to_segments(pk, dev_vec(pk, far), torch.tensor(segf), 1400)
    assert host(pk, got) == oracle_fold(opk, far, list(range(len(far))), segf, 1400)


def test_fold_segments_large_key_space(env):
    """(segment, exponent) key spaces past the per-block LDS counters (16384 keys: the global
    counter-copy path of the counting sort) and just inside them, against the oracle."""
    fx, sk, pk, coder, opk, cts = env
    src = mixed_sources(opk, cts, 200, 13)  # exponents -40 .. 18: 59 per segment
    rng = random.Random(13)
    for nseg in (270, 300):  # 15,930 and 17,700 keys
        T = 900
        idx = [rng.randrange(len(src)) for _ in range(T)]
        seg = [rng.randrange(nseg) for _ in range(T)]
        got = P._fold_to_segments(pk, dev_vec(pk, src), torch.tensor(seg), nseg, index=torch.tensor(idx))
        assert host(pk, got) == oracle_fold(opk, src, idx, seg, nseg)


def test_fold_segments_bad_index_panics(env):
    fx, sk, pk, coder, opk, cts = env
    v = dev_vec(pk, more(opk, cts, 10))
    with pytest.raises(P.PanicException):
        P._fold_to_segments(pk, v, torch.tensor([0, 1]), 2, index=torch.tensor([0, v.count]))
    with pytest.raises(P.PanicException):
        P._fold_to_segments(pk, v, torch.tensor([0, 1]), 2, index=torch.tensor([-1, 0]))
    with pytest.raises(P.PanicException):
        P._fold_to_segments(pk, v, torch.tensor([0, 2]), 2, index=torch.tensor([0, 1]))
    hist = P.CiphertextVector.zeros(4, pk._key.L2)
    with pytest.raises(P.PanicException):
        hist.iupdate(v, [[0], [4]], 1, pk)  # a position past the histogram
    with pytest.raises(P.PanicException):
        hist.iupdate(v, [[0]] * (v.count + 1), 1, pk)  # more samples than the source holds


def test_iupdate_tensor_positions_device(env):
    """iupdate with a [samples, positions] tensor (expanded on the device) and with masks, from
    a non-empty histogram, against the oracle."""
    fx, sk, pk, coder, opk, cts = env
    rng = random.Random(8)
    src = mixed_sources(opk, cts, 120, 8)  # 60 samples x stride 2
    data = mixed_sources(opk, cts, 24, 81)  # 12 bins x stride 2
    pos = torch.tensor([[rng.randrange(12) for _ in range(3)] for _ in range(60)])
    hist = dev_vec(pk, data)
    hist.iupdate(dev_vec(pk, src), pos, 2, pk)
    od = list(data)
    O.iupdate(opk, od, src, pos.tolist(), 2)
    assert host(pk, hist) == [(c.c, c.exp) for c in od]
    masks = [rng.random() < 0.6 for _ in range(60)]
    k = sum(masks)
    hist2 = dev_vec(pk, data)
    hist2.iupdate_with_masks(dev_vec(pk, src), pos[:k].tolist(), masks, 2, pk)
    od2 = list(data)
    O.iupdate_with_masks(opk, od2, src, pos[:k].tolist(), masks, 2)
    assert host(pk, hist2) == [(c.c, c.exp) for c in od2]


def test_fold_chunked_past_term_limit(env, monkeypatch):
    """More terms than fphe_fold_segments' int32 count: the fold runs in chunks added onto the
    running result (literal-1 segments, segments a chunk misses, and segments only a later chunk
    reaches included).  The limit is lowered to 97 terms so the split is exercised at test size."""
    fx, sk, pk, coder, opk, cts = env
    rng = random.Random(17)
    src = mixed_sources(opk, cts, 150, 17)
    nseg = 19
    T = 500
    idx = [rng.randrange(len(src)) for _ in range(T)]
    seg = [rng.randrange(nseg - 4) for _ in range(T)]
    lits = [i for i, c in enumerate(src) if c.c == 1]
    idx += lits[:3]
    seg += [nseg - 3] * len(lits[:3])  # only the last chunk reaches this all-literal segment
    want = oracle_fold(opk, src, idx, seg, nseg)
    monkeypatch.setattr(P, "FOLD_MAX_TERMS", 97)
    got, present = P._fold_to_segments(pk, dev_vec(pk, src), torch.tensor(seg), nseg, index=torch.tensor(idx),
                                       with_present=True)
    assert host(pk, got) == want
    assert present[:nseg].tolist() == [int(s in set(seg)) for s in range(nseg)]
    hist = dev_vec(pk, mixed_sources(opk, cts, 2 * nseg, 171))
    od = [O.Ciphertext(c[0], c[1]) for c in host(pk, hist)]
    pos = [[rng.randrange(nseg) for _ in range(4)] for _ in range(60)]
    hist.iupdate(dev_vec(pk, src[:120]), pos, 2, pk)
    O.iupdate(opk, od, src[:120], pos, 2)
    assert host(pk, hist) == [(c.c, c.exp) for c in od]


def test_iupdate_position_range_checked_before_narrowing(env):
    """Positions are usize in the reference: one past the histogram panics, and so does one that
    would wrap onto a valid slot if narrowed to int32 first (2^32 + 1 -> 1)."""
    fx, sk, pk, coder, opk, cts = env
    v = dev_vec(pk, more(opk, cts, 4))
    hist = P.CiphertextVector.zeros(4, pk._key.L2)
    for bad in ([[0], [(1 << 32) + 1]], torch.tensor([[0], [(1 << 32) + 1]]), torch.tensor([[0], [-1]]),
                torch.tensor([[0], [4]], dtype=torch.int32), torch.tensor([[0], [-1]], dtype=torch.int32)):
        with pytest.raises(P.PanicException):
            hist.iupdate(v, bad, 1, pk)
    # stride 3 over 4 slots: position 1 reaches slots 3, 4, 5 -- past the end, as the reference's
    # index panic (fphe_positions_terms: positions below count / stride only)
    with pytest.raises(P.PanicException):
        hist.iupdate(v, torch.tensor([[1]], dtype=torch.int32), 3, pk)
    # a valid uint8 position matrix takes the same path (widened) and equals the list form
    a, b = P.CiphertextVector.zeros(4, pk._key.L2), P.CiphertextVector.zeros(4, pk._key.L2)
    a.iupdate(v, torch.tensor([[3, 0], [1, 1]], dtype=torch.uint8), 1, pk)
    b.iupdate(v, [[3, 0], [1, 1]], 1, pk)
    assert host(pk, a) == host(pk, b)


def test_fold_raised_keys_forced(env, monkeypatch):
    """FPHE_FOLD_RAISE=force: every key above its segment's least exponent gets its own slots
    and k_segfold27 raises its partial in place (the slot plan of k_gr_plan), against the
    oracle -- wide exponents, literal 1s (a segment whose least key holds only literals makes
    the device report it, and the call folds without the device merge), empty segments."""
    fx, sk, pk, coder, opk, cts = env
    rng = random.Random(23)
    src = mixed_sources(opk, cts, 160, 23)
    nseg = 17
    T = 900
    idx = [rng.randrange(len(src)) for _ in range(T)]
    seg = [rng.randrange(nseg - 2) for _ in range(T)]
    lits = [i for i, c in enumerate(src) if c.c == 1]
    low = min(range(len(src)), key=lambda i: src[i].exp if src[i].c != 1 else 99)
    idx += [lits[0], lits[1], low]  # segment nseg-2: a literal below a real term far above it
    seg += [nseg - 2] * 3
    want = oracle_fold(opk, src, idx, seg, nseg)
    monkeypatch.setenv("FPHE_FOLD_RAISE", "force")
    got = P._fold_to_segments(pk, dev_vec(pk, src), torch.tensor(seg), nseg, index=torch.tensor(idx))
    assert host(pk, got) == want


@pytest.mark.parametrize("bits", [2048])
def test_fold_raised_keys_auto_matches_merge(bits, monkeypatch):
    """The automatic choice at 2.1M terms, outliers 9 and 10 exponents above and below the
    bulk of their segments (k_gr_gapchoose weighs raising each segment's bulk against the
    merge's chain) returns the same integers as the plain exponent merge (FPHE_FOLD_RAISE=0)."""
    fx, sk, pk, coder, opk, cts = load(bits)
    base = more(opk, cts, 512, 31)
    rng = random.Random(31)
    exps = [-13] * 512
    for i in range(0, 512, 37):
        exps[i] = -13 + rng.choice([9, 10, -9, -10])
    src = [O.Ciphertext(c.c, e) for c, e in zip(base, exps)]
    v = dev_vec(pk, src)
    g = torch.Generator().manual_seed(31)
    T = 2_100_000
    idx = torch.randint(0, 512, (T,), generator=g)
    seg = torch.randint(0, 64, (T,), generator=g)
    got = host(pk, P._fold_to_segments(pk, v, seg, 64, index=idx))
    monkeypatch.setenv("FPHE_FOLD_RAISE", "0")
    want = host(pk, P._fold_to_segments(pk, v, seg, 64, index=idx))
    assert got == want
    # and against libgmp: six segments of ~33k terms, each with outliers below its bulk (every
    # later term pays decrese_exp_to's powm there: ~0.4 ms per term on one core)
    gmp_spot_check(pk, src, idx, seg, got, [0, 9, 22, 40, 51, 63])


def test_fold_raised_keys_past_the_cap(env, monkeypatch):
    """More keys to raise than the plan takes (kRaiseMax = 512): 600 segments each with a term
    8 exponents above its least one.  The keys past the cap stay in the exponent merge; every
    segment is still the reference's fold."""
    fx, sk, pk, coder, opk, cts = env
    base = more(opk, cts, 40, 41)
    rng = random.Random(41)
    nseg = 600
    src, seg = [], []
    for s_ in range(nseg):
        for e in (-13, -5, -13):
            src.append(O.Ciphertext(base[rng.randrange(len(base))].c, e))
            seg.append(s_)
    idx = list(range(len(src)))
    want = oracle_fold(opk, src, idx, seg, nseg)
    monkeypatch.setenv("FPHE_FOLD_RAISE", "force")
    got = P._fold_to_segments(pk, dev_vec(pk, src), torch.tensor(seg), nseg)
    assert host(pk, got) == want


def test_fold_raised_keys_multi_round_plan(monkeypatch):
    """A fold longer than one round of balanced slots at the largest slot length (36M terms
    against 32,768 slots x 1,024 items at 2048 bits), with outlier keys 9-12 exponents away:
    the plain merge, the automatic raise and the forced raise give the same integers."""
    fx, sk, pk, coder, opk, cts = load(2048)
    base = more(opk, cts, 256, 43)
    exps = [-13] * 256
    for i in range(0, 256, 29):
        exps[i] = -13 + (9 if i % 2 else -12)
    v = dev_vec(pk, [O.Ciphertext(c.c, e) for c, e in zip(base, exps)])
    g = torch.Generator().manual_seed(43)
    T = 36_000_000
    idx = torch.randint(0, 256, (T,), generator=g, dtype=torch.int32).cuda()
    seg = torch.randint(0, 500, (T,), generator=g, dtype=torch.int32).cuda()  # 500 x 22 keys: LDS counts
    outs = []
    for mode in ("0", None, "force"):
        if mode is None:
            monkeypatch.delenv("FPHE_FOLD_RAISE", raising=False)
        else:
            monkeypatch.setenv("FPHE_FOLD_RAISE", mode)
        r = P._fold_to_segments(pk, v, seg, 500, index=idx)
        outs.append((r.C[: (500 + 63) // 64].clone(), r.sign[:500].clone(), r.exp[:500].clone()))
        if mode is None:
            auto = host(pk, r)
    for o in outs[1:]:
        assert all(torch.equal(a, b) for a, b in zip(outs[0], o))
    # two segments of ~72k terms against libgmp (~30 s: most terms need an exponent alignment)
    src = [O.Ciphertext(c.c, e) for c, e in zip(base, exps)]
    gmp_spot_check(pk, src, idx, seg, auto, [7, 311])
