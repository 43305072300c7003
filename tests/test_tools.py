"""CPU checks of the measurement and code-generation tooling: bench.py's sliding-window
schedule (the mad counts behind roofline.issue) against a direct simulation of the
kernel's window walk, and the generated asm headers against their generator."""
import filecmp
import os
import shutil
import subprocess
import sys
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _walk(e: int, w: int):
    """powm27's schedule (fate_amd/csrc/kernels27.h): table build = X^2 (general) + 2^(w-1)-1
    odd powers; then from the top, each window [j, i] with bit j set: (i-j+1) squarings and
    one product, zero bits one squaring each (the first window costs no squarings)."""
    sq, mul = 0, 1 + (1 << (w - 1)) - 1
    i = e.bit_length() - 1
    first = True
    while i >= 0:
        if not (e >> i) & 1:
            sq += 1
            i -= 1
            continue
        j = max(i - w + 1, 0)
        while not (e >> j) & 1:
            j += 1
        if first:
            first = False
        else:
            sq += i - j + 1
            mul += 1
        i = j - 1
    return sq, mul


@pytest.mark.parametrize("seed", range(5))
def test_sliding_window_schedule_matches_walk(seed):
    sys.path.insert(0, ROOT)
    import random

    import bench
    rng = random.Random(seed)
    for bits in (17, 1024, 2048):
        e = rng.getrandbits(bits) | (1 << (bits - 1)) | 1
        for w in (4, 5, 6):
            assert bench.sliding_window_schedule(e, w) == _walk(e, w)
    # exponent with a long zero run and a lone top bit
    e = (1 << 2047) | 1
    assert bench.sliding_window_schedule(e, 6) == _walk(e, 6)


def test_generated_asm_headers_in_sync():
    """fate_amd/csrc/mont_gen_ll{38,37}.h are exactly what tools/gen_mont27_asm.py writes."""
    with tempfile.TemporaryDirectory() as d:
        shutil.copytree(os.path.join(ROOT, "tools"), os.path.join(d, "tools"))
        os.makedirs(os.path.join(d, "fate_amd", "csrc"))
        subprocess.run([sys.executable, os.path.join(d, "tools", "gen_mont27_asm.py")], check=True)
        for name in ("mont_gen_ll38.h", "mont_gen_ll37.h"):
            assert filecmp.cmp(os.path.join(d, "fate_amd", "csrc", name),
                               os.path.join(ROOT, "fate_amd", "csrc", name), shallow=False), name


@pytest.mark.parametrize("tpi,ll", [(4, 38), (2, 38), (1, 38), (8, 37), (4, 37), (2, 37), (1, 37)])
def test_squaring_window_adds_every_limb_pair_once(tpi, ll):
    """The half-product squaring (mont_engine.inc mont_sqr, rows from the generator's
    sq_window) adds each off-diagonal limb pair exactly twice (once, doubled) and each
    diagonal term once, for the 27 x 38 (TPI 4) and 28 x 37 (TPI 1, 2, 4, 8) engines.  Multiplier
    rules as the kernel's bit-field masks: bf = 2a (q > s), a (q == s), 0 (q < s); bl (even
    LL only) = 2a if q < s or (q == s and a < LL/2), else 0; bm = 2a."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("gen27", os.path.join(ROOT, "tools", "gen_mont27_asm.py"))
    gen = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(gen)
    from collections import Counter
    cov = Counter()
    nl = tpi * ll
    for s in range(tpi):
        for a in range(ll):
            i = ll * s + a
            for q in range(tpi):
                for k, mul in gen.sq_window(ll, a):
                    g = ll * q + k
                    if mul == "bf":
                        f = 2 if q > s else (1 if q == s else 0)
                    elif mul == "bl":
                        f = 2 if (q < s or (q == s and a < ll // 2)) else 0
                    else:
                        f = 2
                    if f:
                        cov[(min(i, g), max(i, g))] += f
    assert set(cov) == {(x, y) for x in range(nl) for y in range(x, nl)}
    assert all(c == (1 if x == y else 2) for (x, y), c in cov.items())
