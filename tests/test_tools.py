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
    """fate_amd/csrc/mont27_*_gen.h are exactly what tools/gen_mont27_asm.py writes."""
    with tempfile.TemporaryDirectory() as d:
        shutil.copytree(os.path.join(ROOT, "tools"), os.path.join(d, "tools"))
        os.makedirs(os.path.join(d, "fate_amd", "csrc"))
        subprocess.run([sys.executable, os.path.join(d, "tools", "gen_mont27_asm.py")], check=True)
        for name in ("mont27_asm_gen.h", "mont27_sq_gen.h", "mont27_fused_gen.h"):
            assert filecmp.cmp(os.path.join(d, "fate_amd", "csrc", name),
                               os.path.join(ROOT, "fate_amd", "csrc", name), shallow=False), name
