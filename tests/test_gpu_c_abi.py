"""GPU parity through a native C consumer of the boundary (tests/c_abi/abi_roundtrip.c,
linked against libfatephe.so alone): injected-r encryption of the golden fixture's encoded
significands, the exported signed ciphertext integers and the CRT decryption, bit-exact
against the oracle's values in the fixture (paillier/src/lib.rs:104-121, 163-176)."""
import json
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
BIN = os.path.join(HERE, "c_abi", "abi_roundtrip")


@pytest.mark.parametrize("mode", ["latency", "throughput"])
@pytest.mark.parametrize("bits", [1024, 2048])
def test_c_program_matches_fixture(bits, mode):
    if not os.path.exists(BIN):
        raise RuntimeError("tests/c_abi/abi_roundtrip is not built (__graft_entry__.build())")
    with open(os.path.join(HERE, "golden", f"paillier_{bits}.json")) as f:
        fx = json.load(f)
    e = fx["encrypt"]
    n = int(fx["p"], 16) * int(fx["q"], 16)
    lines = [str(fx["bits"]), hex(n), fx["p"], fx["q"], str(len(e["sig"]))]
    lines += [f"{s} {r}" for s, r in zip(e["sig"], e["r"])]
    out = subprocess.run([BIN, mode], input="\n".join(lines) + "\n", capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    rows = [ln.split() for ln in out.stdout.strip().splitlines()]
    assert [int(c, 16) for c, _ in rows] == [int(c, 16) for c in e["ct"]]
    assert [int(d, 16) for _, d in rows] == [int(d, 16) for d in e["dec"]]


@pytest.mark.parametrize("mode", ["latency", "throughput"])
def test_c_program_4096_vs_gmp(mode):
    """The same native consumer on a 4096-bit key (the TPI-8 geometry, L2 = 256): injected-r
    encryptions of 64 encoded floats checked against libgmp (oracle/gmp_ref.c, the mpz_* call
    sequence of paillier/src/lib.rs:104-121) and the CRT decryptions against the significands."""
    import random
    from oracle import gmp_ref
    from oracle import paillier_oracle as O
    if not os.path.exists(BIN):
        raise RuntimeError("tests/c_abi/abi_roundtrip is not built (__graft_entry__.build())")
    with open(os.path.join(HERE, "golden", "key_4096.json")) as f:
        k = json.load(f)
    p, q = int(k["p"], 16), int(k["q"], 16)
    n = p * q
    rng = random.Random(4096)
    sigs = [O.encode_f64(n, rng.uniform(-1e6, 1e6)).significant for _ in range(64)]
    rs = [1 + rng.randrange(n - 1) for _ in sigs]
    lines = ["4096", hex(n), format(p, "x"), format(q, "x"), str(len(sigs))]
    lines += [f"{format(s, 'x')} {format(r, 'x')}" for s, r in zip(sigs, rs)]
    out = subprocess.run([BIN, mode], input="\n".join(lines) + "\n", capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    rows = [ln.split() for ln in out.stdout.strip().splitlines()]
    gk = gmp_ref.GmpKey(n, p, q)
    assert [int(c, 16) for c, _ in rows] == [gk.encrypt(s, r, True) for s, r in zip(sigs, rs)]
    assert [int(d, 16) for _, d in rows] == [s % n for s in sigs]
