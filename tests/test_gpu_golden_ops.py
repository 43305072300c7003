"""GPU parity of the vector algebra against the committed ops fixtures
(tests/golden/paillier_{bits}_ops.json, made by tests/golden/make_fixtures.py from the oracle,
whose values tests/test_oracle.py re-derives with libgmp): neg / sub / rsub, ct x pt on every
branch of Ciphertext::mul, matmul / rmatmul, iupdate and pack_squeeze, bit-exact on signed
ciphertext integers and exponents (fixedpoint_paillier/src/lib.rs:259-285, 334-349, 439-450,
724-735, 852-908)."""
import json
import os

import pytest

from fate_amd import paillier as P

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(params=[1024, 2048], scope="module")
def env(request):
    bits = request.param
    with open(os.path.join(HERE, "golden", f"paillier_{bits}.json")) as f:
        base = json.load(f)
    with open(os.path.join(HERE, "golden", f"paillier_{bits}_ops.json")) as f:
        ops = json.load(f)
    sk, pk, coder = P.keypair_from_primes(int(base["p"], 16), int(base["q"], 16))
    return ops, pk


def vec(pk, pairs):
    return P.CiphertextVector.from_signed_ints([int(c, 16) for c, _ in pairs], [e for _, e in pairs], pk.ns,
                                               pk._key.L2)


def pts(pairs):
    return P.PlaintextVector.from_ints([int(s, 16) for s, _ in pairs], [e for _, e in pairs])


def js(pk, v):
    cs, es = v.to_signed_ints(pk.ns)
    return [[hex(c), e] for c, e in zip(cs, es)]


def test_neg(env):
    ops, pk = env
    assert js(pk, vec(pk, ops["neg"]["a"]).neg(pk)) == ops["neg"]["out"]


def test_sub_rsub(env):
    ops, pk = env
    s = ops["sub"]
    a, b = vec(pk, s["a"]), vec(pk, s["b"])
    assert js(pk, a.sub(pk, b)) == s["out"]
    assert js(pk, a.rsub(pk, b)) == s["rsub"]


def test_mul_every_branch(env):
    ops, pk = env
    m = ops["mul"]
    assert js(pk, vec(pk, m["c"]).mul(pk, pts(m["p"]))) == m["out"]


def test_matmul_rmatmul(env):
    ops, pk = env
    for name in ("matmul", "rmatmul"):
        t = ops[name]
        got = getattr(vec(pk, t["a"]), name)(pk, pts(t["b"]), t["lshape"], t["rshape"])
        assert js(pk, got) == t["out"], name


def test_iupdate(env):
    ops, pk = env
    t = ops["iupdate"]
    v = vec(pk, t["data"])
    v.iupdate(vec(pk, t["other"]), t["indexes"], t["stride"], pk)
    assert js(pk, v) == t["out"]


def test_pack_squeeze(env, kernel_path):
    ops, pk = env
    t = ops["pack_squeeze"]
    assert js(pk, vec(pk, t["data"]).pack_squeeze(t["pack_num"], t["shift_bit"], pk)) == t["out"]
