"""Wire format of the reference's pickles (fate_amd/wire.py; bincode(serde) of
fate_utils.paillier objects, paillier.rs:67-74,91-98,128-135,219-226,395-402).  The rug
Integer record layout is unpinned (no rug / bincode in this image): these tests pin the
layout as documented in include/fate_phe.h (8) -- rug's serde radix rule included: decimal
up to 32 significant bits, lowercase hex above -- and check device encode/decode against a
record-by-record construction written here from the spec, plus round trips."""
import json
import os
import struct

import numpy as np
import pytest
import torch

from fate_amd import _lib, wire
from fate_amd import paillier as P

HERE = os.path.dirname(os.path.abspath(__file__))


def fixture(bits):
    with open(os.path.join(HERE, "golden", f"paillier_{bits}.json")) as f:
        return json.load(f)


def rec(v, radix=None):
    """One rug Integer record built from the spec: i32 radix, u64 len, sign + digits; the
    radix rug's serde picks unless one is given."""
    if radix is None:
        radix = 10 if abs(v).bit_length() <= 32 else 16
    digs = "0123456789abcdefghijklmnopqrstuvwxyz"
    m, out = abs(v), ""
    while True:
        m, d = divmod(m, radix)
        out = digs[d] + out
        if m == 0:
            break
    s = ("-" if v < 0 else "") + out
    return struct.pack("<i", radix) + struct.pack("<Q", len(s)) + s.encode()


def ct_vec_bytes(cs, es, radix=None):
    return struct.pack("<Q", len(cs)) + b"".join(rec(c, radix) + struct.pack("<i", e) for c, e in zip(cs, es))


def test_bint_records():
    assert wire.bint(0) == struct.pack("<iQ", 10, 1) + b"0"
    assert wire.bint(-255) == struct.pack("<iQ", 10, 4) + b"-255"
    assert wire.bint(2**32 - 1) == struct.pack("<iQ", 10, 10) + b"4294967295"  # 32 bits: decimal
    assert wire.bint(2**32) == struct.pack("<iQ", 16, 9) + b"100000000"        # 33 bits: hex
    assert wire.bint(-(2**40)) == struct.pack("<iQ", 16, 12) + b"-10000000000"
    for v in (1, -1, 2**64, -(2**4095 + 12345), 0xDEADBEEF, 2**31, -(2**32) + 1):
        assert wire.bint(v) == rec(v)
        assert wire.Reader(rec(v)).bint() == v
        assert wire.Reader(rec(v, 10)).bint() == v  # any radix reads back
        assert wire.Reader(rec(v, 36)).bint() == v
    with pytest.raises(ValueError):
        wire.Reader(rec(5)[:-1]).bint()
    with pytest.raises(ValueError):
        wire.Reader(struct.pack("<iQ", 40, 1) + b"1").bint()
    for bad in (b"--5", b"1_0", b" 7", b"+7", b"", b"-", b"12a"):  # int() would take some of these
        with pytest.raises(ValueError):
            wire.Reader(struct.pack("<iQ", 10, len(bad)) + bad).bint()


def test_untrusted_counts_rejected_before_allocation():
    """A vector header claiming more elements than the bytes can hold is a ValueError, not
    an allocation sized by the untrusted count."""
    with pytest.raises(ValueError):
        wire.plaintext_vector_from_bincode(struct.pack("<Q", 2**60) + b"x" * 40)


def test_key_and_coder_records():
    fx = fixture(1024)
    p, q = int(fx["p"], 16), int(fx["q"], 16)
    n = p * q
    sk, pk, coder = P.keypair_from_primes(p, q)
    b = wire.pk_to_bincode(pk)
    assert b == rec(n) + rec(n * n) + rec(n // 2)
    assert wire.pk_from_bincode(b).n == n
    lo, hi = min(p, q), max(p, q)
    g = n + 1
    hp = pow((pow(g, lo - 1, lo * lo) - 1) // lo, -1, lo)
    hq = pow((pow(g, hi - 1, hi * hi) - 1) // hi, -1, hi)
    want = [lo, hi, n, lo - 1, hi - 1, lo * lo, hi * hi, pow(lo, -1, hi), hp, hq]
    b = wire.sk_to_bincode(sk)
    assert b == b"".join(rec(v) for v in want)
    back = wire.sk_from_bincode(b)
    assert (back.p, back.q) == (lo, hi)
    assert wire.coder_to_bincode(n) == rec(n) + rec(n // 2)
    assert wire.coder_from_bincode(wire.coder_to_bincode(n)) == n
    with pytest.raises(ValueError):
        wire.pk_from_bincode(rec(n) + rec(n * n + 1) + rec(n // 2))


def test_scan_walks_records():
    """fphe_wire_scan (host code in the C ABI library): offsets, signs, exps, radixes."""
    lib = _lib.load()
    cs, es = [0, -5, 2**100 + 7, 255], [-14, 3, 0, -2**31]
    buf = ct_vec_bytes(cs[:2], es[:2], radix=16) + ct_vec_bytes(cs[2:], es[2:], radix=10)[8:]
    raw = np.frombuffer(buf, dtype=np.uint8)
    n = len(cs)
    off, ln = np.empty(n, np.int64), np.empty(n, np.int32)
    neg, ex, rdx = np.empty(n, np.uint8), np.empty(n, np.int32), np.empty(n, np.int32)
    import ctypes
    end = ctypes.c_size_t(0)
    st = lib.fphe_wire_scan(raw.ctypes.data, raw.size, 8, n, off.ctypes.data, ln.ctypes.data, neg.ctypes.data,
                            ex.ctypes.data, rdx.ctypes.data, ctypes.byref(end))
    assert st == 0 and end.value == len(buf)
    assert ex.tolist() == es and neg.tolist() == [0, 1, 0, 0] and rdx.tolist() == [16, 16, 10, 10]
    for i, c in enumerate(cs):
        txt = buf[off[i]: off[i] + ln[i]].decode()
        assert int(txt, int(rdx[i])) == abs(c)
    st = lib.fphe_wire_scan(raw.ctypes.data, raw.size - 1, 8, n, off.ctypes.data, ln.ctypes.data, neg.ctypes.data,
                            ex.ctypes.data, rdx.ctypes.data, ctypes.byref(end))
    assert st != 0  # truncated


def _dev_cts(bits, count, seed):
    fx = fixture(bits)
    p, q = int(fx["p"], 16), int(fx["q"], 16)
    sk, pk, coder = P.keypair_from_primes(p, q)
    cs0 = [int(c, 16) for c in fx["encrypt"]["ct"]]
    es0 = list(fx["encrypt"]["exp"])
    rng = np.random.default_rng(seed)
    pick = rng.integers(0, len(cs0), count).tolist()
    cs, es = [cs0[i] for i in pick], [es0[i] for i in pick]
    cs[:3] = [1, 0, -(p * q) ** 2 + 1][:min(3, count)]  # literal 1, zero, most negative
    es[:3] = [0, -14, 5][:min(3, count)]
    cv = P.CiphertextVector.from_signed_ints(cs, es, pk.ns, pk._key.L2)
    return pk, cv, cs, es


@pytest.mark.gpu
@pytest.mark.parametrize("bits,count", [(1024, 1), (1024, 300), (2048, 4097)])
def test_ciphertext_vector_device_codec(bits, count):
    pk, cv, cs, es = _dev_cts(bits, count, count)
    b = wire.ciphertext_vector_to_bincode(cv, pk)
    assert b == ct_vec_bytes(cs, es)
    back, used = wire.ciphertext_vector_from_bincode(b + b"tail", pk)
    assert used == len(b)
    assert back.to_signed_ints(pk.ns) == (cs, es)


@pytest.mark.gpu
def test_ciphertext_vector_decode_other_radix_and_errors():
    pk, cv, cs, es = _dev_cts(1024, 40, 1)
    back, _ = wire.ciphertext_vector_from_bincode(ct_vec_bytes(cs, es, radix=10), pk)  # long decimal: host
    assert back.to_signed_ints(pk.ns) == (cs, es)
    back, _ = wire.ciphertext_vector_from_bincode(ct_vec_bytes(cs, es, radix=16), pk)  # all hex: device
    assert back.to_signed_ints(pk.ns) == (cs, es)
    small = [0, 1, -7, 2**32 - 1, 2**33, -(2**32 - 1), 10**18]  # <= 19 decimal digits: device
    back, _ = wire.ciphertext_vector_from_bincode(ct_vec_bytes(small, [0] * 7, radix=10), pk)
    assert back.to_signed_ints(pk.ns) == (small, [0] * 7)
    with pytest.raises(ValueError):  # a non-decimal character in a decimal record (device path)
        wire.ciphertext_vector_from_bincode(struct.pack("<QiQ", 1, 10, 3) + b"1a2" + struct.pack("<i", 0), pk)
    with pytest.raises(ValueError):  # doubled sign (host path: radix 7)
        wire.ciphertext_vector_from_bincode(struct.pack("<QiQ", 1, 7, 3) + b"--5" + struct.pack("<i", 0), pk)
    with pytest.raises(ValueError):  # more elements claimed than the buffer holds
        wire.ciphertext_vector_from_bincode(struct.pack("<Q", 2**40) + b"\0" * 64, pk)
    up = ct_vec_bytes(cs, es).replace(b"a", b"A")  # uppercase hex digits are accepted
    assert wire.ciphertext_vector_from_bincode(up, pk)[0].to_signed_ints(pk.ns) == (cs, es)
    with pytest.raises(ValueError):  # |c| >= n^2
        wire.ciphertext_vector_from_bincode(ct_vec_bytes([pk.ns], [0]), pk)
    with pytest.raises(ValueError):  # non-digit
        wire.ciphertext_vector_from_bincode(struct.pack("<QiQ", 1, 16, 3) + b"1g2" + struct.pack("<i", 0), pk)
    with pytest.raises(ValueError):  # truncated
        wire.ciphertext_vector_from_bincode(ct_vec_bytes(cs, es)[:-2], pk)
    empty, used = wire.ciphertext_vector_from_bincode(struct.pack("<Q", 0), pk)
    assert empty.count == 0 and used == 8


@pytest.mark.gpu
def test_plaintext_vector_codec():
    fx = fixture(1024)
    sk, pk, coder = P.keypair_from_primes(int(fx["p"], 16), int(fx["q"], 16))
    sigs, exps = [0, -3, 2**60 + 1, pk.n - 5], [-14, 2, 0, 0]
    pv = P.PlaintextVector.from_ints(sigs, exps)
    b = wire.plaintext_vector_to_bincode(pv)
    assert b == ct_vec_bytes(sigs, exps)
    assert wire.plaintext_vector_from_bincode(b).to_ints() == (sigs, exps)


def test_pickle_state_is_the_reference_bincode():
    """PK / SK / Coder pickle as the reference does (paillier.rs:67-74, 91-98, 128-135): the
    state is bincode(serde(...)), and __setstate__ takes it back as bytes or as the list of
    ints pyo3 makes of a Vec<u8>."""
    import pickle
    fx = fixture(1024)
    p, q = int(fx["p"], 16), int(fx["q"], 16)
    sk, pk, coder = P.keypair_from_primes(p, q)
    assert pk.__getstate__() == wire.pk_to_bincode(pk)
    assert sk.__getstate__() == wire.sk_to_bincode(sk)
    assert coder.__getstate__() == wire.coder_to_bincode(pk.n)
    for obj in (pk, sk, coder):
        back = pickle.loads(pickle.dumps(obj))
        assert type(back) is type(obj) and back.__getstate__() == obj.__getstate__()
        fresh = type(obj).__new__(type(obj))
        fresh.__setstate__(list(obj.__getstate__()))  # pyo3's Vec<u8> form
        assert fresh.__getstate__() == obj.__getstate__()
    assert pickle.loads(pickle.dumps(pk)).keyholder is False  # a pickled PK is public-only


def test_fate_utils_alias_passes_the_federation_allowlist():
    """compat.install(): the classes pickle under fate_utils.paillier, which FATE's restricted
    unpickler admits (arch/federation/api/_serdes.py:280, 311-333: module prefixes "fate." and
    "fate_utils." only), and FATE's adapter imports resolve (protocol/phe/paillier.py:18-23)."""
    import io
    import pickle
    import subprocess
    import sys
    code = r'''
import io, pickle, sys, json
sys.path.insert(0, %r)
from fate_amd import compat
mod = compat.install()
from fate_utils.paillier import CiphertextVector, PlaintextVector, Coder, Evaluator, PK, SK, keygen  # noqa
fx = json.load(open(%r))
import fate_amd.paillier as P
p, q = int(fx["p"], 16), int(fx["q"], 16)
sk, pk, _ = P.keypair_from_primes(p, q)
coder = Coder(p * q)
class Restricted(pickle.Unpickler):
    def find_class(self, module, name):
        if not any(module.startswith(m) for m in ("fate.", "fate_utils.")):
            raise pickle.UnpicklingError(module)
        return super().find_class(module, name)
out = []
for obj in (pk, sk, coder):
    b = pickle.dumps(obj)
    assert b"fate_utils.paillier" in b and b"fate_amd" not in b, b[:80]
    back = Restricted(io.BytesIO(b)).load()
    out.append(type(back).__module__ + "." + type(back).__name__)
assert compat.install() is mod
print(json.dumps(out))
''' % (os.path.dirname(HERE), os.path.join(HERE, "golden", "paillier_1024.json"))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert json.loads(r.stdout.strip().splitlines()[-1]) == ["fate_utils.paillier.PK", "fate_utils.paillier.SK",
                                                             "fate_utils.paillier.Coder"]


def test_alias_pickles_load_with_and_without_install(tmp_path):
    """install() leaves fate_amd.paillier's classes alone (alias subclasses
    plus copyreg reducers instead of rewriting __module__).  Objects pickled in an installed
    process load in an installed process and in one that never called install() (fate_amd's
    fallback finder serves the aliases when no real fate_utils exists), while a real fate_utils
    on sys.path still wins over the aliases."""
    import subprocess
    import sys
    root, fx = os.path.dirname(HERE), os.path.join(HERE, "golden", "paillier_1024.json")
    blob = tmp_path / "objs.pkl"
    head = f"import sys, json, pickle\nsys.path.insert(0, {root!r})\n"
    dump = head + f"""
import fate_amd.paillier as P
from fate_amd import compat
fx = json.load(open({fx!r}))
sk, pk, coder = P.keypair_from_primes(int(fx["p"], 16), int(fx["q"], 16))
compat.install()
assert P.PK.__module__ == "fate_amd.paillier" and P.CiphertextVector.__module__ == "fate_amd.paillier"
b = pickle.dumps((pk, sk, coder, P.Evaluator()))
assert b"fate_amd" not in b and b"fate_utils.paillier" in b
open({str(blob)!r}, "wb").write(b)
print(json.dumps([pk.__getstate__().hex(), sk.__getstate__().hex(), coder.__getstate__().hex()]))
"""
    load = head + f"""
INSTALL = int(sys.argv[1])
import fate_amd.paillier as P
if INSTALL:
    from fate_amd import compat
    compat.install()
objs = pickle.load(open({str(blob)!r}, "rb"))
assert [type(o).__module__ + "." + type(o).__name__ for o in objs] == [
    "fate_utils.paillier.PK", "fate_utils.paillier.SK", "fate_utils.paillier.Coder", "fate_utils.paillier.Evaluator"]
assert isinstance(objs[0], P.PK) and isinstance(objs[1], P.SK) and isinstance(objs[2], P.Coder)
print(json.dumps([o.__getstate__().hex() for o in objs[:3]]))
"""
    r = subprocess.run([sys.executable, "-c", dump], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    want = json.loads(r.stdout.strip().splitlines()[-1])
    for install in ("1", "0"):
        r = subprocess.run([sys.executable, "-c", load, install], capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, (install, r.stderr[-2000:])
        assert json.loads(r.stdout.strip().splitlines()[-1]) == want
    # a real fate_utils (here a stand-in package on sys.path) is found before the aliases
    real = tmp_path / "site" / "fate_utils"
    real.mkdir(parents=True)
    (real / "__init__.py").write_text("REAL = True\n")
    probe = head + f"sys.path.insert(0, {str(tmp_path / 'site')!r})\nimport fate_amd\nimport fate_utils\n" \
        "assert getattr(fate_utils, 'REAL', False) and not getattr(fate_utils, '_fate_amd_alias', False)\n"
    r = subprocess.run([sys.executable, "-c", probe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]


@pytest.mark.gpu
@pytest.mark.parametrize("bits", [1024, 2048])
def test_ciphertext_and_plaintext_vector_pickle(bits):
    """CiphertextVector / PlaintextVector pickle through the reference's bincode state
    (paillier.rs:219-226, 395-402).  A vector's state is the reference's key-less signed
    integers: unpickled, it stays key-less (raw) -- slices and re-pickles keep it so -- until an
    operation supplies the key, or is read under fate_amd.paillier.unpickle_key."""
    import copy
    import pickle
    pk, cv, cs, es = _dev_cts(bits, 300, 7)
    assert cv.__getstate__() == wire.ciphertext_vector_to_bincode(cv, pk) == ct_vec_bytes(cs, es)
    pk2, back = pickle.loads(pickle.dumps((pk, cv)))
    assert back.raw and back.n is None and back.to_signed_ints() == (cs, es)
    assert pickle.loads(pickle.dumps(back)).to_signed_ints() == (cs, es)  # re-pickled without a key
    sl = back.slice(5, 100)
    assert sl.raw and sl.to_signed_ints() == (cs[5:105], es[5:105])
    z = back.add(pk, P.CiphertextVector.zeros(300, pk._key.L2))  # the op gives the key
    assert not back.raw and back.n == pk.n and back.to_signed_ints(pk.ns) == (cs, es)
    assert z.to_signed_ints(pk.ns) == (cs, es)  # add(x, literal 1) = x (lib.rs:303-308)
    assert sl.add(pk, sl).to_signed_ints(pk.ns) == cv.slice(5, 100).add(pk, cv.slice(5, 100)).to_signed_ints(pk.ns)
    dc = copy.deepcopy(cv)  # a device clone, not a wire round trip
    assert dc.n == pk.n and not dc.raw and dc.C.data_ptr() != cv.C.data_ptr()
    assert dc.to_signed_ints(pk.ns) == (cs, es)
    with P.unpickle_key(pk):
        again = pickle.loads(pickle.dumps(cv))
    assert again.to_signed_ints(pk.ns) == (cs, es)
    fresh = P.CiphertextVector.__new__(P.CiphertextVector)
    with P.unpickle_key(pk):
        fresh.__setstate__(list(cv.__getstate__()))  # pyo3's Vec<u8> form
    assert fresh.to_signed_ints(pk.ns) == (cs, es)
    # ops stamp the key: an encryption's sums pickle without help
    x = torch.linspace(-3, 3, 70, device="cuda")
    e = pk.encrypt_encoded(P.Coder(pk.n).encode_f32_vec(x), True)
    s = e.add(pk, e)
    assert s.n == pk.n and pickle.loads(pickle.dumps((pk, s)))[1].to_signed_ints(pk.ns) == s.to_signed_ints(pk.ns)
    pv = P.PlaintextVector.from_ints([0, -3, 2**60 + 1], [-14, 2, 0])
    assert pickle.loads(pickle.dumps(pv)).to_ints() == pv.to_ints()


@pytest.mark.gpu
def test_two_keys_never_guessed():
    """with two keys of one size in a process, a vector pickled under key A and
    unpickled after PK B must not be read under B.  The state stays key-less and the first
    operation's key decides: under A it is bit-exact, and decrypting it under B's SK is B's
    business (no silent conversion happened in between)."""
    import pickle
    pkA, cvA, cs, es = _dev_cts(2048, 200, 11)
    assert any(c < 0 for c in cs)  # negative elements: the case a wrong n^2 would corrupt
    from fate_amd._keygen import keygen_primes
    p, q = keygen_primes(2048)
    skB, pkB, _ = P.keypair_from_primes(p, q)
    pickle.loads(pickle.dumps(pkB))  # PK B unpickled last in this thread
    back = pickle.loads(pickle.dumps(cvA))
    assert back.raw and back.to_signed_ints() == (cs, es)
    assert back.add(pkA, P.CiphertextVector.zeros(200, 128)).to_signed_ints(pkA.ns) == (cs, es)
