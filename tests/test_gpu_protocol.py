"""The drop-in seam on the GPU: fate_amd.protocol (keygen / evaluator / SK / PK / Coder, the
module PHECipherBuilder.setup imports, arch/context/_cipher.py:111-124) driven with the
call sequences of the reference's own tests, python/fate/test/test_vertor_paillier.py:10-66.
There the PHETensor layer (tensor/phe/_ops.py:52-266) turns torch.add(enc, enc) into
evaluator.add, torch.add(enc, 1) into add_plain_scalar, torch.add(enc, t) into add_plain,
and so on.  The reference tests only print; here the decrypted results are checked against
the float computation.  Inputs are CPU tensors, as in the reference."""
import pytest
import torch

from fate_amd import protocol as PR

pytestmark = pytest.mark.gpu

EV = PR.evaluator
X = torch.tensor([[1.0, 2.0, 3.0, 4.0], [5.0, 6.0, 7.0, -8.0]])


@pytest.fixture(scope="module")
def keys():
    return PR.keygen(1024)


def enc(keys, x):
    sk, pk, coder = keys
    return pk.encrypt_encoded(coder.encode_tensor(x), obfuscate=True)


def dec(keys, e, dtype, shape):
    sk, pk, coder = keys
    return coder.decode_tensor(sk.decrypt_to_encoded(e), dtype, shape)


def test_add(keys):
    sk, pk, coder = keys
    r = torch.rand(2, 4, generator=torch.Generator().manual_seed(1))
    e = enc(keys, X)
    e = EV.add(e, e, pk)
    e = EV.add_plain_scalar(e, 1, pk, coder, torch.float32)
    e = EV.add_plain(e, r, pk, coder)
    e = EV.add_plain_scalar(e, torch.tensor(0.3), pk, coder, torch.float32)
    assert torch.allclose(dec(keys, e, torch.float32, X.shape), X + X + 1 + r + 0.3)


def test_sub(keys):
    sk, pk, coder = keys
    r = torch.rand(2, 4, generator=torch.Generator().manual_seed(2))
    e = enc(keys, X)
    e = EV.sub(e, e, pk)
    e = EV.sub_plain_scalar(e, 1, pk, coder, torch.float32)
    e = EV.sub_plain(e, r, pk, coder)
    e = EV.sub_plain_scalar(e, torch.tensor(0.3), pk, coder, torch.float32)
    assert torch.allclose(dec(keys, e, torch.float32, X.shape), X - X - 1 - r - 0.3)


def test_rsub(keys):
    sk, pk, coder = keys
    r = torch.rand(2, 4, generator=torch.Generator().manual_seed(3))
    e = enc(keys, X)
    e = EV.rsub(e, e, pk)
    e = EV.rsub_plain_scalar(e, 1, pk, coder, torch.float32)
    e = EV.rsub_plain(e, r, pk, coder)
    e = EV.rsub_plain_scalar(e, torch.tensor(0.3), pk, coder, torch.float32)
    want = 0.3 - (r - (1 - (X - X)))
    assert torch.allclose(dec(keys, e, torch.float32, X.shape), want)


def test_mul(keys):
    sk, pk, coder = keys
    r = torch.rand(2, 4, generator=torch.Generator().manual_seed(4))
    e = enc(keys, X)
    e = EV.mul_plain_scalar(e, 2, pk, coder, torch.int64)
    e = EV.mul_plain(e, r, pk, coder)
    assert torch.allclose(dec(keys, e, torch.float32, X.shape), X * 2 * r)


def test_matmul_rmatmul(keys):
    sk, pk, coder = keys
    g = torch.Generator().manual_seed(5)
    x, y = torch.rand(5, 2, generator=g), torch.rand(2, 4, generator=g)
    z = EV.matmul(enc(keys, x), y, [5, 2], [2, 4], pk, coder, torch.float32)
    assert torch.allclose(dec(keys, z, torch.float32, (5, 4)), x @ y)
    x2, y2 = torch.rand(2, 5, generator=g), torch.rand(4, 2, generator=g)
    z2 = EV.rmatmul(enc(keys, x2), y2, [2, 5], [4, 2], pk, coder, torch.float32)
    assert torch.allclose(dec(keys, z2, torch.float32, (4, 5)), y2 @ x2)


def test_slice_cat_update_cumsum(keys):
    """The histogram-side evaluator calls (arch/histogram/values/_cipher.py:43-149)."""
    sk, pk, coder = keys
    v = torch.arange(12, dtype=torch.float64)
    e = enc(keys, v)
    parts = [EV.slice(e, 0, 4), EV.slice(e, 4, 8)]
    c = EV.cat(parts)
    assert torch.equal(dec(keys, c, torch.float64, (12,)), v)
    h = EV.zeros(3, torch.float64)
    EV.i_update(pk, h, e, [[0], [1], [2], [0]] * 3, 1)
    want = torch.zeros(3, dtype=torch.float64)
    for i, p in enumerate([0, 1, 2, 0] * 3):
        want[p] += v[i]
    assert torch.equal(dec(keys, h, torch.float64, (3,)), want)
    EV.chunking_cumsum_with_step(pk, e, [6, 6], 1)
    assert torch.equal(dec(keys, e, torch.float64, (12,)), torch.cat([v[:6].cumsum(0), v[6:].cumsum(0)]))
