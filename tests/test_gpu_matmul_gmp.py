"""BASELINE config 3's gradient step at scale, bit-exact against libgmp: the Hetero-LR host's
``torch.matmul(encode_as_int_f(X.T), enc_half_d)`` (ml/glm/hetero/coordinated_lr/host.py:242),
i.e. ``CiphertextVector.rmatmul`` (fixedpoint_paillier/src/lib.rs:882-908): out[i] = the fold
of enc_d[k].mul(X[i, k]) over k, from the reference's zero.  20,000 samples x 4 features at
2048 bits, float32 features (float significands: the exponents differ, so the fold aligns) and
int64 features of both signs (encoded negative integers: the invert branch of
Ciphertext::mul, lib.rs:334-349).  libgmp (oracle/gmp_ref.c gref_mul, gref_fold) recomputes
the products and the reference's sequential add_assign loop from the device's own encrypted
d, and every output must agree bit for bit (matmul / rmatmul are checked against the Python
oracle at small sizes in tests/test_gpu_ops.py)."""
import json
import os

import numpy as np
import pytest
import torch

from fate_amd import paillier as P
from oracle import gmp_ref

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
NS, F = 20_000, 4


def exported(pk, v):
    mag, neg, exp = v.export_signed(pk)
    return mag.cpu().numpy().view(np.uint32), neg.cpu().numpy(), exp.cpu().numpy()


@pytest.mark.parametrize("features", ["float32", "int64"])
def test_rmatmul_hetero_lr_gradient_vs_gmp(features):
    with open(os.path.join(HERE, "golden", "paillier_2048.json")) as f:
        fx = json.load(f)
    sk, pk, coder = P.keypair_from_primes(int(fx["p"], 16), int(fx["q"], 16))
    g = torch.Generator().manual_seed(31337)
    xw = torch.randn(NS, generator=g)
    y = (torch.rand(NS, generator=g) < 0.5).float() * 2 - 1
    d = (0.25 * xw - 0.5 * y).cuda()
    enc_d = pk.encrypt_encoded(coder.encode_f32_vec(d), True)
    if features == "float32":
        X = torch.randn(NS, F, generator=g)
        pt = coder.encode_f32_vec(X.t().contiguous().reshape(-1).cuda())
    else:
        X = torch.randint(-1000, 1000, (NS, F), generator=g, dtype=torch.int64)
        pt = coder.encode_i64_vec(X.t().contiguous().reshape(-1).cuda())
    grad = enc_d.rmatmul(pk, pt, [NS, 1], [F, NS])
    got = exported(pk, grad)
    # libgmp: products enc_d[k] * X[i, k] for every (i, k), then the per-feature fold
    dw, dn, de = exported(pk, enc_d)
    src = (np.tile(dw, (F, 1)), np.tile(dn, F), np.tile(de, F))
    sig, exp = pt.to_ints()
    L = dw.shape[1]
    lp = max(1, max(abs(s).bit_length() for s in sig) // 32 + 1)
    gk = gmp_ref.GmpKey(pk.n)
    prods = gk.mul(src, gmp_ref.to_vec(sig, exp, lp))
    want = gk.fold(prods, np.arange(F * NS), np.repeat(np.arange(F), NS), gmp_ref.to_vec([1] * F, [0] * F, L))
    assert all(np.array_equal(a, b) for a, b in zip(got, want))
