"""BASELINE config 4 on a 100k-sample subset, every slot bit-exact
against libgmp.

The SecureBoost histogram of 100,000 samples x 10 features x 32 bins (1 node), 2048-bit key,
config 4's generator (p = sigmoid(N(0,1)), g = p - y, h = p(1 - p), w ~ U(0.5, 1.5), bins
~ U[0, 32), seed 20241218):

  unpacked  ct x pt of the encrypted (g, h) by the per-sample weight, then iupdate with
            stride 2 (2M scatter-adds into 640 slots, 16^d exponent alignment included);
  packed    (g + 1, h) packed at precision 52, iupdate with stride 1 (1M adds into 320
            slots), chunking_cumsum_with_step per feature, pack_squeeze.

The device's own ciphertexts (exported as the reference's signed integers) are the common
input; every later stage runs once on the device and once as the reference's sequential loops
on libgmp (oracle/gmp_ref.c: gref_mul = Ciphertext::mul, lib.rs:334-349; gref_fold = the
iupdate loop of Ciphertext::add, lib.rs:724-735 and :301-333; gref_cumsum, lib.rs:760-771;
gref_squeeze, lib.rs:439-450), and the two must agree bit for bit on every element.  The
fold's large-term machinery (the raised-key slot plan, multi-round plans) is spot-checked
the same way in tests/test_gpu_fold.py.
"""
import json
import math
import os

import numpy as np
import pytest
import torch

from fate_amd import paillier as P
from oracle import gmp_ref
from oracle import paillier_oracle as O

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
S, HF, NB = 100_000, 10, 32


def exported(pk, v):
    """A device vector as libgmp's (words, neg, exp) triple."""
    mag, neg, exp = v.export_signed(pk)
    return mag.cpu().numpy().view(np.uint32), neg.cpu().numpy(), exp.cpu().numpy()


def same(a, b):
    return all(np.array_equal(x, y) for x, y in zip(a, b))


def literal_ones(k, L):
    return gmp_ref.to_vec([1] * k, [0] * k, L)


@pytest.fixture(scope="module")
def cfg4():
    with open(os.path.join(HERE, "golden", "paillier_2048.json")) as f:
        fx = json.load(f)
    p, q = int(fx["p"], 16), int(fx["q"], 16)
    sk, pk, coder = P.keypair_from_primes(p, q, keyholder=True)
    g0 = torch.Generator().manual_seed(20241218)
    pr = torch.sigmoid(torch.randn(S, generator=g0, dtype=torch.float64))
    y = (torch.rand(S, generator=g0, dtype=torch.float64) < 0.5).double()
    g, h = (pr - y).float(), (pr * (1 - pr)).float()
    w = (torch.rand(S, generator=g0) + 0.5).float()
    positions = torch.randint(0, NB, (S, HF), generator=g0) + torch.arange(HF) * NB
    return pk, coder, g, h, w, positions, gmp_ref.GmpKey(pk.n)


def test_config4_unpacked_subset_bit_exact(cfg4):
    pk, coder, g, h, w, positions, gk = cfg4
    dev = torch.device("cuda", 0)
    L = pk._key.L2
    egh = pk.encrypt_encoded(coder.encode_f32_vec(torch.stack([g, h], 1).reshape(-1).to(dev)), True)
    ew = egh.mul(pk, coder.encode_f32_vec(w.repeat_interleave(2).to(dev)))
    hist = P.CiphertextVector.zeros(HF * NB * 2, L, dev)
    hist.iupdate(ew, positions.to(dev, torch.int32), 2, pk)
    # libgmp: the weights encoded by the oracle (Coder::encode_f32), the device ciphertexts in
    src = exported(pk, egh)
    enc = [O.encode_f32(pk.n, float(x)) for x in w.tolist()]
    sig = [e.significant for e in enc for _ in (0, 1)]
    pexp = [e.exp for e in enc for _ in (0, 1)]
    got_mul = gk.mul(src, gmp_ref.to_vec(sig, pexp, 2))
    assert same(exported(pk, ew), got_mul), "ct x pt differs from libgmp"
    t = np.arange(2)
    terms = np.broadcast_to(np.arange(S)[:, None, None] * 2 + t, (S, HF, 2)).reshape(-1)
    slots = (positions.numpy()[:, :, None] * 2 + t).reshape(-1)
    want = gk.fold(got_mul, terms, slots, literal_ones(HF * NB * 2, L))
    got = exported(pk, hist)
    bad = [i for i in range(HF * NB * 2) if not (np.array_equal(got[0][i], want[0][i]) and got[1][i] == want[1][i]
                                                and got[2][i] == want[2][i])]
    assert not bad, f"{len(bad)} of 640 histogram slots differ from libgmp, e.g. {bad[:5]}"


def test_config4_packed_subset_bit_exact(cfg4):
    pk, coder, g, h, w, positions, gk = cfg4
    dev = torch.device("cuda", 0)
    L = pk._key.L2
    shift = int(math.log2(2 ** 52 * S * 2) + 1)  # compute_offset_bit (guest.py:203-206)
    squeeze_num = (pk.n.bit_length() - 2) // (shift * 2)
    vals = torch.stack([g.double() + 1.0, h.double()], 1).reshape(-1).to(dev)
    en = pk.encrypt_encoded(coder.pack_floats(vals, shift, 2, 52), True)
    hp = P.CiphertextVector.zeros(HF * NB, L, dev)
    hp.iupdate(en, positions.to(dev, torch.int32), 1, pk)
    folded = exported(pk, hp)
    want = gk.fold(exported(pk, en), np.repeat(np.arange(S), HF), positions.numpy().reshape(-1),
                   literal_ones(HF * NB, L))
    assert same(folded, want), "packed iupdate differs from libgmp"
    hp.chunking_cumsum_with_step(pk, [NB] * HF, 1)
    want = gk.cumsum(want, [NB] * HF, 1)
    assert same(exported(pk, hp), want), "chunking_cumsum_with_step differs from libgmp"
    sq = hp.pack_squeeze(squeeze_num, shift * 2, pk)
    assert same(exported(pk, sq), gk.squeeze(want, squeeze_num, shift * 2)), "pack_squeeze differs from libgmp"
