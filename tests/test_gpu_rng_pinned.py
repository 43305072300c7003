"""Device-drawn obfuscation pinned to the oracle, integer for integer.

The reference draws r from OS entropy (math/src/rug/random.rs:15-25), so its ciphertexts
cannot be reproduced; the parity tests inject r instead.  This backend draws r (or the key
holder's (z_p, z_q)) from ChaCha20 keyed per key context (fate_phe.hip draw_r / k_draw_z).
With the key and the call nonce fixed, tests/chacha_ref.py recomputes every element's draw on
the host, and the device's ciphertexts must equal the reference's encryption
(paillier/src/lib.rs:104-121 through fixedpoint_paillier/src/lib.rs:370-381; libgmp,
oracle/gmp_ref.c) with that r.  This covers the paths the bench times with device RNG:

- public-key encrypt, r drawn (k_draw_r, then k_encrypt27 + k_mont_const27, or k_encrypt_wide);
- key-holder encrypt, r drawn (FPHE_OPT_KH_DIRECT_Z = 0: k_draw_r, k_pow_small27,
  k_pow_half27<., ., true>, k_encrypt_crt27);
- key-holder encrypt, (z_p, z_q) drawn (k_draw_z, then k_pow_half27<., ., true, true> or
  k_pow_half_enc_wide, then k_encrypt_crt27).  The device never forms r here.  The test
  recovers the r whose CRT coordinates the draw stands for: r_s = z_s^(e_s^-1 mod (s - 1))
  mod s, with e_p = q mod (p - 1), which is invertible because gcd(q, p - 1) = 1.  Then
  r^n = (r^(e_p))^p = z_p^p mod p^2, and likewise mod q^2.  So the device's ciphertext must be
  the reference's encrypt(m, CRT(r_p, r_q)).  (z_p, z_q) is uniform, and so is that r
  (DESIGN.md §3).
"""
import ctypes
import json
import os

import numpy as np
import pytest
import torch

from fate_amd import paillier as P
from tests.chacha_ref import DRAW_HALF_TAG, DRAW_Z_TAG, draw_below_host

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
KEY = [0x01234567, 0x89ABCDEF, 0xDEADBEEF, 0x0BADF00D, 0x13579BDF, 0x2468ACE0, 0xFEEDFACE, 0x31415926]
NONCE = (0x5EED << 40) ^ 0xC0FFEE


def _key(bits):
    name = f"paillier_{bits}.json" if bits in (1024, 2048) else f"key_{bits}.json"
    with open(os.path.join(HERE, "golden", name)) as f:
        fx = json.load(f)
    p, q = sorted((int(fx["p"], 16), int(fx["q"], 16)))
    return p, q


def _inputs(n, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, generator=g, dtype=torch.float64) * 4
    x[:4] = torch.tensor([0.0, -1e-300, 3e38, -1.0], dtype=torch.float64)
    return x


def _fix_rng(monkeypatch, kctx):
    monkeypatch.setattr(kctx, "rng_key", (ctypes.c_uint32 * 8)(*KEY))
    monkeypatch.setattr(kctx, "next_nonce", lambda: NONCE)


COUNTS = {1024: 2500, 2048: 2500, 4096: 300}


@pytest.mark.parametrize("bits", [1024, 2048, 4096])
def test_public_drawn_r_matches_reference(monkeypatch, kernel_path, bits):
    from oracle import gmp_ref
    p, q = _key(bits)
    n = p * q
    sk, pk, coder = P.keypair_from_primes(p, q, keyholder=False)
    _fix_rng(monkeypatch, pk._key)
    x = _inputs(COUNTS[bits], bits)
    pv = coder.encode_f64_vec(x.cuda())
    sig, exp = pv.to_ints()
    got, got_e = pk.encrypt_encoded(pv, True).to_signed_ints(pk.ns)
    r = draw_below_host(KEY, NONCE, len(sig), n, pk._key.L1)
    assert got_e == exp
    assert got == gmp_ref.parallel("encrypt", n, p, q, list(zip(sig, r)))


@pytest.mark.parametrize("bits", [1024, 2048])
def test_keyholder_drawn_r_matches_reference(monkeypatch, bits):
    """FPHE_OPT_KH_DIRECT_Z = 0: the key holder draws r as the public path does (same stream),
    and its two-step CRT modexp gives the reference's integers for that r."""
    from oracle import gmp_ref
    p, q = _key(bits)
    n = p * q
    sk, pk, coder = P.keypair_from_primes(p, q)
    assert pk.keyholder
    _fix_rng(monkeypatch, pk._priv)
    x = _inputs(COUNTS[bits], bits + 1)
    pv = coder.encode_f64_vec(x.cuda())
    sig, _ = pv.to_ints()
    with P.path_options(kh_direct_z=0):
        assert P.path_option(pv.device, pk._priv, "kh_direct_z") == 0
        got, _ = pk.encrypt_encoded(pv, True).to_signed_ints(pk.ns)
    r = draw_below_host(KEY, NONCE, len(sig), n, pk._key.L1)
    assert got == gmp_ref.parallel("encrypt", n, p, q, list(zip(sig, r)))


@pytest.mark.parametrize("bits", [1024, 2048, 4096])
def test_keyholder_drawn_z_matches_reference(monkeypatch, kernel_path, bits):
    from oracle import gmp_ref
    p, q = _key(bits)
    n = p * q
    sk, pk, coder = P.keypair_from_primes(p, q)
    _fix_rng(monkeypatch, pk._priv)
    x = _inputs(COUNTS[bits], bits + 2)
    pv = coder.encode_f64_vec(x.cuda())
    assert P.path_option(pv.device, pk._priv, "kh_direct_z") == 1  # gcd(q, p-1) = gcd(p, q-1) = 1
    sig, exp = pv.to_ints()
    got, got_e = pk.encrypt_encoded(pv, True).to_signed_ints(pk.ns)
    lq = pk._key.L1 // 2
    zp = draw_below_host(KEY, NONCE, len(sig), p, lq, DRAW_Z_TAG)
    zq = draw_below_host(KEY, NONCE, len(sig), q, lq, DRAW_Z_TAG | DRAW_HALF_TAG)
    dp = pow(q % (p - 1), -1, p - 1)
    dq = pow(p % (q - 1), -1, q - 1)
    qinv = pow(q, -1, p)
    r = []
    for a, b in zip(zp, zq):
        rp, rq = pow(a, dp, p), pow(b, dq, q)
        r.append(rq + q * ((rp - rq) * qinv % p))  # CRT: r = rp mod p, rq mod q, in [1, n-1]
    assert got_e == exp
    assert got == gmp_ref.parallel("encrypt", n, p, q, list(zip(sig, r)))
    # the draws are distinct per element and per half (no repeated stream)
    assert len(set(zp)) == len(zp) and len(set(zq)) == len(zq)
    assert np.mean([a < p // 2 for a in zp]) == pytest.approx(0.5, abs=0.1)
