"""BASELINE config 3 (up to its full 1M size) across two loopback parties: a guest process encrypts half_d with its
key, a host process (public key only) receives PK and ciphertexts as the reference's pickles,
encrypts its own term and adds, and the guest decrypts the returned sum -- two processes on
the GPU, ciphertexts crossing a socket as fate_utils.paillier bincode state under FATE's
restricted unpickler (tests/loopback_party.py)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.parametrize("bits,n", [(1024, 20000), (2048, 5000), (2048, 1 << 20)])
def test_two_party_hetero_lr_exchange(bits, n):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    fixture = os.path.join(HERE, "golden", f"paillier_{bits}.json")
    script = os.path.join(HERE, "loopback_party.py")
    cmd = lambda role: [sys.executable, script, role, str(port), fixture, str(n)]  # noqa: E731
    guest = subprocess.Popen(cmd("guest"), stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    host = subprocess.Popen(cmd("host"), stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    try:
        hout, herr = host.communicate(timeout=240)
        gout, gerr = guest.communicate(timeout=120)
    finally:
        for p in (host, guest):
            if p.poll() is None:
                p.kill()
                p.wait()
    assert host.returncode == 0, herr[-2000:]
    assert guest.returncode == 0, gerr[-2000:]
    res = json.loads(gout.strip().splitlines()[-1])
    assert res["allclose"] and res["bit_exact"], res
    assert res["types"] == ["fate_utils.paillier.CiphertextVector"]
    assert res["received_key_less"]  # no PK travelled with the sum: read under the SK at decrypt
    assert res["checked"] == (n if n <= 8192 else 4096)
