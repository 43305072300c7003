"""Writes tests/golden/key_4096.json: one 4096-bit Paillier key (p < q, bits(pq) = 4096) drawn
the way fate_amd._keygen draws keys (paillier/src/lib.rs:72-87: two random half-size primes,
next-prime search), for bench.py's 4096-bit leg, so the bench does not spend its time on
prime generation.  Data, not a vector: the bench checks its own round trips."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from fate_amd._keygen import keygen_primes  # noqa: E402

p, q = keygen_primes(4096)
with open(os.path.join(HERE, "key_4096.json"), "w") as f:
    json.dump({"bits": 4096, "p": format(p, "x"), "q": format(q, "x")}, f, indent=1)
