"""2^17 obfuscated public-key encryptions and their decryption at 2048 bits (k_encrypt27 at TPI 4,
k_pow_half27 at TPI 2): a short program for SQ counter passes comparing the two geometries."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from fate_amd import paillier as P  # noqa: E402

fx = json.load(open(os.path.join(ROOT, "tests", "golden", "paillier_2048.json")))
sk, pk, coder = P.keypair_from_primes(int(fx["p"], 16), int(fx["q"], 16), keyholder=False)
x = torch.randn(1 << 17, generator=torch.Generator().manual_seed(2)).cuda()
c = pk.encrypt_encoded(coder.encode_f32_vec(x), True)
d = sk.decrypt_to_encoded(c)
torch.cuda.synchronize()
print(json.dumps({"ok": bool(torch.equal(coder.decode_f32_vec(d), x))}))
