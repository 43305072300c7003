"""One party of the two-process loopback test (tests/test_gpu_loopback.py): BASELINE config 3's
Hetero-LR gradient exchange between a guest (key holder) and a host over a local socket,
ciphertexts crossing as the reference's pickles (fate_utils.paillier classes, bincode
state) under FATE's restricted unpickler (arch/federation/api/_serdes.py:280, 311-333).

    python tests/loopback_party.py guest|host PORT FIXTURE N
"""
import io
import json
import os
import pickle
import socket
import struct
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


class Restricted(pickle.Unpickler):
    def find_class(self, module, name):
        if not any(module.startswith(m) for m in ("fate.", "fate_utils.")):
            raise pickle.UnpicklingError(f"{module}.{name} is not allowed")
        return super().find_class(module, name)


def send(sock, obj):
    b = pickle.dumps(obj)
    sock.sendall(struct.pack("<Q", len(b)) + b)
    return len(b)


def recv(sock):
    def exact(k):
        buf = b""
        while len(buf) < k:
            chunk = sock.recv(k - len(buf))
            if not chunk:
                raise EOFError("peer closed")
            buf += chunk
        return buf
    (k,) = struct.unpack("<Q", exact(8))
    return Restricted(io.BytesIO(exact(k))).load()


def main():
    role, port, fixture, n = sys.argv[1], int(sys.argv[2]), sys.argv[3], int(sys.argv[4])
    from fate_amd import compat
    fu = compat.install()
    import torch
    from fate_amd import paillier as P
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(20241218)
    if role == "guest":
        fx = json.load(open(fixture))
        sk, pk, coder = P.keypair_from_primes(int(fx["p"], 16), int(fx["q"], 16))
        xw = torch.randn(n, generator=g)
        y = torch.where(torch.rand(n, generator=g) < 0.5, -1.0, 1.0)
        d = (0.25 * xw - 0.5 * y).to(torch.float32)  # half_d of coordinated_lr/guest.py
        srv = socket.create_server(("127.0.0.1", port))
        conn, _ = srv.accept()
        ct_d = pk.encrypt_encoded(coder.encode_f32_vec(d.to(dev)), True)
        nbytes = send(conn, (fu.PK(pk.n), ct_d))
        ct_sum, ct_h = recv(conn)
        # the host's sum, decrypted, against the float sum; and bit-exact against the
        # guest's own add of the same two ciphertext vectors
        got = coder.decode_f32_vec(sk.decrypt_to_encoded(ct_sum)).cpu().double()
        xh = (0.25 * torch.randn(n, generator=torch.Generator().manual_seed(7))).to(torch.float32)
        want = d.double() + xh.double()
        mine = ct_d.add(pk, ct_h)
        out = {"allclose": bool(torch.allclose(got, want, rtol=1e-6, atol=1e-6)),
               "bit_exact": mine.to_signed_ints(pk.ns) == ct_sum.to_signed_ints(pk.ns),
               "types": [type(ct_sum).__module__ + "." + type(ct_sum).__name__],
               "pickle_bytes_sent": nbytes}
        print(json.dumps(out), flush=True)
        conn.close()
    else:
        for _ in range(600):
            try:
                sock = socket.create_connection(("127.0.0.1", port))
                break
            except OSError:
                time.sleep(0.1)
        pk, ct_d = recv(sock)
        assert not pk.keyholder  # a pickled PK is public-only
        coder = fu.Coder(pk.n)
        xh = (0.25 * torch.randn(n, generator=torch.Generator().manual_seed(7))).to(torch.float32)
        ct_h = pk.encrypt_encoded(coder.encode_f32_vec(xh.to(dev)), True)
        ct_sum = ct_d.add(pk, ct_h)
        send(sock, (ct_sum, ct_h))
        sock.close()


if __name__ == "__main__":
    main()
