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
        buf = bytearray(k)
        view, got = memoryview(buf), 0
        while got < k:
            r = sock.recv_into(view[got:], k - got)
            if not r:
                raise EOFError("peer closed")
            got += r
        return bytes(buf)
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
        # the host's sum, decrypted, against the float sum; and bit-exact against the CPU
        # oracle's Ciphertext::add (fixedpoint_paillier/src/lib.rs:301-333) of the exchanged
        # signed integers (all of them up to 8192 elements, else a random subset of 4096)
        raw_key_less = bool(ct_sum.raw)  # unpickled without a PK: key-less until decrypt
        got = coder.decode_f32_vec(sk.decrypt_to_encoded(ct_sum)).cpu().double()
        xh = (0.25 * torch.randn(n, generator=torch.Generator().manual_seed(7))).to(torch.float32)
        want = d.double() + xh.double()
        from oracle import paillier_oracle as O
        opk = O.keypair_from_primes(int(fx["p"], 16), int(fx["q"], 16))[1]
        idx = torch.arange(n) if n <= 8192 else torch.randperm(n, generator=torch.Generator().manual_seed(3))[:4096]
        idx = idx.sort().values
        sub = lambda v: v.slice_indexes(idx.tolist()).to_signed_ints(pk.ns)  # noqa: E731
        (a, ea), (b, eb), (s, es) = sub(ct_d), sub(ct_h), sub(ct_sum)
        oracle = [O.ct_add(opk, O.Ciphertext(x, ex), O.Ciphertext(y, ey)) for x, ex, y, ey in zip(a, ea, b, eb)]
        out = {"allclose": bool(torch.allclose(got, want, rtol=1e-6, atol=1e-6)),
               "bit_exact": [(c.c, c.exp) for c in oracle] == list(zip(s, es)),
               "checked": len(oracle), "received_key_less": raw_key_less,
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
