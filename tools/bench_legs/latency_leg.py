"""Latency of the calls that hold few elements -- pack_squeeze and decrypt of a handful of
ciphertexts (SecureBoost's squeezed histograms, a Hetero-LR gradient), encryption of a
batch by either party -- on the one-element-
per-wave kernels (fate_amd/csrc/wide_dev.h) against the throughput kernels, 2048-bit key.
Each mode runs in its own process (FPHE_WIDE_DECRYPT_MAX is read once per process):

    python tools/bench_legs/latency_leg.py          # both modes, one JSON line each
"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(mode: str) -> dict:
    sys.path.insert(0, ROOT)
    import torch
    from fate_amd import paillier as P
    fx = json.load(open(os.path.join(ROOT, "tests", "golden", "paillier_2048.json")))
    sk, pk, coder = P.keypair_from_primes(int(fx["p"], 16), int(fx["q"], 16), keyholder=False)
    dev = torch.device("cuda", 0)
    if mode == "throughput":
        P.WIDE_SQUEEZE_MAX_CHUNKS = 0
    out = {"mode": mode}
    x = torch.randn(2048, generator=torch.Generator().manual_seed(5), dtype=torch.float64).to(dev)
    v = pk.encrypt_encoded(coder.encode_f64_vec(x), True)
    for n in (4, 25, 320, 2048):
        s = v.slice(0, n)
        sk.decrypt_to_encoded(s)  # warm
        torch.cuda.synchronize(dev)
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            d = sk.decrypt_to_encoded(s)
            torch.cuda.synchronize(dev)
            ts.append(time.perf_counter() - t0)
        out[f"decrypt_{n}_ms"] = round(min(ts) * 1e3, 3)
        out[f"decrypt_{n}_ok"] = bool(torch.allclose(coder.decode_f64_vec(d), x[:n], rtol=0, atol=0))
    for n in (1, 16, 256, 2048):
        xe = coder.encode_f64_vec(x[:n])
        pk.encrypt_encoded(xe, True)  # warm
        torch.cuda.synchronize(dev)
        ts = []
        for _ in range(2):
            t0 = time.perf_counter()
            pk.encrypt_encoded(xe, True)
            torch.cuda.synchronize(dev)
            ts.append(time.perf_counter() - t0)
        out[f"encrypt_{n}_ms"] = round(min(ts) * 1e3, 3)
    _, pk_kh, _ = P.keypair_from_primes(int(fx["p"], 16), int(fx["q"], 16), keyholder=True)
    for n in (1, 16, 256, 2048, 4096):
        xe = coder.encode_f64_vec(x[:n] if n <= 2048 else x.repeat(2))
        pk_kh.encrypt_encoded(xe, True)  # warm
        torch.cuda.synchronize(dev)
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            pk_kh.encrypt_encoded(xe, True)
            torch.cuda.synchronize(dev)
            ts.append(time.perf_counter() - t0)
        out[f"keyholder_encrypt_{n}_ms"] = round(min(ts) * 1e3, 3)
    for slots, shift in ((128, 148), (320, 154)):
        s = v.slice(0, slots)
        s.pack_squeeze(13, shift, pk)
        torch.cuda.synchronize(dev)
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            s.pack_squeeze(13, shift, pk)
            torch.cuda.synchronize(dev)
            ts.append(time.perf_counter() - t0)
        out[f"squeeze_{slots}_ms"] = round(min(ts) * 1e3, 3)
    return out


if __name__ == "__main__":
    if len(sys.argv) > 1:
        print(json.dumps(run(sys.argv[1])), flush=True)
    else:
        for mode, env in (("wide", {}), ("throughput", {"FPHE_WIDE_DECRYPT_MAX": "0", "FPHE_WIDE_ENCRYPT_MAX": "0",
                                                                "FPHE_WIDE_KH_ENCRYPT_MAX": "0"})):
            r = subprocess.run([sys.executable, os.path.abspath(__file__), mode], env={**os.environ, **env},
                               capture_output=True, text=True, timeout=600)
            line = [l for l in r.stdout.splitlines() if l.startswith("{")]
            print(line[-1] if line else json.dumps({"mode": mode, "error": r.stderr[-500:]}), flush=True)
