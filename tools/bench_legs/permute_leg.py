"""Time fphe_permute gathers/scatters of 2^20 2048-bit ciphertexts (identity, stable-sorted
and random index orders)."""
import json, os, sys, time, torch
sys.path.insert(0, os.environ["GRAFT_REPO_ROOT"])
from fate_amd import paillier as P
N = 1 << 20
dev = torch.device("cuda", 0)
C = torch.randint(0, 2**31 - 1, (N // 64, 128, 64), dtype=torch.int32, device=dev)
v = P.CiphertextVector(C, torch.zeros(N, dtype=torch.uint8, device=dev), torch.zeros(N, dtype=torch.int32, device=dev), N)
for name, idx in (("identity", torch.arange(N)), ("sorted_half", torch.sort(torch.randint(0, 3, (N,)), stable=True)[1]), ("random", torch.randperm(N))):
    idx = idx.to(dev)
    for rep in range(2):
        torch.cuda.synchronize(); t0 = time.perf_counter(); g = v._gather(idx); torch.cuda.synchronize(); tg = time.perf_counter() - t0
        torch.cuda.synchronize(); t0 = time.perf_counter(); v._assign(idx, g); torch.cuda.synchronize(); ta = time.perf_counter() - t0
    print(json.dumps({"idx": name, "gather_ms": round(tg * 1e3, 3), "assign_ms": round(ta * 1e3, 3), "GBps_gather": round(2 * N * 512 / tg / 1e9, 1)}))
