"""Child process of tests/test_gpu_rccl.py: the multi-GPU data path of fate_amd.dist on the
real collective backend (torch.distributed "nccl" = RCCL on ROCm), world_size 1 on the one
GPU of the test box.  The process group is initialised before any other GPU work, as a
bench.py rank does.  Prints one JSON line; exit status 0 iff every check passed.

Checks (bit for bit):
  * gather_tiles / gather_ciphertexts of encrypted shards (whole tiles, a partial last tile,
    an empty shard) return the shard itself, sign gathered as uint8, onto every rank and onto
    one rank (gather_ciphertexts(dst=0));
  * compact_gathered on padded multi-rank buffers (whole-tile and ragged shard counts);
  * fold_across_ranks / fold_partials -- the cross-rank SecureBoost histogram fold -- against
    the sequential ct-add chain (k_add27) over the same partials and against the oracle.
"""
import json
import os
import socket
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    res = {"backend": dist.get_backend()}
    try:
        from fate_amd import paillier as P
        from fate_amd.dist import compact_gathered, fold_across_ranks, fold_partials, gather_ciphertexts, gather_tiles
        from oracle import paillier_oracle as O

        fx = json.load(open(os.path.join(ROOT, "tests", "golden", "paillier_2048.json")))
        p, q = int(fx["p"], 16), int(fx["q"], 16)
        sk, pk, coder = P.keypair_from_primes(p, q)
        g = torch.Generator().manual_seed(7)
        ok = True
        # 1. all-gather of ciphertext shards over RCCL (world 1: the shard comes back)
        for n in (0, 64, 1000, 4096 + 17):
            x = (torch.randn(max(n, 1), generator=g) * 3)[:n].to(dev)
            cv = pk.encrypt_encoded(coder.encode_f32_vec(x), True)
            if n:
                cv.sign[: n // 3] = 1  # exercise the byte-wide sign gather
            C, sg, eg, tot = gather_tiles(cv.C, cv.sign, cv.exp, n)
            nt = (n + 63) // 64
            ok &= tot == n and sg.dtype == torch.uint8
            ok &= bool(torch.equal(C[:nt], cv.C[:nt])) and bool(torch.equal(sg[:n], cv.sign[:n]))
            ok &= bool(torch.equal(eg[:n], cv.exp[:n]))
            gv = gather_ciphertexts(cv)
            ok &= gv.n == pk.n and gv.count == n
            g0 = gather_ciphertexts(cv, dst=0)  # onto one rank: point-to-point (here: the rank itself)
            ok &= g0.n == pk.n and g0.count == n and bool(torch.equal(g0.C[:nt], cv.C[:nt]))
            if n:
                ok &= gv.to_signed_ints(pk.ns) == cv.to_signed_ints(pk.ns)
        res["gather"] = ok
        # 2. compaction of padded multi-rank buffers on the device (what ranks > 1 receive)
        ok2 = True
        L = pk._key.L2
        for counts in ([128, 128, 70], [128, 64, 0], [70, 5, 64], [0, 33, 64]):
            nt_max = max((c + 63) // 64 for c in counts)
            world = len(counts)
            full = [torch.randint(0, 2 ** 31 - 1, (c, L), generator=g, dtype=torch.int32) for c in counts]
            Cg = torch.zeros((world * nt_max, L, 64), dtype=torch.int32)
            sg = torch.zeros(world * nt_max * 64, dtype=torch.uint8)
            eg = torch.zeros(world * nt_max * 64, dtype=torch.int32)
            for r, rows in enumerate(full):
                for k in range(rows.shape[0]):
                    Cg[r * nt_max + k // 64, :, k % 64] = rows[k]
                    sg[r * nt_max * 64 + k] = (r + k) % 2
                    eg[r * nt_max * 64 + k] = -(r * 7 + k)
            C2, s2, e2, tot = compact_gathered(Cg.to(dev), sg.to(dev), eg.to(dev), counts)
            want = torch.cat(full) if sum(counts) else torch.zeros((0, L), dtype=torch.int32)
            got = C2.permute(0, 2, 1).reshape(-1, L)[:tot].cpu()
            ws = torch.tensor([(r + k) % 2 for r, c in enumerate(counts) for k in range(c)], dtype=torch.uint8)
            we = torch.tensor([-(r * 7 + k) for r, c in enumerate(counts) for k in range(c)], dtype=torch.int32)
            ok2 &= tot == sum(counts) and bool(torch.equal(got, want))
            ok2 &= bool(torch.equal(s2[:tot].cpu(), ws)) and bool(torch.equal(e2[:tot].cpu(), we))
        res["compact"] = ok2
        # 3. cross-rank histogram fold
        ok3 = True
        NS, HF, NB = 3000, 2, 8
        m = HF * NB * 2
        parts = []
        for r in range(3):  # three "ranks'" partial histograms from their own samples
            x = (torch.randn(2 * NS, generator=g) * 2).to(dev)
            gh = pk.encrypt_encoded(coder.encode_f32_vec(x), True)
            pos = torch.randint(0, NB, (NS, HF), generator=g) + torch.arange(HF) * NB
            h = P.CiphertextVector.zeros(m, L, dev)
            if r != 1:  # rank 1 holds an untouched zeros() histogram: literal 1s
                h.iupdate(gh, pos, 2, pk)
            parts.append(h)
        folded1, tg, tf = fold_across_ranks(pk, parts[0])  # world 1 over RCCL: itself
        ok3 &= folded1.to_signed_ints(pk.ns) == parts[0].to_signed_ints(pk.ns)
        allp = P.Evaluator.cat(parts)
        fp = fold_partials(pk, allp, 3, m)
        chain = parts[0]
        for r in (1, 2):
            chain = chain.add(pk, parts[r])
        ok3 &= fp.to_signed_ints(pk.ns) == chain.to_signed_ints(pk.ns)
        # oracle: the same chain of Ciphertext::add on the signed integers
        opk = O.keypair_from_primes(p, q)[1]
        ints = [parts[r].to_signed_ints(pk.ns) for r in range(3)]
        want = []
        for j in range(m):
            acc = O.Ciphertext(ints[0][0][j], ints[0][1][j])
            for r in (1, 2):
                acc = O.ct_add(opk, acc, O.Ciphertext(ints[r][0][j], ints[r][1][j]))
            want.append((acc.c, acc.exp))
        got_c, got_e = fp.to_signed_ints(pk.ns)
        ok3 &= list(zip(got_c, got_e)) == want
        res["fold"] = ok3
        res["gather_s"], res["fold_s"] = round(tg, 5), round(tf, 5)
        res["ok"] = bool(ok and ok2 and ok3)
    finally:
        dist.destroy_process_group()
    print(json.dumps(res), flush=True)
    return 0 if res.get("ok") else 1


if __name__ == "__main__":
    sys.exit(main())
