"""Multi-process (world sizes 2, 4 and 8, gloo, CPU) tests of the element sharding and the ciphertext
all-gather used for N>1 GPUs (fate_amd/dist.py).  The data-path collective is exercised on
CPU tensors in the same tile-major layout the GPU kernels produce."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from fate_amd.dist import WAVE, compact_gathered, gather_tiles, gather_tiles_to, shard_bounds


def test_shard_bounds_cover_and_align():
    for count in [0, 1, 63, 64, 65, 1000, 1 << 20, 100_000_001]:
        for world in [1, 2, 3, 4, 8]:
            spans = [shard_bounds(count, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == count
            for (a0, a1), (b0, b1) in zip(spans, spans[1:]):
                assert a1 == b0
            for (s, e), (s2, e2) in zip(spans, spans[1:]):
                if e2 > s2:  # every shard followed by a non-empty one is whole tiles
                    assert s % WAVE == 0 and (e - s) % WAVE == 0
            sizes = [e - s for s, e in spans]
            assert max(sizes) - min(sizes) < 2 * WAVE  # one tile of imbalance + a partial last tile


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, count, L, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # full vector: element e, limb j = e * 1000 + j (tile-major)
        full = torch.arange(count, dtype=torch.int64)
        s, e = shard_bounds(count, rank, world)
        n = e - s
        nt = (n + WAVE - 1) // WAVE
        C = torch.zeros((nt, L, WAVE), dtype=torch.int32)
        sign = torch.zeros(nt * WAVE, dtype=torch.uint8)
        exp = torch.zeros(nt * WAVE, dtype=torch.int32)
        for k in range(n):
            g = s + k
            C[k // WAVE, :, k % WAVE] = torch.tensor([g * 1000 + j for j in range(L)], dtype=torch.int32)
            sign[k] = g % 2
            exp[k] = -(g % 7)
        def check(Cg, sg, eg, total):
            ok = total == count and sg.dtype == torch.uint8  # one byte of sign per element on the wire
            for g in range(count):
                ok &= bool(torch.equal(Cg[g // WAVE, :, g % WAVE],
                                       torch.tensor([g * 1000 + j for j in range(L)], dtype=torch.int32)))
                ok &= int(sg[g]) == g % 2 and int(eg[g]) == -(g % 7)
            return ok

        ok = check(*gather_tiles(C, sign, exp, n))
        # the gather onto one rank (the federation sender): the full vector there, None elsewhere
        for dst in range(world):
            got = gather_tiles_to(C, sign, exp, n, dst)
            ok &= (got is None) if rank != dst else check(*got)
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


def _run(target, world, *args, timeout=300):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, *args, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = dict(q.get(timeout=timeout) for _ in range(world))
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    return res


@pytest.mark.parametrize("world,count", [(2, 200), (4, 333), (8, 200), (8, 1000)])
def test_gather_tiles(world, count):
    """The all-gather and the gather onto each rank in turn.  Ragged shards: 200 elements at
    world 2 are 128 + 72 (a partial last tile); at world 8 they are 4 tiles over 8 ranks, so
    four ranks hold nothing; 333 at world 4 and 1000 at world 8 end in partial tiles."""
    L = 5
    res = _run(_worker, world, count, L)
    assert res == {r: True for r in range(world)}


def test_compact_gathered_ragged_and_whole_tiles():
    """The receiving side of the all-gather: per-rank padded shards -> one vector in rank
    order, for whole-tile shards (tile concatenation) and ragged ones (element gather)."""
    g = torch.Generator().manual_seed(3)
    L = 3
    for counts in ([128, 128, 70], [128, 64, 0], [70, 5, 64], [0, 33, 64], [64], [10]):
        world, nt_max = len(counts), max((c + WAVE - 1) // WAVE for c in counts)
        full = [torch.randint(0, 1000, (c, L), generator=g, dtype=torch.int32) for c in counts]
        Cg = torch.zeros((world * nt_max, L, WAVE), dtype=torch.int32)
        sg = torch.zeros(world * nt_max * WAVE, dtype=torch.uint8)
        eg = torch.zeros(world * nt_max * WAVE, dtype=torch.int32)
        for r, rows in enumerate(full):
            for k in range(rows.shape[0]):
                Cg[r * nt_max + k // WAVE, :, k % WAVE] = rows[k]
                sg[r * nt_max * WAVE + k] = (r + k) % 2
                eg[r * nt_max * WAVE + k] = -(r * 7 + k)
        C2, s2, e2, tot = compact_gathered(Cg, sg, eg, counts)
        assert tot == sum(counts)
        got = C2.permute(0, 2, 1).reshape(-1, L)[:tot]
        assert torch.equal(got, torch.cat(full))
        assert s2[:tot].tolist() == [(r + k) % 2 for r, c in enumerate(counts) for k in range(c)]
        assert e2[:tot].tolist() == [-(r * 7 + k) for r, c in enumerate(counts) for k in range(c)]


def _fold_worker(rank, world, port, q):
    """Each rank holds its partial histogram (m slots of ciphertexts, tile-major CPU layout);
    the shards are all-gathered (gather_tiles) and every rank folds slot j over the ranks with
    Ciphertext::add (the oracle's; bench.py does the same on the device with k_add27)."""
    import json
    import random

    from oracle import paillier_oracle as O
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        here = os.path.dirname(os.path.abspath(__file__))
        fx = json.load(open(os.path.join(here, "golden", "paillier_1024.json")))
        osk, opk = O.keypair_from_primes(int(fx["p"], 16), int(fx["q"], 16))
        m, L = 70, 64  # 70 slots: a partial last tile per rank
        rng = random.Random(1000 + rank)
        part = []
        for j in range(m):  # signed ciphertexts, mixed exponents, a literal 1 now and then
            c = rng.randrange(2, opk.ns)
            part.append(O.ct_zero() if rng.random() < 0.1 else
                        O.Ciphertext(-c if rng.random() < 0.4 else c, rng.choice([0, -1, -13, -14])))
        nt = (m + WAVE - 1) // WAVE
        C = torch.zeros((nt, L, WAVE), dtype=torch.int32)
        sign = torch.zeros(nt * WAVE, dtype=torch.uint8)
        exp = torch.zeros(nt * WAVE, dtype=torch.int32)
        for k, ct in enumerate(part):
            canon = ct.c + opk.ns if ct.c < 0 else ct.c
            words = [(canon >> (32 * w)) & 0xFFFFFFFF for w in range(L)]
            C[k // WAVE, :, k % WAVE] = torch.tensor(words, dtype=torch.int64).to(torch.int32)
            sign[k] = 1 if ct.c < 0 else 0
            exp[k] = ct.exp
        Cg, sg, eg, total = gather_tiles(C, sign, exp, m)
        assert total == world * m

        def elem(g):
            words = Cg[g // WAVE, :, g % WAVE].to(torch.int64) & 0xFFFFFFFF
            v = sum(int(w) << (32 * i) for i, w in enumerate(words.tolist()))
            return O.Ciphertext(v - opk.ns if (int(sg[g]) and v) else v, int(eg[g]))

        folded = []
        for j in range(m):
            acc = elem(j)
            for r in range(1, world):
                acc = O.ct_add(opk, acc, elem(r * m + j))
            folded.append((acc.c, acc.exp))
        # every rank's partials, rebuilt from the same seeds, folded in a different order
        want = []
        parts = []
        for r in range(world):
            rr = random.Random(1000 + r)
            pr = []
            for j in range(m):
                c = rr.randrange(2, opk.ns)
                pr.append(O.ct_zero() if rr.random() < 0.1 else
                          O.Ciphertext(-c if rr.random() < 0.4 else c, rr.choice([0, -1, -13, -14])))
            parts.append(pr)
        for j in range(m):
            acc = O.ct_zero()
            for r in reversed(range(world)):
                acc = O.ct_add(opk, acc, parts[r][j])
            want.append((acc.c, acc.exp))
        q.put((rank, folded == want))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_cross_rank_ciphertext_fold(world):
    """SecureBoost's histogram across GPUs: per-rank partial folds,
    all-gathered, then folded again with ct-add; bit-exact against a fold of the same
    partials in another order -- what one rank folding every sample
    gives -- over gloo at world sizes 2, 4 and 8 (config 4's 8-way split)."""
    res = _run(_fold_worker, world)
    assert res == {r: True for r in range(world)}
