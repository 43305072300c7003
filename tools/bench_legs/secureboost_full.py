"""BASELINE config 4 at its full size: the SecureBoost histogram over 10M samples, 10 features
x 32 bins, 1 node (320 slots), 2048-bit key, sharded over the ranks
(each takes a contiguous tile-aligned slice of the samples, fate_amd.dist.shard_bounds).

  (i)  unpacked (the reference's gh_pack=False, guest.py:245-246): g and h encrypted as
       separate float32 ciphertexts (key holder; timed and reported apart, not in the op
       rates), then timed: ct x pt by a per-sample weight w ~ U(0.5, 1.5) (GOSS-style
       stand-in, float significands, so the exponents change) and the per-bin iupdate fold
       (10M x 10 x 2 = 200M scatter-adds, with 16^d exponent alignment).  The 640 slots are
       decrypted and compared (allclose) with the float64 histogram.
  (ii) packed (the reference default): (g + 1, h) packed at precision 52 with shift_bit from
       compute_offset_bit(10M, 2, 1), 10M key-holder encryptions, the per-bin fold (100M
       adds, exponent 0), per-feature cumsum, pack_squeeze, decrypt + unpack, allclose.

With several ranks each folds its own samples and the partial histograms are all-gathered
over RCCL and folded slot by slot (fate_amd.dist.fold_across_ranks); every phase reports the
slowest rank.  bench.py runs :func:`config4` as its ``histogram_config4`` leg; standalone:

    python tools/bench_legs/secureboost_full.py [samples]
"""
import json
import math
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

HF, NB = 10, 32


def config4(P, pk, sk, coder, dev, total: int = 10_000_000, rank: int = 0, world: int = 1, iupdate_roofline=None,
            log=None) -> dict:
    """Run config 4 on this rank's shard; returns the leg's record (identical on every rank)."""
    dist = world > 1
    if dist:
        import torch.distributed as tdist
        from fate_amd.dist import fold_across_ranks, shard_bounds
        s0, s1 = shard_bounds(total, rank, world)
    else:
        s0, s1 = 0, total
    out = {"samples": total, "features": HF, "bins": NB, "ranks": world, "samples_rank0": s1 - s0}
    times = {}

    def timed(name, f):
        torch.cuda.synchronize(dev)
        if dist:
            tdist.barrier()
        t0 = time.perf_counter()
        r = f()
        torch.cuda.synchronize(dev)
        times[name] = time.perf_counter() - t0
        if log:
            log({"phase": name, "s": round(times[name], 4)})
        return r

    g0 = torch.Generator().manual_seed(20241218)
    p = torch.sigmoid(torch.randn(total, generator=g0, dtype=torch.float64))
    y = (torch.rand(total, generator=g0, dtype=torch.float64) < 0.5).double()
    g, h = (p - y).float(), (p * (1 - p)).float()
    w = (torch.rand(total, generator=g0) + 0.5).float()
    bins = torch.randint(0, NB, (total, HF), generator=g0)
    positions = bins + torch.arange(HF) * NB
    n = s1 - s0
    gs, hs, ws, pos_r = g[s0:s1], h[s0:s1], w[s0:s1], positions[s0:s1]
    # the bin indexes live in HBM like the ciphertexts (bench.py)
    positions_d = pos_r.to(dev, torch.int32)

    # (i) unpacked
    gh = torch.stack([gs, hs], 1).reshape(-1).to(dev)
    egh = timed("unpacked_encrypt_s", lambda: pk.encrypt_encoded(coder.encode_f32_vec(gh), True))
    wrep = coder.encode_f32_vec(ws.repeat_interleave(2).to(dev))
    egh.mul(pk, wrep)  # untimed: grows the context scratch to the op's size
    ew = timed("unpacked_ct_x_pt_s", lambda: egh.mul(pk, wrep))
    del egh, wrep
    # one untimed full-size pass first maps the call's stream-ordered scratch into the pool
    P.CiphertextVector.zeros(HF * NB * 2, pk._key.L2, dev).iupdate(ew, positions_d, 2, pk)
    hist = P.CiphertextVector.zeros(HF * NB * 2, pk._key.L2, dev)
    timed("unpacked_iupdate_s", lambda: hist.iupdate(ew, positions_d, 2, pk))
    if iupdate_roofline is not None:
        blk = iupdate_roofline(ew, pos_r, 2, HF * NB * 2, times["unpacked_iupdate_s"], pk.n.bit_length())
        out["unpacked_iupdate_roofline"] = {k: blk[k] for k in ("frac", "achieved", "unit", "kernel_ms", "terms",
                                                                "alignment_squarings", "scope")}
    del ew
    if dist:
        hist = timed("unpacked_cross_rank_fold_s", lambda: fold_across_ranks(pk, hist)[0])
    dec = coder.decode_f64_vec(sk.decrypt_to_encoded(hist)).cpu().reshape(HF * NB, 2)
    want = torch.zeros(HF * NB, 2, dtype=torch.float64)
    for f in range(HF):
        want[:, 0].index_add_(0, positions[:, f], g.double() * w.double())
        want[:, 1].index_add_(0, positions[:, f], h.double() * w.double())
    out["unpacked_allclose"] = bool(torch.allclose(dec, want, rtol=1e-9, atol=1e-6))
    del hist

    # (ii) packed
    shift = int(math.log2(2 ** 52 * total * 2) + 1)
    squeeze_num = (pk.n.bit_length() - 2) // (shift * 2)
    vals = torch.stack([gs.double() + 1.0, hs.double()], 1).reshape(-1).to(dev)
    pv = timed("packed_pack_s", lambda: coder.pack_floats(vals, shift, 2, 52))
    en = timed("packed_encrypt_s", lambda: pk.encrypt_encoded(pv, True))
    P.CiphertextVector.zeros(HF * NB, pk._key.L2, dev).iupdate(en, positions_d, 1, pk)
    hp = P.CiphertextVector.zeros(HF * NB, pk._key.L2, dev)
    timed("packed_iupdate_s", lambda: hp.iupdate(en, positions_d, 1, pk))
    del en
    if dist:
        hp = timed("packed_cross_rank_fold_s", lambda: fold_across_ranks(pk, hp)[0])
    timed("packed_cumsum_s", lambda: hp.chunking_cumsum_with_step(pk, [NB] * HF, 1))
    sq = timed("packed_squeeze_s", lambda: hp.pack_squeeze(squeeze_num, shift * 2, pk))
    dq = sk.decrypt_to_encoded(sq)
    got = torch.tensor(coder.unpack_floats(dq, shift, 2 * squeeze_num, 52, HF * NB * 2), dtype=torch.float64)
    wantp = torch.zeros(HF * NB, 2, dtype=torch.float64)
    for f in range(HF):
        wantp[:, 0].index_add_(0, positions[:, f], g.double() + 1.0)
        wantp[:, 1].index_add_(0, positions[:, f], h.double())
    wantp = wantp.view(HF, NB, 2).cumsum(1).reshape(-1)
    out["packed_allclose"] = bool(torch.allclose(got, wantp, rtol=1e-12, atol=1e-9))

    if dist:  # the slowest rank sets every phase
        names = sorted(times)
        tt = torch.tensor([times[k] for k in names], dtype=torch.float64, device=dev)
        tdist.all_reduce(tt, op=tdist.ReduceOp.MAX)
        times = dict(zip(names, tt.tolist()))
    out.update({k: round(v, 4) for k, v in times.items()})
    out.update({
        "packed_shift_bit": shift, "packed_squeeze_num": squeeze_num, "packed_squeezed_ciphertexts": sq.count,
        "unpacked_ct_x_pt_per_s": round(2 * total / times["unpacked_ct_x_pt_s"], 1),
        "unpacked_scatter_adds_per_s": round(total * HF * 2 / times["unpacked_iupdate_s"], 1),
        "packed_scatter_adds_per_s": round(total * HF / times["packed_iupdate_s"], 1),
        "encrypt_per_s_untimed_setup": round((2 * total + total) / (times["unpacked_encrypt_s"]
                                                                    + times["packed_encrypt_s"]), 1),
    })
    return out


if __name__ == "__main__":
    from fate_amd import paillier as P

    N = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    fx = json.load(open(os.path.join(ROOT, "tests", "golden", "paillier_2048.json")))
    sk, pk, coder = P.keypair_from_primes(int(fx["p"], 16), int(fx["q"], 16), keyholder=True)
    dev = torch.device("cuda", 0)
    print(json.dumps(config4(P, pk, sk, coder, dev, N, log=lambda d: print(json.dumps(d), flush=True))), flush=True)
