"""Element sharding of the PHE hot path across the GPUs of a node (one process per GPU).

Paillier encrypt / decrypt / ct-add / ct x pt are independent per element, so a tensor of
``count`` elements is split into contiguous, tile-aligned (64-element) ranges, one per rank
-- the same decomposition as the reference's ``DTensor.map_shard``
(python/fate/arch/tensor/distributed/_tensor.py:365-385), with GPUs instead of computing
partitions.  The only exchange step is the optional gather of the ciphertext shards when
the consumer needs the whole vector in one place: onto one rank (the federation sender,
:func:`gather_tiles_to`, point-to-point) or onto every rank (:func:`gather_tiles`, one
``all_gather_into_tensor`` of the byte-packed tiles per component), over RCCL/xGMI on GPUs
(backend "nccl") or gloo on CPU.  Reductions across ranks are gather-then-modmul
(RCCL has no modular-product reduce), as the reference's ``map_reduce_shard(..., add)``
(_tensor.py:387-395) reduces per-partition partials; ciphertext folds are order independent
(SURVEY.md §0 fact 3), so that stays bit-exact.
"""
from __future__ import annotations

from typing import List, Tuple

import torch

WAVE = 64


def shard_bounds(count: int, rank: int, world: int) -> Tuple[int, int]:
    """[start, end) of rank's elements: contiguous, 64-aligned (whole tiles), balanced."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    tiles = (count + WAVE - 1) // WAVE
    base, extra = divmod(tiles, world)
    t0 = rank * base + min(rank, extra)
    t1 = t0 + base + (1 if rank < extra else 0)
    return min(t0 * WAVE, count), min(t1 * WAVE, count)


def _pad_tiles(t: torch.Tensor, nt: int) -> torch.Tensor:
    if t.shape[0] == nt:
        return t.contiguous()
    out = t.new_zeros((nt,) + tuple(t.shape[1:]))
    out[: t.shape[0]] = t[:nt]
    return out


def _pad_flat(t: torch.Tensor, n: int) -> torch.Tensor:
    if t.shape[0] == n:
        return t.contiguous()
    out = t.new_zeros(n)
    m = min(n, t.shape[0])
    out[:m] = t[:m]
    return out


def compact_gathered(Cg: torch.Tensor, sg: torch.Tensor, eg: torch.Tensor, counts: List[int]):
    """The gathered, per-rank padded shards (rank r's shard at tiles [r * nt_max, ...)) as
    one vector, elements in rank order.  Returns (C, sign, exp, total).  Whole-tile shards
    (shard_bounds) are concatenated tile by tile; ragged shards (e.g. per-rank partial
    histograms of any slot count) by an element gather of the valid slots."""
    world = len(counts)
    nt_max = Cg.shape[0] // max(world, 1)
    L = Cg.shape[1]
    dev = Cg.device
    total = sum(counts)
    if all(c == nt_max * WAVE for c in counts[:-1]) and (counts[-1] + WAVE - 1) // WAVE == nt_max:
        return Cg, sg, eg, total  # no padding tiles (only the last shard's own partial tile)
    if all(c % WAVE == 0 for c in counts[:-1]):
        Cs, ss, es = [], [], []
        for r, c in enumerate(counts):
            nt = (c + WAVE - 1) // WAVE
            Cs.append(Cg[r * nt_max: r * nt_max + nt])
            ss.append(sg[r * nt_max * WAVE: r * nt_max * WAVE + nt * WAVE])
            es.append(eg[r * nt_max * WAVE: r * nt_max * WAVE + nt * WAVE])
        return torch.cat(Cs), torch.cat(ss), torch.cat(es), total
    # ragged: rank r's element k sits at r * nt_max * 64 + k of the gathered tiles
    idx = torch.cat([torch.arange(c, device=dev) + r * nt_max * WAVE for r, c in enumerate(counts)])
    rows = Cg.permute(0, 2, 1).reshape(-1, L)[idx]
    nt = (total + WAVE - 1) // WAVE
    Cf = rows.new_zeros((nt * WAVE, L))
    Cf[:total] = rows
    sf = sg.new_zeros(nt * WAVE)
    sf[:total] = sg[idx]
    ef = eg.new_zeros(nt * WAVE)
    ef[:total] = eg[idx]
    return Cf.view(nt, WAVE, L).permute(0, 2, 1).contiguous(), sf, ef, total


def gather_tiles(C: torch.Tensor, sign: torch.Tensor, exp: torch.Tensor, count: int, group=None,
                 trim: bool = True):
    """All-gather the per-rank shards (tile-major C [nt, L, 64], sign uint8 / exp int32
    [nt*64]) into the full vector on every rank, elements in rank order: three
    ``all_gather_into_tensor`` calls (limbs, one byte of sign, exponent per element) over
    RCCL on GPU tensors.  Shards are padded to the largest shard for the collective and, with
    ``trim``, the padding is cut out after (:func:`compact_gathered`).  Returns (C, sign, exp,
    total_count); with ``trim=False`` the padded buffers as gathered ([world * nt_max] tiles)
    and the per-rank counts instead of the total."""
    import torch.distributed as dist

    world = dist.get_world_size(group)
    dev = C.device
    cnt = torch.tensor([count], dtype=torch.int64, device=dev)
    counts = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(counts, cnt, group=group)
    counts = [int(c.item()) for c in counts]
    nt_max = max((c + WAVE - 1) // WAVE for c in counts) if counts else 0
    L = C.shape[1]
    Cg = torch.empty((world * nt_max, L, WAVE), dtype=C.dtype, device=dev)
    dist.all_gather_into_tensor(Cg, _pad_tiles(C, nt_max), group=group)
    sg = torch.empty(world * nt_max * WAVE, dtype=torch.uint8, device=dev)
    dist.all_gather_into_tensor(sg, _pad_flat(sign.to(torch.uint8), nt_max * WAVE), group=group)
    eg = torch.empty(world * nt_max * WAVE, dtype=exp.dtype, device=dev)
    dist.all_gather_into_tensor(eg, _pad_flat(exp, nt_max * WAVE), group=group)
    if not trim:
        return Cg, sg, eg, counts
    return compact_gathered(Cg, sg, eg, counts)


def gather_tiles_to(C: torch.Tensor, sign: torch.Tensor, exp: torch.Tensor, count: int, dst: int = 0, group=None,
                    trim: bool = True):
    """Gather the per-rank shards onto rank ``dst`` only -- the federation sender's case
    (one party process sends the whole ciphertext vector), where an
    all-gather would put every rank's copy of the vector in every GPU's HBM (52 GB per rank for
    BASELINE config 5's 100M elements at 2048 bits).  Point-to-point over RCCL/xGMI: each other
    rank sends its padded shard's three components, rank ``dst`` receives them straight into
    one buffer (rank r's shard at tiles [r * nt_max, ...)) and compacts it as
    :func:`gather_tiles` does.  The shard counts travel in one small all-gather first.  Returns
    (C, sign, exp, total) on ``dst`` (with ``trim=False`` the padded buffers and the per-rank
    counts) and None on every other rank."""
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = C.device
    cnt = torch.tensor([count], dtype=torch.int64, device=dev)
    counts = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(counts, cnt, group=group)
    counts = [int(c.item()) for c in counts]
    nt_max = max((c + WAVE - 1) // WAVE for c in counts) if counts else 0
    L = C.shape[1]
    mine = (_pad_tiles(C, nt_max), _pad_flat(sign.to(torch.uint8), nt_max * WAVE), _pad_flat(exp, nt_max * WAVE))
    # gloo's point-to-point takes host tensors only (the CPU tests, and bench.py's gloo
    # rehearsal of several ranks on one GPU); RCCL moves the device buffers directly
    host = dist.get_backend(group) == "gloo"
    if host:
        mine = tuple(t.cpu() for t in mine)
    if rank != dst:
        for t in mine:
            dist.send(t, dst, group=group)
        return None
    bdev = torch.device("cpu") if host else dev
    Cg = torch.empty((world * nt_max, L, WAVE), dtype=C.dtype, device=bdev)
    sg = torch.empty(world * nt_max * WAVE, dtype=torch.uint8, device=bdev)
    eg = torch.empty(world * nt_max * WAVE, dtype=exp.dtype, device=bdev)
    outs = (Cg, sg, eg)
    per = (nt_max, nt_max * WAVE, nt_max * WAVE)
    reqs = []
    for r in range(world):
        for buf, k, t in zip(outs, per, mine):
            view = buf[r * k:(r + 1) * k]
            if r == rank:
                view.copy_(t)
            else:
                reqs.append(dist.irecv(view, r, group=group))
    for q in reqs:
        q.wait()
    if host:
        Cg, sg, eg = Cg.to(dev), sg.to(dev), eg.to(dev)
    if not trim:
        return Cg, sg, eg, counts
    return compact_gathered(Cg, sg, eg, counts)


def gather_ciphertexts(cv, group=None, dst=None):
    """Gather a sharded ``fate_amd.paillier.CiphertextVector`` (every shard but the last must be
    whole tiles, as produced by :func:`shard_bounds`): onto every rank (``dst`` None: the
    all-gather) or onto rank ``dst`` only (None returned elsewhere).  The key stamp travels."""
    from .paillier import CiphertextVector

    if dst is None:
        C, s, e, n = gather_tiles(cv.C, cv.sign, cv.exp, cv.count, group)
    else:
        got = gather_tiles_to(cv.C, cv.sign, cv.exp, cv.count, dst, group)
        if got is None:
            return None
        C, s, e, n = got
    return CiphertextVector(C, s, e, n, cv.n, cv.raw)


def fold_partials(pk, parts, nparts: int, m: int):
    """Fold ``nparts`` partial vectors of ``m`` slots each, laid end to end in ``parts`` (part
    r's slot j at r * m + j): out[j] = add(... add(parts[j], parts[m + j]) ...), with the
    device segmented fold (the same path as iupdate), bit-exact with the sequential ct-add
    chain by the order independence of the fold."""
    from .paillier import _fold_to_segments

    dev = parts.device
    if nparts == 1:
        return parts.slice(0, m)
    seg = torch.arange(nparts * m, device=dev) % m
    return _fold_to_segments(pk, parts, seg, m)


def fold_across_ranks(pk, hist, group=None):
    """BASELINE config 4 across GPUs: every rank folded its own samples
    into ``hist`` (m slots); the partial histograms are all-gathered over RCCL and folded
    slot by slot, in rank order, on every rank.  Returns (folded vector, gather seconds,
    fold seconds)."""
    import time

    import torch.distributed as dist

    from .paillier import CiphertextVector

    dev = hist.device
    world = dist.get_world_size(group)
    torch.cuda.synchronize(dev) if dev.type == "cuda" else None
    t0 = time.perf_counter()
    Cg, sg, eg, total = gather_tiles(hist.C, hist.sign, hist.exp, hist.count, group)
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    if total != world * hist.count:
        raise ValueError("fold_across_ranks: every rank must hold the same number of slots")
    folded = fold_partials(pk, CiphertextVector(Cg, sg, eg, total, pk.n), world, hist.count)
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    return folded, t1 - t0, time.perf_counter() - t1
