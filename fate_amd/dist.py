"""Element sharding of the PHE hot path across the GPUs of a node (one process per GPU).

Paillier encrypt / decrypt / ct-add / ct x pt are independent per element, so a tensor of
``count`` elements is split into contiguous, tile-aligned (64-element) ranges, one per rank
-- the same decomposition as the reference's ``DTensor.map_shard``
(python/fate/arch/tensor/distributed/_tensor.py:365-385), with GPUs instead of computing
partitions.  The only exchange step is the optional all-gather of the ciphertext shards
when the consumer needs the whole vector in one place (e.g. the federation sender on rank
0): one ``all_gather_into_tensor`` of the byte-packed tiles per component, over RCCL/xGMI
on GPUs (backend "nccl") or gloo on CPU.  Reductions across ranks would be gather-then-
modmul (RCCL has no modular-product reduce); ciphertext reductions are order independent
(SURVEY.md §0 fact 3), so that stays bit-exact.
"""
from __future__ import annotations

from typing import Tuple

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


def gather_tiles(C: torch.Tensor, sign: torch.Tensor, exp: torch.Tensor, count: int, group=None,
                 trim: bool = True):
    """All-gather the per-rank shards (tile-major C [nt, L, 64], sign/exp [nt*64]) into the
    full vector on every rank, elements in rank order.  Shards are padded to the largest
    shard for the collective and, with ``trim``, the padding is cut out after (one copy of
    the gathered vector; ragged shards by an element gather).  Returns (C, sign, exp, total_count); with ``trim=False`` the padded buffers
    as gathered ([world * nt_max] tiles, rank r's shard at tiles [r * nt_max, ...)) and the
    per-rank counts instead of the total."""
    import torch.distributed as dist

    world = dist.get_world_size(group)
    dev = C.device
    cnt = torch.tensor([count], dtype=torch.int64, device=dev)
    counts = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(counts, cnt, group=group)
    counts = [int(c.item()) for c in counts]
    nt_max = max((c + WAVE - 1) // WAVE for c in counts) if counts else 0
    L = C.shape[1]

    def pad_tiles(t: torch.Tensor) -> torch.Tensor:
        if t.shape[0] == nt_max:
            return t.contiguous()
        out = t.new_zeros((nt_max,) + tuple(t.shape[1:]))
        out[: t.shape[0]] = t
        return out

    def pad_flat(t: torch.Tensor) -> torch.Tensor:
        n = nt_max * WAVE
        if t.shape[0] == n:
            return t.contiguous()
        out = t.new_zeros(n)
        out[: t.shape[0]] = t
        return out

    Cg = torch.empty((world * nt_max, L, WAVE), dtype=C.dtype, device=dev)
    dist.all_gather_into_tensor(Cg, pad_tiles(C), group=group)
    # sign is uint8: gather as int32 for backend portability (gloo lacks uint8 on some builds)
    sg = torch.empty(world * nt_max * WAVE, dtype=torch.int32, device=dev)
    dist.all_gather_into_tensor(sg, pad_flat(sign.to(torch.int32)), group=group)
    eg = torch.empty(world * nt_max * WAVE, dtype=exp.dtype, device=dev)
    dist.all_gather_into_tensor(eg, pad_flat(exp), group=group)
    if not trim:
        return Cg, sg, eg, counts
    total = sum(counts)
    if all(c == nt_max * WAVE for c in counts[:-1]) and (counts[-1] + WAVE - 1) // WAVE == nt_max:
        # no padding tiles (only the last shard's partial tile, which is the vector's end)
        return Cg, sg.to(torch.uint8), eg, total
    if all(c % WAVE == 0 for c in counts[:-1]):
        # whole-tile shards (shard_bounds): drop the per-rank padding tiles
        Cs, ss, es = [], [], []
        for r, c in enumerate(counts):
            nt = (c + WAVE - 1) // WAVE
            Cs.append(Cg[r * nt_max: r * nt_max + nt])
            ss.append(sg[r * nt_max * WAVE: r * nt_max * WAVE + nt * WAVE])
            es.append(eg[r * nt_max * WAVE: r * nt_max * WAVE + nt * WAVE])
        return torch.cat(Cs), torch.cat(ss).to(torch.uint8), torch.cat(es), total
    # ragged shards (e.g. per-rank partial histograms of any slot count): element gather of
    # the valid slots, rank r's element k sitting at r * nt_max * 64 + k of the gathered tiles
    idx = torch.cat([torch.arange(c, device=dev) + r * nt_max * WAVE for r, c in enumerate(counts)])
    rows = Cg.permute(0, 2, 1).reshape(-1, L)[idx]
    nt = (total + WAVE - 1) // WAVE
    Cf = rows.new_zeros((nt * WAVE, L))
    Cf[:total] = rows
    sf = sg.new_zeros(nt * WAVE)
    sf[:total] = sg[idx]
    ef = eg.new_zeros(nt * WAVE)
    ef[:total] = eg[idx]
    return Cf.view(nt, WAVE, L).permute(0, 2, 1).contiguous(), sf.to(torch.uint8), ef, total


def gather_ciphertexts(cv, group=None):
    """All-gather a sharded ``fate_amd.paillier.CiphertextVector`` (every shard but the last
    must be whole tiles, as produced by :func:`shard_bounds`)."""
    from .paillier import CiphertextVector

    C, s, e, n = gather_tiles(cv.C, cv.sign, cv.exp, cv.count, group)
    return CiphertextVector(C, s, e, n)
