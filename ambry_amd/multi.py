"""One-process-per-GPU sharding of a CRC batch, with the 4-byte results exchanged by all-gather.

The batch path shards trivially: chunk CRCs are independent, so
rank r computes a contiguous block of chunks balanced by bytes and the only
exchange is one all-gather of uint32 CRCs (RCCL over xGMI on MI355X; gloo in
the CPU tests). A single blob larger than one GPU is split by byte range and
the per-rank CRCs are folded with the GF(2) combine after an all-gather of
(crc, length) pairs. There is no Ambry counterpart: the reference never splits
one blob's CRC across workers (CrcInputStream streams it serially).
"""
from __future__ import annotations

from typing import Callable, Sequence

import numpy as np

from .crc32 import combine


def shard_by_bytes(lengths: Sequence[int], world: int) -> list[tuple[int, int]]:
    """Contiguous chunk ranges [lo, hi) per rank with near-equal byte totals.

    Rank r takes the chunks whose start byte s satisfies r/world <= s/total < (r+1)/world
    (exact rational comparison, the rule of ambrycrc_shard_by_bytes in the C ABI, which
    tests/test_multi.py checks this against). Every chunk belongs to exactly one rank; ranks
    may be empty when n < world; an all-empty batch is split by count.
    """
    lengths = np.asarray(lengths, dtype=np.int64)
    n = len(lengths)
    starts = np.concatenate([[0], np.cumsum(lengths)[:-1]]) if n else np.zeros(0, dtype=np.int64)
    total = int(lengths.sum()) if n else 0
    bounds = []
    for r in range(world + 1):
        if r == world:
            bounds.append(n)
        elif total == 0:
            bounds.append((n * r) // world)  # all-empty batch: split by count
        else:
            bounds.append(int(np.searchsorted(starts * world, total * r, side="left")))
    return [(bounds[r], bounds[r + 1]) for r in range(world)]


SEG_ALIGN = 64  # CRCs per gather-segment quantum (256 B), as ambrycrc_multi.cpp kSegAlign


def gather_layout(counts: Sequence[int]):
    """Layout of the all-gather of per-rank CRCs, the rule ambrycrc_batch_dev_multi/_gather
    use (ambrycrc_multi.cpp seg_width/enqueue_gather): every rank sends a segment of `width`
    CRCs (the largest shard rounded up to 64); when every shard has exactly `width` chunks the
    gather lands in place, otherwise rank r's CRCs are compacted from [r*width, r*width+counts[r])
    to [starts[r], starts[r+1]). Returns (width, in_place, starts)."""
    counts = [int(c) for c in counts]
    width = -(-max(counts, default=0) // SEG_ALIGN) * SEG_ALIGN
    starts = [0]
    for c in counts:
        starts.append(starts[-1] + c)
    return width, width > 0 and all(c == width for c in counts), starts


def gather_crcs(local, lo: int, hi: int, n: int, shards, dist, group=None, device=None):
    """All-gather each rank's CRCs (int32 tensor of hi-lo) into the full int32[n] on every rank."""
    import torch

    world = len(shards)
    width, in_place, starts = gather_layout([h - l for l, h in shards])
    dev = local.device if device is None else device
    seg = max(width, 1)
    padded = torch.zeros(seg, dtype=torch.int32, device=dev)
    if hi > lo:
        padded[: hi - lo] = local
    gathered = torch.empty(world * seg, dtype=torch.int32, device=dev)
    dist.all_gather_into_tensor(gathered, padded, group=group)
    if in_place:
        out = gathered[:n]
    else:
        out = torch.empty(n, dtype=torch.int32, device=dev)
        for r, (l, h) in enumerate(shards):
            out[starts[r]:starts[r + 1]] = gathered[r * seg: r * seg + (h - l)]
    assert out.numel() == n
    return out


def distributed_batch(lengths: Sequence[int], compute: Callable[[int, int], "object"], dist, group=None,
                      device=None):
    """Shard chunks by bytes, run `compute(lo, hi)` (-> int32 tensor of hi-lo CRCs) on this rank, all-gather.

    Returns (all CRCs as int32[n] tensor, (lo, hi) of this rank).
    """
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    shards = shard_by_bytes(lengths, world)
    lo, hi = shards[rank]
    local = compute(lo, hi)
    return gather_crcs(local, lo, hi, len(lengths), shards, dist, group=group, device=device), (lo, hi)


def split_blob(total: int, world: int) -> list[tuple[int, int]]:
    """Byte ranges [a, b) of one blob per rank (equal sizes, 16-B aligned cuts)."""
    cuts = [min(total, ((total * r) // world + 15) & ~15) for r in range(world)] + [total]
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


def distributed_blob_crc(total: int, compute_range: Callable[[int, int], int], dist, group=None, device=None):
    """CRC of one blob split across ranks: local crc32 of [a, b), all-gather (crc, len), GF(2) fold."""
    import torch

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    a, b = split_blob(total, world)[rank]
    crc = compute_range(a, b) & 0xFFFFFFFF
    mine = torch.tensor([crc, b - a], dtype=torch.int64, device=device)
    allv = torch.empty(2 * world, dtype=torch.int64, device=device)
    dist.all_gather_into_tensor(allv, mine, group=group)
    vals = allv.cpu().tolist()
    acc = 0
    for r in range(world):
        acc = combine(acc, vals[2 * r], vals[2 * r + 1])
    return acc
