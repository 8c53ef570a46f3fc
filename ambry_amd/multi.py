"""One-process-per-GPU sharding of a CRC batch, with the 4-byte results exchanged by all-gather.

The batch path shards trivially: chunk CRCs are independent, so rank r computes
a contiguous block of chunks balanced by bytes and the only exchange is one all-gather of uint32
CRCs. On MI355X that all-gather is RCCL over xGMI inside libambrycrc (ambrycrc_batch_dev_gather);
here any torch.distributed group (gloo in the CPU tests) carries the padded segments, and every
other step is libambrycrc's own C code through ctypes -- the shard cuts
(ambrycrc_shard_by_bytes), the segment layout (ambrycrc_gather_layout) and the compaction
(ambrycrc_gather_compact_host, the copy list the device path enqueues) -- so the multi-rank CPU
tests run the arithmetic the GPU path runs, not a restatement of it.

A single blob larger than one GPU is split by byte range and the per-rank CRCs are folded with
the GF(2) combine after an all-gather of (crc, length) pairs. There is no Ambry counterpart: the
reference never splits one blob's CRC across workers (CrcInputStream streams it serially).
"""
from __future__ import annotations

import ctypes
from typing import Callable, Sequence

import numpy as np

from ._lib import check, lib
from .crc32 import combine


def shard_by_bytes(lengths: Sequence[int], world: int) -> list[tuple[int, int]]:
    """ambrycrc_shard_by_bytes: contiguous chunk ranges [lo, hi) per rank with near-equal bytes."""
    from .device import shard_by_bytes as c_shard

    return c_shard(lengths, world)


def gather_layout(counts: Sequence[int]):
    """ambrycrc_gather_layout: (width, in_place, starts) of the CRC all-gather for shard sizes
    `counts` -- every rank sends `width` CRCs, rank r's at [r*width, r*width + counts[r]); unless
    in_place they are compacted to [starts[r], starts[r+1])."""
    c = np.ascontiguousarray(np.asarray(counts, dtype=np.uint64))
    nr = len(c)
    width, in_place = ctypes.c_uint64(0), ctypes.c_int(0)
    starts = (ctypes.c_uint64 * (nr + 1))()
    check(lib().ambrycrc_gather_layout(c.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), nr, ctypes.byref(width),
                                       ctypes.byref(in_place), starts), "ambrycrc_gather_layout")
    return int(width.value), bool(in_place.value), [int(x) for x in starts]


def gather_compact(padded: np.ndarray, counts: Sequence[int]) -> np.ndarray:
    """ambrycrc_gather_compact_host: the shard-order CRC vector from the padded gather buffer."""
    c = np.ascontiguousarray(np.asarray(counts, dtype=np.uint64))
    src = np.ascontiguousarray(padded, dtype=np.uint32)
    out = np.empty(int(c.sum()), dtype=np.uint32)
    if out.size == 0:
        return out
    check(lib().ambrycrc_gather_compact_host(src.ctypes.data, c.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                                             len(c), out.ctypes.data), "ambrycrc_gather_compact_host")
    return out


def gather_crcs(local, lo: int, hi: int, n: int, shards, dist, group=None, device=None):
    """All-gather each rank's CRCs (int32 tensor of hi-lo) into the full int32[n] on every rank: the
    padded segment layout of ambrycrc_gather_layout, one all_gather_into_tensor on `device` (None:
    the CPU, for gloo; a CUDA device for an NCCL/RCCL group, which rejects CPU tensors), then the C
    compaction on the host. The result lives on `device` (CPU when None)."""
    import torch

    counts = [h - l for l, h in shards]
    world = len(shards)
    width, _, _ = gather_layout(counts)
    seg = max(width, 1)
    padded = torch.zeros(seg, dtype=torch.int32, device=device)
    if hi > lo:
        padded[: hi - lo] = local.to(padded.device)
    gathered = torch.empty(world * seg, dtype=torch.int32, device=device)
    dist.all_gather_into_tensor(gathered, padded, group=group)
    out = gather_compact(gathered.cpu().numpy().view(np.uint32), counts)
    assert out.size == n
    res = torch.from_numpy(out.view(np.int32).copy())
    return res if device is None else res.to(device)


def distributed_batch(lengths: Sequence[int], compute: Callable[[int, int], "object"], dist, group=None,
                      device=None):
    """Shard chunks by bytes, run `compute(lo, hi)` (-> int32 tensor of hi-lo CRCs) on this rank, all-gather
    (on `device`: None for a gloo group, the rank's CUDA device for NCCL/RCCL -- gather_crcs).

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
