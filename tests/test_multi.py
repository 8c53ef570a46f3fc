"""Multi-rank path on CPU: world_size-2 gloo process group, byte-balanced shards + all-gather.

On MI355X the same code runs one process per GPU over RCCL (bench.py --gpus N);
here the per-rank compute is libambrycrc's host primitive, so the sharding,
padding and gather logic is what is under test."""
import bisect
import os
import socket
import zlib

import numpy as np
import pytest
import torch.multiprocessing as mp

from datagen import stream_bytes


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_by_bytes_covers_everything():
    from ambry_amd.multi import shard_by_bytes

    rng = np.random.default_rng(0)
    for world in (1, 2, 3, 8):
        for n in (0, 1, 5, 100):
            lens = rng.integers(0, 1 << 20, size=n)
            shards = shard_by_bytes(lens, world)
            assert shards[0][0] == 0 and shards[-1][1] == n
            for (a, b), (c, d) in zip(shards, shards[1:]):
                assert b == c and a <= b
            if n >= world * 4 and lens.sum() > 0:
                per = [int(lens[a:b].sum()) for a, b in shards]
                assert max(per) - min(per) <= 2 * int(lens.max())
    assert shard_by_bytes([0, 0, 0, 0], 2) == [(0, 2), (2, 4)]


def _ref_shard_by_bytes(lengths, world):
    """The cut rule, stated independently for the test: rank r takes the chunks whose start byte s
    satisfies r/world <= s/total < (r+1)/world (exact integers); an all-empty batch splits by count."""
    lengths = np.asarray(lengths, dtype=object)
    n = len(lengths)
    starts, acc = [], 0
    for x in lengths:
        starts.append(acc)
        acc += int(x)
    total = acc
    scaled = [s * world for s in starts]
    bounds = []
    for r in range(world):
        bounds.append((n * r) // world if total == 0 else bisect.bisect_left(scaled, total * r))
    bounds.append(n)
    return [(bounds[r], bounds[r + 1]) for r in range(world)]


def test_shard_by_bytes_matches_rule(ambry):
    """ambrycrc_shard_by_bytes (used by ambrycrc_batch_multi, ambrycrc_batch_cpu, bench.py's
    multi-GPU shards and ambry_amd.multi) against the rule restated above, including chunks that
    start exactly on a shard boundary and totals past 2^32."""
    from ambry_amd import device as D

    shard_by_bytes = _ref_shard_by_bytes
    rng = np.random.default_rng(11)
    cases = [[4] * 8, [4] * 9, [0, 0, 0], [], [1], [0, 5, 0, 5, 0], [1 << 40, 1, 1, 1 << 40],
             [4 << 20] * 65536, [3, 3, 3, 3, 3, 3, 3]]
    cases += [rng.integers(0, 1 << 22, size=int(rng.integers(1, 3000))).tolist() for _ in range(30)]
    cases += [(rng.integers(0, 4, size=40) * 1024).tolist() for _ in range(30)]  # ties on boundaries
    for lens in cases:
        for world in (1, 2, 3, 4, 7, 8, 16):
            assert D.shard_by_bytes(lens, world) == shard_by_bytes(lens, world), (lens[:10], world)


def test_gather_layout_index_math(ambry):
    """Segment width, in-place case and compaction offsets of the CRC all-gather: the C arithmetic
    ambrycrc_batch_dev_multi / _gather run (ambrycrc_gather_layout), through ctypes."""
    from ambry_amd.multi import gather_layout

    assert gather_layout([64, 64, 64]) == (64, True, [0, 64, 128, 192])
    assert gather_layout([8192] * 8)[:2] == (8192, True)
    assert gather_layout([65536] * 8)[:2] == (65536, True)
    w, inplace, starts = gather_layout([5, 0, 70, 64])
    assert (w, inplace, starts) == (128, False, [0, 5, 5, 75, 139])
    assert gather_layout([0, 0]) == (0, False, [0, 0, 0])
    assert gather_layout([1]) == (64, False, [0, 1])
    # the padded buffer holds world*width CRCs; each rank's segment fits its width
    rng = np.random.default_rng(3)
    for _ in range(100):
        counts = rng.integers(0, 300, size=int(rng.integers(1, 9))).tolist()
        w, inplace, starts = gather_layout(counts)
        assert w % 64 == 0 and w >= max(counts) and w - max(counts) < 64
        assert starts[-1] == sum(counts)
        assert starts == [0] + np.cumsum(counts).tolist()
        assert inplace == (w > 0 and all(c == w for c in counts))


def test_gather_compact_host(ambry):
    """ambrycrc_gather_compact_host runs the device path's copy list on host memory: rank r's
    segment [r*width, r*width + counts[r]) of the padded buffer lands at starts[r]; the in-place
    layout is the identity."""
    from ambry_amd.multi import gather_compact, gather_layout

    rng = np.random.default_rng(4)
    for trial in range(100):
        counts = rng.integers(0, 300, size=int(rng.integers(1, 9))).tolist()
        if trial % 10 == 0:
            counts = [128] * len(counts)
        w, inplace, starts = gather_layout(counts)
        padded = rng.integers(0, 1 << 32, size=max(w, 1) * len(counts), dtype=np.uint64).astype(np.uint32)
        got = gather_compact(padded, counts)
        exp = np.concatenate([padded[r * w:r * w + c] for r, c in enumerate(counts)] + [np.zeros(0, np.uint32)])
        assert np.array_equal(got, exp), counts
        if inplace:
            assert np.array_equal(got, padded[:sum(counts)])


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ambry_amd.crc32 import crc32
        from ambry_amd.multi import distributed_batch, distributed_blob_crc

        mem = stream_bytes(77, 0, 3 << 20).tobytes()
        rng = np.random.default_rng(5)
        n = 37
        lens = rng.integers(0, 200000, size=n)
        lens[3] = 0
        offs = rng.integers(0, (3 << 20) - 200000, size=n)

        def compute(lo, hi):
            vals = [crc32(mem[offs[i]:offs[i] + lens[i]]) for i in range(lo, hi)]
            return torch.tensor(np.asarray(vals, dtype=np.uint32).view(np.int32), dtype=torch.int32)

        crcs, (lo, hi) = distributed_batch(lens, compute, dist)
        got = crcs.numpy().view(np.uint32).tolist()

        def blob_range(a, b):
            return crc32(mem[a:b])

        blob = distributed_blob_crc(len(mem), blob_range, dist)
        q.put((rank, got, (lo, hi), blob))
    except Exception:  # report instead of leaving the parent waiting on the queue
        import traceback

        q.put((rank, "error", traceback.format_exc(), None))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_gloo_distributed_batch_and_blob(world, ambry):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for r in res:
        assert r[1] != "error", r[2]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    mem = stream_bytes(77, 0, 3 << 20).tobytes()
    rng = np.random.default_rng(5)
    n = 37
    lens = rng.integers(0, 200000, size=n)
    lens[3] = 0
    offs = rng.integers(0, (3 << 20) - 200000, size=n)
    exp = [zlib.crc32(mem[offs[i]:offs[i] + lens[i]]) for i in range(n)]
    ranges = sorted(r[2] for r in res)
    assert ranges[0][0] == 0 and ranges[-1][1] == n and ranges[0][1] == ranges[1][0]
    for rank, got, _, blob in res:
        assert got == exp, rank
        assert blob == zlib.crc32(mem)
