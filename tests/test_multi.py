"""Multi-rank path on CPU: world_size-2 gloo process group, byte-balanced shards + all-gather.

On MI355X the same code runs one process per GPU over RCCL (bench.py --gpus N);
here the per-rank compute is libambrycrc's host primitive, so the sharding,
padding and gather logic is what is under test."""
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
