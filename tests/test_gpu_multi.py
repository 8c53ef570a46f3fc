"""Multi-GPU batch path behind the C ABI (ambrycrc_batch_dev_multi / _gather + RCCL all-gather),
on the one-GPU test box: world size 1, both communicator forms, the in-place and the padded
gather layouts, and C5's 65,536 x 4 MiB per-GPU shard (256 GiB resident, swept in 32 GiB rounds)
checked through size-independent properties. SURVEY.md §8e; BASELINE.json configs[4]."""
import numpy as np
import pytest

from datagen import stream_bytes

pytestmark = pytest.mark.gpu


def _torch():
    import torch

    return torch


def _batch(seed, n, max_len, mem_bytes=16 << 20):
    rng = np.random.default_rng(seed)
    mem = stream_bytes(seed, 0, mem_bytes)
    ln = rng.integers(0, max_len, size=n)
    off = rng.integers(0, mem_bytes - max_len, size=n)
    return mem, off, ln


def _dev(torch, mem, off, ln):
    base = torch.from_numpy(mem.copy()).cuda()
    return base, torch.from_numpy(off.astype(np.int64)).cuda(), torch.from_numpy(ln.astype(np.int64)).cuda()


@pytest.mark.parametrize("n", [64, 4096, 1, 1000, 20000])
def test_batch_dev_multi_one_device(gpu, oracle, n):
    """ncclCommInitAll over [0]; n a multiple of 64 gathers in place, other n through the padded
    scratch and the compaction copy; 20,000 chunks engage the group phase."""
    torch = _torch()
    mem, off, ln = _batch(600 + n, n, 20000 if n >= 16384 else 300000)
    base, o, l = _dev(torch, mem, off, ln)
    comm = gpu.Comm.all_devices([0])
    try:
        assert comm.size() == 1
        gathered = torch.full((n,), -1, dtype=torch.int32, device="cuda")
        gpu.crc32_batch_multi_dev(comm, [dict(base=base, off=o, len=l, gathered=gathered)])
        torch.cuda.synchronize()
    finally:
        comm.destroy()
    assert np.array_equal(gathered.cpu().numpy().view(np.uint32), oracle.batch(mem, off, ln, threads=8))


def test_batch_dev_gather_rank_form(gpu, oracle):
    """One process per GPU: unique id -> ncclCommInitRank (nranks 1) -> ambrycrc_batch_dev_gather,
    with crc_in and on a side stream; repeated calls reuse the communicator."""
    torch = _torch()
    uid = gpu.unique_id()
    assert len(uid) == 128
    comm = gpu.Comm.rank(uid, 1, 0, 0)
    try:
        s = torch.cuda.Stream()
        for it, n in enumerate((100, 128, 3)):
            mem, off, ln = _batch(700 + it, n, 200000)
            cin = np.random.default_rng(it).integers(0, 1 << 32, size=n, dtype=np.uint64).astype(np.uint32)
            base, o, l = _dev(torch, mem, off, ln)
            c = torch.from_numpy(cin.view(np.int32)).cuda()
            gathered = torch.empty(n, dtype=torch.int32, device="cuda")
            torch.cuda.synchronize()
            with torch.cuda.stream(s):
                gpu.crc32_batch_gather(comm, base, o, l, gathered, [n], crc_in=c, stream=s)
            s.synchronize()
            assert np.array_equal(gathered.cpu().numpy().view(np.uint32),
                                  oracle.batch(mem, off, ln, crc_in=cin, threads=8)), n
    finally:
        comm.destroy()


def test_padded_gather_two_streams(gpu, oracle):
    """Two padded-layout batches in flight at once on two streams (unequal counts, neither a
    multiple of 64), then the first stream again with a larger count (its scratch regrows): each
    stream has its own gather scratch, so the second batch's CRC kernel cannot overwrite the
    first's segment before its all-gather and compaction ran. Then nine more streams, past the
    per-device scratch cap (the least recently used buffer is reused after its event fired)."""
    torch = _torch()
    comm = gpu.Comm.all_devices([0])
    try:
        streams = [torch.cuda.Stream() for _ in range(2)]
        jobs = []
        for k, (n, max_len, s) in enumerate(((5000, 400000, streams[0]), (70, 3000, streams[1]),
                                             (9000, 100000, streams[0]))):
            mem, off, ln = _batch(900 + k, n, max_len, mem_bytes=32 << 20)
            base, o, l = _dev(torch, mem, off, ln)
            jobs.append((mem, off, ln, base, o, l, s))
        torch.cuda.synchronize()
        outs = []
        for mem, off, ln, base, o, l, s in jobs:  # no sync between the launches
            g = torch.full((len(off),), -1, dtype=torch.int32, device="cuda")
            with torch.cuda.stream(s):
                gpu.crc32_batch_multi_dev(comm, [dict(base=base, off=o, len=l, gathered=g, stream=s)])
            outs.append(g)
        torch.cuda.synchronize()
        for (mem, off, ln, *_), g in zip(jobs, outs):
            assert np.array_equal(g.cpu().numpy().view(np.uint32), oracle.batch(mem, off, ln, threads=8)), len(off)
        mem, off, ln = _batch(990, 333, 5000)
        base, o, l = _dev(torch, mem, off, ln)
        exp = oracle.batch(mem, off, ln, threads=8)
        extra = [torch.cuda.Stream() for _ in range(9)]
        gs = []
        for s in extra:
            g = torch.full((333,), -1, dtype=torch.int32, device="cuda")
            with torch.cuda.stream(s):
                gpu.crc32_batch_multi_dev(comm, [dict(base=base, off=o, len=l, gathered=g, stream=s)])
            gs.append(g)
        torch.cuda.synchronize()
        for g in gs:
            assert np.array_equal(g.cpu().numpy().view(np.uint32), exp)
    finally:
        comm.destroy()


def test_multi_entry_argument_checks(gpu):
    torch = _torch()
    from ambry_amd._lib import AmbryCrcError

    comm = gpu.Comm.all_devices([0])
    try:
        base = torch.zeros(64, dtype=torch.uint8, device="cuda")
        o = torch.zeros(2, dtype=torch.int64, device="cuda")
        g = torch.zeros(4, dtype=torch.int32, device="cuda")
        with pytest.raises(AmbryCrcError):  # two shards for a one-device communicator
            gpu.crc32_batch_multi_dev(comm, [dict(base=base, off=o, len=o, gathered=g)] * 2)
        with pytest.raises(AmbryCrcError):  # counts[rank] != shard size
            gpu.crc32_batch_gather(comm, base, o, o, torch.zeros(3, dtype=torch.int32, device="cuda"), [3])
    finally:
        comm.destroy()


def test_c5_shard_256gib_through_multi_entry(gpu, oracle):
    """C5's per-GPU shard: 65,536 distinct 4 MiB chunks = 256 GiB resident, through
    ambrycrc_batch_dev_multi (sweep in 32 GiB rounds, then the RCCL gather). Checked by
    size-independent properties: 24 sampled chunks against the oracle (the splitmix stream is
    regenerated on the CPU at each chunk's offset), the CRC of the whole 256 GiB region as one
    chunk equal to the GF(2) fold of the 65,536 per-chunk CRCs, and a second pass identical."""
    torch = _torch()
    from ambry_amd import combine

    n, chunk = 65536, 4 << 20
    total = n * chunk
    free, _ = torch.cuda.mem_get_info()
    if free < total + (2 << 30):
        pytest.skip(f"needs {total >> 30} GiB free HBM, {free >> 30} GiB free")
    seed = 0xC5C5C5C5
    buf = torch.empty(total, dtype=torch.uint8, device="cuda")
    gpu.fill_random(buf, seed, 0)
    o = torch.arange(n, dtype=torch.int64, device="cuda") * chunk
    l = torch.full((n,), chunk, dtype=torch.int64, device="cuda")
    comm = gpu.Comm.all_devices([0])
    try:
        gathered = torch.empty(n, dtype=torch.int32, device="cuda")
        gpu.crc32_batch_multi_dev(comm, [dict(base=buf, off=o, len=l, gathered=gathered)])
        again = torch.empty(n, dtype=torch.int32, device="cuda")
        gpu.crc32_batch_multi_dev(comm, [dict(base=buf, off=o, len=l, gathered=again)])
        whole = gpu.crc32_batch(buf, torch.zeros(1, dtype=torch.int64, device="cuda"),
                                torch.full((1,), total, dtype=torch.int64, device="cuda"))
        torch.cuda.synchronize()
    finally:
        comm.destroy()
    crcs = gathered.cpu().numpy().view(np.uint32)
    assert np.array_equal(crcs, again.cpu().numpy().view(np.uint32))
    rng = np.random.default_rng(55)
    picks = sorted(set([0, 1, n - 1, 8191, 8192, 32767, 32768] + rng.integers(0, n, size=17).tolist()))
    for i in picks:
        assert crcs[i] == oracle.crc32(stream_bytes(seed, i * chunk, chunk)), i
    acc = 0
    for v in crcs.tolist():
        acc = combine(acc, v, chunk)
    assert acc == int(whole.cpu().numpy().view(np.uint32)[0])
    del buf
    torch.cuda.empty_cache()


def test_distributed_batch_on_rccl_group(gpu, oracle):
    """ambry_amd.multi.distributed_batch on an NCCL (= RCCL) process group of world size 1 with
    device="cuda": the padded all-gather runs on device tensors (RCCL rejects CPU ones), the
    compaction in C, and the CRCs equal the oracle's (the device argument)."""
    import torch
    import torch.distributed as dist

    from ambry_amd import device as D
    from ambry_amd.multi import distributed_batch

    mem, off, ln = _batch(61, 300, 100000)
    base, d_off, d_len = _dev(torch, mem, off, ln)
    # an in-process store: world size 1 needs no rendezvous port (a probed free port can be taken
    # by another process on a shared box before the group binds it)
    dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        def compute(lo, hi):
            return D.crc32_batch(base, d_off[lo:hi].contiguous(), d_len[lo:hi].contiguous())

        crcs, (lo, hi) = distributed_batch(ln.tolist(), compute, dist, device="cuda")
        torch.cuda.synchronize()
        assert crcs.is_cuda and (lo, hi) == (0, len(ln))
        assert np.array_equal(crcs.cpu().numpy().view(np.uint32), oracle.batch(mem, off, ln))
    finally:
        dist.destroy_process_group()
