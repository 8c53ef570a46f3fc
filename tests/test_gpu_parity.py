"""GPU parity: libambrycrc's gfx950 kernels (through the C ABI) vs the CPU oracle and golden vectors.

Bit-exact comparisons only (integer path). Full-size configs (C2, C3) are checked
through size-independent properties: per-chunk samples against the oracle, the
whole region as one chunk vs the combine-fold of the per-chunk CRCs, determinism.
"""
import ctypes

import numpy as np
import pytest

from datagen import stream_bytes, zipf_sizes

pytestmark = pytest.mark.gpu


def _torch():
    import torch

    return torch


def dev_bytes(arr: np.ndarray):
    torch = _torch()
    return torch.from_numpy(np.array(arr, dtype=np.uint8, copy=True)).cuda()


def dev_u64(vals):
    torch = _torch()
    return torch.tensor(np.asarray(vals, dtype=np.int64), dtype=torch.int64, device="cuda")


def host_u32(t):
    return t.cpu().numpy().view(np.uint32)


def run_batch(gpu, mem_np, off, ln, crc_in=None, mem_dev=None):
    torch = _torch()
    base = dev_bytes(mem_np) if mem_dev is None else mem_dev
    cin = None if crc_in is None else torch.from_numpy(np.asarray(crc_in, dtype=np.uint32).view(np.int32)).cuda()
    out = gpu.crc32_batch(base, dev_u64(off), dev_u64(ln), crc_in=cin)
    torch.cuda.synchronize()
    return host_u32(out)


def test_fill_matches_generator(gpu):
    torch = _torch()
    for n, soff in ((1 << 20, 0), (12345, 16), (17, 4096)):
        buf = torch.empty(n, dtype=torch.uint8, device="cuda")
        gpu.fill_random(buf, 0xA3B1C2D3, soff)
        torch.cuda.synchronize()
        assert np.array_equal(buf.cpu().numpy(), stream_bytes(0xA3B1C2D3, soff, n))


def test_known_answers_on_device(gpu, vectors):
    items = [bytes.fromhex(v["hex"]) for v in vectors["known_answers"] + vectors["message_headers"]]
    items += [bytes(v["len"]) for v in vectors["zero_runs"]]
    expect = [int(v["crc"], 16) for v in vectors["known_answers"] + vectors["message_headers"] + vectors["zero_runs"]]
    pos, off, mem = 0, [], bytearray()
    for i, b in enumerate(items):
        pad = (-(len(mem)) + (i % 16)) % 64  # varied alignment
        mem += bytes(pad)
        off.append(len(mem))
        mem += b
    got = run_batch(gpu, np.frombuffer(bytes(mem), dtype=np.uint8), off, [len(b) for b in items])
    assert list(got) == expect


def test_golden_random_vectors(gpu, vectors):
    rnd = vectors["random"]
    mem, off, ln, cin = bytearray(), [], [], []
    for v in rnd:
        data = stream_bytes(int(v["seed"], 16), v["offset"], v["len"]).tobytes()
        mem += bytes((v["offset"] - len(mem)) % 64)  # keep the fixture's misalignment
        off.append(len(mem))
        ln.append(len(data))
        cin.append(int(v["crc_in"], 16))
        mem += data
    got = run_batch(gpu, np.frombuffer(bytes(mem), dtype=np.uint8), off, ln, crc_in=cin)
    assert [f"0x{x:08x}" for x in got] == [v["crc"] for v in rnd]


def test_every_small_length_and_alignment(gpu, oracle):
    mem = stream_bytes(99, 0, 1 << 16)
    off, ln = [], []
    for a in range(16):
        for n in range(0, 80):
            off.append(1000 + 113 * len(off) % 60000 // 16 * 16 + a)
            ln.append(n)
    got = run_batch(gpu, mem, off, ln)
    assert np.array_equal(got, oracle.batch(mem, off, ln))


@pytest.mark.parametrize("grid", [1, 3, 17, 256, 0])
def test_ragged_batch_grid_sizes(gpu, oracle, grid):
    """Different persistent-grid sizes move every wave cut point through the chunks."""
    rng = np.random.default_rng(grid)
    mem = stream_bytes(5, 0, 24 << 20)
    n = 300
    ln = rng.integers(0, 3 << 20, size=n)
    ln[:20] = [0, 1, 15, 16, 17, 1023, 1024, 1025, 4095, 4096, 4097, 65535, 65536, 65537, 262143, 262144, 262145,
               (1 << 20) - 1, 1 << 20, (1 << 20) + 1]
    off = rng.integers(0, (24 << 20) - (3 << 20), size=n)
    off[::3] = off[::3] // 16 * 16
    gpu.set_grid(0, grid)
    try:
        got = run_batch(gpu, mem, off, ln)
    finally:
        gpu.set_grid(0, 0)
    assert np.array_equal(got, oracle.batch(mem, off, ln, threads=8))


VARIANTS = (0, 29)  # built into the library: the 16-B-piece fallback and the default (32: A/B builds only)


@pytest.mark.parametrize("variant", VARIANTS)
def test_kernel_variants(gpu, oracle, variant):
    rng = np.random.default_rng(100 + variant)
    mem = stream_bytes(6, 0, 16 << 20)
    ln = rng.integers(0, 2 << 20, size=64)
    off = rng.integers(0, (16 << 20) - (2 << 20), size=64)
    default = gpu.get_variant(0)
    gpu.set_variant(0, variant)
    try:
        got = run_batch(gpu, mem, off, ln)
    finally:
        gpu.set_variant(0, default)
    assert np.array_equal(got, oracle.batch(mem, off, ln, threads=8))


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("grid", [0, 3])
def test_small_chunk_group_kernel(gpu, oracle, variant, grid):
    """Group phase (variant 29; variant 0 sweeps every chunk): whole chunks <= 16 KiB, G lanes
    each, init register folded into the data, size-classed rounds. Lengths 0..20000 at every
    alignment, crc_in, large chunks between; batches of >= 16384 chunks so the group phase engages."""
    rng = np.random.default_rng(700 + variant * 10 + grid)
    mem = stream_bytes(70 + variant, 0, 8 << 20)
    n = 20000  # >= kGroupMinChunks (16384): group modes engage
    ln = rng.integers(0, 20000, size=n)
    ln[:46] = list(range(0, 20)) + [255, 256, 257, 511, 512, 513, 2047, 2048, 2049, 4095, 4096, 4097,
                                    1 << 20, 3, 2, 1, 0, 16, 17, 33, 8191, 8192, 8193, 16383, 16384, 16385]
    ln[::397] = rng.integers(5000, 1 << 20, size=len(ln[::397]))  # large chunks mixed in
    off = rng.integers(0, (8 << 20) - (1 << 20), size=n)
    off[:16] = np.arange(16)  # chunks in the first bytes of the allocation
    cin = rng.integers(0, 1 << 32, size=n, dtype=np.uint64).astype(np.uint32)
    cin[::3] = 0
    default = gpu.get_variant(0)
    gpu.set_variant(0, variant)
    gpu.set_grid(0, grid)
    try:
        got = run_batch(gpu, mem, off, ln, crc_in=cin)
    finally:
        gpu.set_variant(0, default)
        gpu.set_grid(0, 0)
    assert np.array_equal(got, oracle.batch(mem, off, ln, crc_in=cin, threads=8))


def test_class0_small_records(gpu, oracle):
    """Group class 0 (<= 256 B, 2-lane groups, 32 chunks per round): every length 1..256 at every
    offset mod 16 with and without a seed, a batch whose class-0 count is not a multiple of 32
    (idle groups in a wave's last round), and chunks ending at the buffer's last byte."""
    rng = np.random.default_rng(4242)
    size = 4 << 20
    mem = stream_bytes(77, 0, size)
    n = 16384 + 4133  # >= kGroupMinChunks; odd count
    ln = rng.integers(1, 257, size=n)
    ln[:256] = np.arange(1, 257)
    off = rng.integers(0, size - 256, size=n)
    off[:256] = (np.arange(256) * 4099) % (size - 256)  # all 16 alignments
    off[256:512] = size - ln[256:512]  # ends at the last byte
    cin = rng.integers(0, 1 << 32, size=n, dtype=np.uint64).astype(np.uint32)
    cin[1::2] = 0
    got = run_batch(gpu, mem, off, ln, crc_in=cin)
    assert np.array_equal(got, oracle.batch(mem, off, ln, crc_in=cin, threads=8))


@pytest.mark.parametrize("n", [2048 * 1024 + 777, 2048 * 3 + 1])
def test_plan_many_blocks(gpu, oracle, n):
    """The plan's scan across planning blocks (2048 chunks each): more blocks than one pass of the
    block-sum loop covers (1024), every size class in every block, empty chunks, seeds, in place."""
    torch = _torch()
    rng = np.random.default_rng(n)
    size = 64 << 20
    mem = stream_bytes(78, 0, size)
    ln = rng.integers(0, 600, size=n)
    mid = rng.random(n) < 0.02
    ln[mid] = rng.integers(600, 20000, size=int(mid.sum()))
    big = rng.random(n) < 0.001
    ln[big] = rng.integers(20000, 1 << 20, size=int(big.sum()))
    ln[rng.random(n) < 0.05] = 0
    off = rng.integers(0, size - (1 << 20), size=n)
    cin = rng.integers(0, 1 << 32, size=n, dtype=np.uint64).astype(np.uint32)
    expect = oracle.batch(mem, off, ln, crc_in=cin, threads=8)
    assert np.array_equal(run_batch(gpu, mem, off, ln, crc_in=cin), expect)
    base = dev_bytes(mem)
    io = torch.from_numpy(cin.view(np.int32).copy()).cuda()
    gpu.crc32_batch(base, dev_u64(off), dev_u64(ln), crc_in=io, out=io)  # in place
    torch.cuda.synchronize()
    assert np.array_equal(host_u32(io), expect)


@pytest.mark.parametrize("with_large", [False, True])
def test_all_small_batch_garbage_workspace(gpu, oracle, with_large):
    """A batch the group phase takes whole stores no per-chunk byte_start and leaves its chunks'
    out[] words to the group phase: a workspace and an out buffer full of garbage must not leak
    into the CRCs. with_large: one 1 MiB chunk, so the batch has share bytes and the starts are stored."""
    torch = _torch()
    rng = np.random.default_rng(808 + with_large)
    size = 16 << 20
    mem = stream_bytes(79, 0, size)
    n = 20000
    ln = rng.integers(0, 16385, size=n)
    ln[::7] = 0
    ln[:300] = rng.integers(1, 257, size=300)
    if with_large:
        ln[n // 2] = 1 << 20
    off = rng.integers(0, size - (1 << 20), size=n)
    cin = rng.integers(0, 1 << 32, size=n, dtype=np.uint64).astype(np.uint32)
    ws = torch.full((gpu.workspace_bytes(n),), 0xA5, dtype=torch.uint8, device="cuda")
    out = torch.full((n,), -0x5A5A5A5B, dtype=torch.int32, device="cuda")
    c_in = torch.from_numpy(cin.view(np.int32).copy()).cuda()
    gpu.crc32_batch(dev_bytes(mem), dev_u64(off), dev_u64(ln), crc_in=c_in, out=out, workspace=ws)
    torch.cuda.synchronize()
    assert np.array_equal(host_u32(out), oracle.batch(mem, off, ln, crc_in=cin, threads=8))


def test_crc_in_streaming_composition(gpu, oracle):
    """update(A) then update(B) == update(A||B): PutOperation's slice-by-slice fill (PutOperation.java:1700-1703)."""
    torch = _torch()
    mem = stream_bytes(12, 0, 9 << 20)
    base = dev_bytes(mem)
    cuts = [0, 1, 16, 1000, 1 << 20, (4 << 20) + 3, 9 << 20]
    whole = oracle.crc32(mem)
    for cut in cuts:
        a = gpu.crc32_batch(base, dev_u64([0]), dev_u64([cut]))
        b = gpu.crc32_batch(base, dev_u64([cut]), dev_u64([(9 << 20) - cut]), crc_in=a)
        torch.cuda.synchronize()
        assert host_u32(b)[0] == whole


def test_verify_flags_zipf(gpu, oracle):
    """C4 in miniature: Zipf sizes, 1% single-bit flips; flags must match exactly."""
    torch = _torch()
    sizes = zipf_sizes(2000, seed=20261015) // 16  # scaled down 16x (256 B .. 256 KiB)
    off = np.concatenate([[0], np.cumsum((sizes + 15) // 16 * 16)[:-1]]).astype(np.int64)
    total = int(off[-1] + sizes[-1])
    mem = stream_bytes(20261015, 0, total)
    expected = oracle.batch(mem, off, sizes, threads=8)
    rng = np.random.default_rng(1)
    bad = rng.choice(len(sizes), size=20, replace=False)
    corrupt = mem.copy()
    for i in bad:
        pos = off[i] + rng.integers(0, sizes[i])
        corrupt[pos] ^= np.uint8(1 << int(rng.integers(0, 8)))
    exp_dev = torch.from_numpy(expected.view(np.int32)).cuda()
    crc, mism, count = gpu.crc32_verify(dev_bytes(corrupt), dev_u64(off), dev_u64(sizes), exp_dev)
    torch.cuda.synchronize()
    flags = mism.cpu().numpy()
    assert set(np.nonzero(flags)[0]) == set(int(i) for i in bad)
    assert int(count.item()) == len(bad)
    assert np.array_equal(host_u32(crc), oracle.batch(corrupt, off, sizes, threads=8))


def test_empty_chunks_and_crc_in(gpu, oracle):
    """Zero-length chunks return crc_in unchanged (Crc32.update on an empty buffer is a no-op, Crc32.java:101-103)."""
    mem = stream_bytes(2, 0, 1 << 16)
    off = [0, 100, 100, 200, 5000, 5000, 0]
    ln = [0, 0, 50, 0, 0, 3000, 0]
    cin = [0, 0x1234, 0x55AA, 0xFFFFFFFF, 7, 9, 0xDEADBEEF]
    got = run_batch(gpu, mem, off, ln, crc_in=cin)
    assert np.array_equal(got, oracle.batch(mem, off, ln, crc_in=np.array(cin, dtype=np.uint32)))
    assert got[1] == 0x1234 and got[3] == 0xFFFFFFFF


def test_overlapping_and_repeated_chunks(gpu, oracle):
    mem = stream_bytes(31, 0, 1 << 20)
    off = [0, 0, 5, 5, 100, 0, 65536]
    ln = [1 << 20, 1 << 20, 1000, 1000, 200000, 0, 300000]
    assert np.array_equal(run_batch(gpu, mem, off, ln), oracle.batch(mem, off, ln))


def test_separate_workspaces_two_streams(gpu, oracle):
    torch = _torch()
    from ambry_amd._lib import lib

    mem = stream_bytes(44, 0, 8 << 20)
    base = dev_bytes(mem)
    n = 128
    rng = np.random.default_rng(3)
    off = rng.integers(0, 4 << 20, size=n)
    ln = rng.integers(0, 4 << 20, size=n)
    wsz = lib().ambrycrc_workspace_bytes(n)
    outs = []
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    for s in streams:
        ws = torch.empty(wsz, dtype=torch.uint8, device="cuda")
        with torch.cuda.stream(s):
            outs.append((gpu.crc32_batch(base, dev_u64(off), dev_u64(ln), workspace=ws, stream=s), ws))
    torch.cuda.synchronize()
    exp = oracle.batch(mem, off, ln, threads=8)
    for o, _ in outs:
        assert np.array_equal(host_u32(o), exp)


def _full_size_check(gpu, oracle, n_chunks, chunk, seed, sample):
    """Whole config resident in HBM; sampled chunks vs oracle; region-as-one-chunk vs combine-fold."""
    torch = _torch()
    import ambry_amd

    total = n_chunks * chunk
    buf = torch.empty(total, dtype=torch.uint8, device="cuda")
    gpu.fill_random(buf, seed, 0)
    off = dev_u64(np.arange(n_chunks, dtype=np.int64) * chunk)
    ln = dev_u64(np.full(n_chunks, chunk, dtype=np.int64))
    out1 = gpu.crc32_batch(buf, off, ln)
    out2 = gpu.crc32_batch(buf, off, ln)
    whole = gpu.crc32_batch(buf, dev_u64([0]), dev_u64([total]))
    torch.cuda.synchronize()
    c1, c2 = host_u32(out1), host_u32(out2)
    assert np.array_equal(c1, c2)
    fold = 0
    for c in c1:
        fold = ambry_amd.combine(fold, int(c), chunk)
    assert fold == int(host_u32(whole)[0])
    rng = np.random.default_rng(seed)
    for i in sorted(set([0, n_chunks - 1] + list(rng.integers(0, n_chunks, size=sample)))):
        data = buf[i * chunk:(i + 1) * chunk].cpu().numpy()
        assert oracle.crc32(data) == int(c1[i]), i
    del buf


@pytest.mark.parametrize("window", [1 << 20, 3 << 20, 0])
def test_sweep_rounds_window(gpu, oracle, window):
    """Sweep rounds (ambrycrc_set_window): a 1 MiB or 3 MiB window turns a ~27 MiB ragged batch
    into many rounds of shares, so chunks are cut at round as well as wave boundaries; 0 = one
    round. Results equal the oracle either way, with crc_in and empty chunks mixed in."""
    rng = np.random.default_rng(window + 3)
    mem = stream_bytes(9, 0, 40 << 20)
    n = 400
    ln = rng.integers(0, 300000, size=n)
    ln[:8] = [0, 1, 17, 4096, 1 << 20, (3 << 20) + 5, 16, 0]
    off = rng.integers(0, (40 << 20) - (4 << 20), size=n)
    cin = rng.integers(0, 1 << 32, size=n, dtype=np.uint64).astype(np.uint32)
    cin[::2] = 0
    gpu.set_window(0, window)
    try:
        got = run_batch(gpu, mem, off, ln, crc_in=cin)
    finally:
        gpu.set_window(0, 32 << 30)
    assert np.array_equal(got, oracle.batch(mem, off, ln, crc_in=cin, threads=8))


def test_c3_full_size_rounds(gpu, oracle):
    """C3 swept in 4 GiB rounds (8 rounds of 16,384 shares) gives the same CRCs as one round."""
    torch = _torch()
    total = 8192 * (4 << 20)
    buf = torch.empty(total, dtype=torch.uint8, device="cuda")
    gpu.fill_random(buf, 0xC3, 0)
    off = dev_u64(np.arange(8192, dtype=np.int64) * (4 << 20))
    ln = dev_u64(np.full(8192, 4 << 20, dtype=np.int64))
    one = host_u32(gpu.crc32_batch(buf, off, ln))
    gpu.set_window(0, 4 << 30)
    try:
        rounds = host_u32(gpu.crc32_batch(buf, off, ln))
    finally:
        gpu.set_window(0, 32 << 30)
    assert np.array_equal(one, rounds)
    assert oracle.crc32(buf[:4 << 20].cpu().numpy()) == int(one[0])
    del buf


@pytest.mark.parametrize("window", [0, 1 << 30])
def test_chunks_past_4gib(gpu, oracle, window):
    """64-bit offsets and lengths: one 5 GiB + 3 B chunk starting at an odd offset (its length
    and its end both past 2^32), a short chunk starting past 4 GiB, and a 4 GiB + 1 B chunk with
    crc_in, in one batch, swept in one round or in 1 GiB rounds. The ABI takes uint64 lengths
    (ambrycrc.h); Ambry's own chunks stop at 4 MiB, so this is the boundary's limit, not a
    config. Every CRC is checked against the oracle over the same bytes copied to the host."""
    torch = _torch()
    total = (5 << 30) + 64
    buf = torch.empty(total, dtype=torch.uint8, device="cuda")
    gpu.fill_random(buf, 0x5C, 0)
    off = [7, (4 << 30) + 13, 1]
    ln = [(5 << 30) + 3, 4093, (4 << 30) + 1]
    cin = np.array([0, 0x1234ABCD, 0xDEADBEEF], dtype=np.uint32)
    cin_t = torch.from_numpy(cin.view(np.int32)).cuda()
    gpu.set_window(0, window)
    try:
        got = host_u32(gpu.crc32_batch(buf, dev_u64(off), dev_u64(ln), crc_in=cin_t))
    finally:
        gpu.set_window(0, 32 << 30)
    host = buf.cpu().numpy()
    del buf
    want = [oracle.crc32(host[o:o + n], int(c)) for o, n, c in zip(off, ln, cin)]
    assert [int(x) for x in got] == want


def test_c2_full_size(gpu, oracle):
    """C2: 65,536 x 64 KiB."""
    _full_size_check(gpu, oracle, 65536, 64 << 10, 0xC2, sample=64)


def test_c3_full_size(gpu, oracle):
    """C3 (headline): 8,192 x 4 MiB = 32 GiB resident."""
    _full_size_check(gpu, oracle, 8192, 4 << 20, 0xC3, sample=12)


def test_c4_full_size_verify(gpu, oracle):
    """C4 as SURVEY.md §8d defines it: 32,768 Zipf(1.2) chunks of 4 KiB-4 MiB (9.21 GiB) packed at
    16-B offsets, expected CRCs from the CPU oracle over every chunk, single-bit flips injected
    into 1 % of the chunks on the device; the mismatch flags must name exactly those chunks."""
    torch = _torch()
    sizes = zipf_sizes(32768)
    off = np.concatenate([[0], np.cumsum((sizes + 15) // 16 * 16)[:-1]]).astype(np.int64)
    total = int(off[-1] + sizes[-1])
    buf = torch.empty(total, dtype=torch.uint8, device="cuda")
    gpu.fill_random(buf, 0xC4, 0)
    torch.cuda.synchronize()
    expected = oracle.batch(buf.cpu().numpy(), off, sizes, threads=16)  # oracle over every chunk
    rng = np.random.default_rng(0xC4)
    bad = np.sort(rng.choice(len(sizes), size=len(sizes) // 100, replace=False))
    pos = off[bad] + (rng.random(len(bad)) * sizes[bad]).astype(np.int64)
    bits = torch.from_numpy((1 << rng.integers(0, 8, size=len(bad))).astype(np.uint8)).cuda()
    pos_t = torch.from_numpy(pos).cuda()
    buf[pos_t] ^= bits
    exp_dev = torch.from_numpy(expected.view(np.int32)).cuda()
    crc, mism, count = gpu.crc32_verify(buf, dev_u64(off), dev_u64(sizes), exp_dev)
    torch.cuda.synchronize()
    flags = mism.cpu().numpy()
    assert np.array_equal(np.nonzero(flags)[0], bad)
    assert int(count.item()) == len(bad)
    good = np.ones(len(sizes), dtype=bool)
    good[bad] = False
    assert np.array_equal(host_u32(crc)[good], expected[good])
    del buf


def test_host_resident_path(gpu, oracle):
    """ambrycrc_batch_host: pageable and pinned inputs, including a chunk larger than one staging slab."""
    torch = _torch()
    rng = np.random.default_rng(8)
    lens = [0, 1, 17, 4096, 1 << 20, (300 << 20) + 5, 65536, 3]
    chunks = [torch.from_numpy(stream_bytes(int(rng.integers(1 << 30)), 0, n)) for n in lens]
    exp = [oracle.crc32(c.numpy()) for c in chunks]
    assert gpu.crc32_batch_host(chunks, device=0, pinned=False) == exp
    pinned = [c.pin_memory() for c in chunks]
    assert gpu.crc32_batch_host(pinned, device=0, pinned=True) == exp
    cin = [(i * 0x01000193) & 0xFFFFFFFF for i in range(len(lens))]
    exp2 = [oracle.crc32(c.numpy(), ci) for c, ci in zip(chunks, cin)]
    assert gpu.crc32_batch_host(chunks, device=0, pinned=False, crc_in=cin) == exp2


@pytest.mark.parametrize("ndev", [1, 3, 16])
def test_batch_multi(gpu, oracle, ndev):
    """ambrycrc_batch_multi: byte-balanced ranges, one host thread each. The 1-GPU box lists
    device 0 ndev times, which exercises the partitioning (more ranges than chunks at 16,
    empty chunks, a chunk dominating the bytes) and the concurrent per-range calls."""
    torch = _torch()
    rng = np.random.default_rng(80 + ndev)
    lens = [0, 5, (40 << 20) + 3, 0, 4096, 1 << 20, 65536, 17, 0, 1000, 8 << 20]
    chunks = [torch.from_numpy(stream_bytes(int(rng.integers(1 << 30)), 0, n)) for n in lens]
    cin = [(i * 0x9E3779B9) & 0xFFFFFFFF for i in range(len(lens))]
    exp = [oracle.crc32(c.numpy(), ci) for c, ci in zip(chunks, cin)]
    assert gpu.crc32_batch_multi(chunks, [0] * ndev, crc_in=cin) == exp
    assert gpu.crc32_batch_multi(chunks[:2], [0] * ndev) == [oracle.crc32(c.numpy()) for c in chunks[:2]]


def test_batch_multi_rejects_uninitialised_device(gpu):
    from ambry_amd._lib import AmbryCrcError, lib

    torch = _torch()
    if torch.cuda.device_count() > 7:
        pytest.skip("device 7 may legitimately be initialised on an 8-GPU node")
    with pytest.raises(AmbryCrcError):
        gpu.crc32_batch_multi([torch.zeros(10, dtype=torch.uint8)], [0, 7])
    assert lib().ambrycrc_batch_multi(None, None, None, None, 0, None, 0, 0) != 0  # ndev = 0


def test_timing_hook(gpu):
    torch = _torch()
    gpu.timing_enable(0, True)
    try:
        buf = torch.empty(64 << 20, dtype=torch.uint8, device="cuda")
        gpu.fill_random(buf, 1, 0)
        gpu.crc32_batch(buf, dev_u64([0]), dev_u64([64 << 20]))
        ms, cnt = gpu.timing_collect(0)
        assert cnt == 1 and ms > 0
    finally:
        gpu.timing_enable(0, False)


@pytest.mark.parametrize("shift", [1, 3, 8, 13])
def test_misaligned_base_pointer(gpu, oracle, shift):
    """d_base itself off 16-B alignment (a ByteBuf slice at any address): every chunk's
    alignment math is relative to d_base, so the kernels must still be bit-exact and read
    nothing before d_base. Wave mode and the group phase (>= 16384 chunks) both run."""
    rng = np.random.default_rng(900 + shift)
    mem = stream_bytes(90 + shift, 0, 6 << 20)
    full = dev_bytes(mem)
    base = full[shift:]  # data_ptr() = allocation + shift
    view = mem[shift:]
    for n, hi in ((300, 1 << 20), (20000, 20000)):
        ln = rng.integers(0, hi, size=n)
        ln[:6] = [0, 1, 15, 16, 17, 4095]
        off = rng.integers(0, len(view) - hi, size=n)
        off[:4] = [0, 1, 2, 3]  # chunks at the very start of the shifted base
        got = run_batch(gpu, view, off, ln, mem_dev=base)
        assert np.array_equal(got, oracle.batch(view, off, ln, threads=8)), (shift, n)


def test_hip_graph_capture_and_replay(gpu, oracle):
    """ambrycrc_batch_dev with a caller workspace is stream-capture safe:
    captured once into a HIP graph and replayed after the bytes change, it CRCs the new bytes."""
    torch = _torch()
    mem = stream_bytes(31, 0, 3 << 20)
    base = dev_bytes(mem)
    off = dev_u64([0, 5, 4096, 1 << 20])
    ln = dev_u64([100, 70000, 1 << 20, (2 << 20) - 3])
    out = torch.empty(4, dtype=torch.int32, device="cuda")
    ws = torch.empty(gpu.workspace_bytes(4), dtype=torch.uint8, device="cuda")
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        gpu.crc32_batch(base, off, ln, out=out, workspace=ws)
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            gpu.crc32_batch(base, off, ln, out=out, workspace=ws)
    torch.cuda.synchronize()
    offs, lens = [0, 5, 4096, 1 << 20], [100, 70000, 1 << 20, (2 << 20) - 3]
    for seed in (32, 33):
        new = stream_bytes(seed, 0, 3 << 20)
        base.copy_(torch.from_numpy(new).cuda())
        g.replay()
        torch.cuda.synchronize()
        assert np.array_equal(host_u32(out), oracle.batch(new, offs, lens)), seed


def test_hip_graph_default_workspace_outlives_growth_and_eviction(gpu, oracle):
    """A graph captured with the stream's DEFAULT workspace (d_ws = NULL) stays valid after that workspace
    is replaced: a later, larger uncaptured call on the same stream grows it, and calls on 17 other streams
    evict the stream's entry (kMaxStreamWs = 16). The captured buffer is kept until shutdown, so every
    replay still CRCs the current bytes exactly (a freed buffer would be read by the replay)."""
    torch = _torch()
    offs, lens = [0, 5, 4096, 1 << 20], [100, 70000, 1 << 20, (2 << 20) - 3]
    mem = stream_bytes(41, 0, 3 << 20)
    base = dev_bytes(mem)
    off, ln = dev_u64(offs), dev_u64(lens)
    out = torch.empty(4, dtype=torch.int32, device="cuda")
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        gpu.crc32_batch(base, off, ln, out=out)  # sizes the stream's default workspace
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            gpu.crc32_batch(base, off, ln, out=out)
    torch.cuda.synchronize()

    def replay_and_check(seed):
        new = stream_bytes(seed, 0, 3 << 20)
        base.copy_(torch.from_numpy(new).cuda())
        with torch.cuda.stream(s):
            g.replay()
        torch.cuda.synchronize()
        assert np.array_equal(host_u32(out), oracle.batch(new, offs, lens)), seed

    replay_and_check(42)
    # growth: 300,000 chunks need a far larger workspace on the same stream
    n = 300_000
    big_off = dev_u64(np.arange(n, dtype=np.int64) * 7)
    big_ln = dev_u64(np.full(n, 9, dtype=np.int64))
    with torch.cuda.stream(s):
        big = gpu.crc32_batch(base, big_off, big_ln)
    torch.cuda.synchronize()
    cur = base.cpu().numpy()
    assert np.array_equal(host_u32(big)[:1000], oracle.batch(cur, np.arange(1000) * 7, np.full(1000, 9)))
    replay_and_check(43)
    # eviction: more streams than the context keeps default workspaces for
    for _ in range(17):
        t = torch.cuda.Stream()
        with torch.cuda.stream(t):
            gpu.crc32_batch(base, off, ln)
    torch.cuda.synchronize()
    replay_and_check(44)


def test_host_path_concurrent_threads(gpu, oracle):
    """Host entry points called from several host threads at once (the reference calls Crc32
    from the ChunkFiller, network and crypto threads): batch_host, verify_trailed_host and the
    host streaming loop interleave and each thread gets its own exact results."""
    import threading
    import zlib

    mem = stream_bytes(77, 0, 96 << 20)
    errors = []

    def worker(t):
        try:
            rng = np.random.default_rng(t)
            for _ in range(3):
                n = int(rng.integers(1, 40))
                offs = rng.integers(0, (96 << 20) - (9 << 20), size=n)
                lens = rng.integers(0, 3 << 20, size=n)
                chunks = [(mem.ctypes.data + int(o), int(ln)) for o, ln in zip(offs, lens)]
                got = gpu.crc32_batch_host(chunks)
                exp = oracle.batch(mem, offs, lens)
                if list(exp) != got:
                    errors.append(("batch_host", t))
                item = mem[int(offs[0]):int(offs[0]) + 100000].tobytes()
                bad = gpu.verify_trailed_host([item + zlib.crc32(item).to_bytes(8, "big"), item[:7]])
                if bad != [False, True]:
                    errors.append(("trailed", t))
        except Exception as e:  # noqa: BLE001 -- reported below
            errors.append((repr(e), t))

    threads = [threading.Thread(target=worker, args=(t,)) for t in range(6)]
    for th in threads:
        th.start()
    for th in threads:
        th.join()
    assert not errors, errors


def test_randomized_batches(gpu, oracle):
    """40 random batches against the oracle: chunk counts from 1 to 40,000 (either side of the
    16,384-chunk group threshold), lengths from 0 to 2 MiB drawn per batch from different size
    mixes, any offset, random crc_in, random grid sizes and sweep windows (rounds)."""
    rng = np.random.default_rng(2026)
    mem = stream_bytes(99, 0, 48 << 20)
    for it in range(40):
        n = int(rng.choice([1, 2, 7, 64, 500, 3000, 16383, 16384, 20000, 40000]))
        mix = it % 4
        if mix == 0:
            ln = rng.integers(0, 300, size=n)
        elif mix == 1:
            ln = rng.integers(0, 20000, size=n)
        elif mix == 2:
            ln = (rng.pareto(1.2, size=n) * 2000).astype(np.int64).clip(0, 2 << 20)
        else:
            ln = rng.integers(0, 2 << 20, size=n) if n <= 64 else rng.integers(0, 5000, size=n)
        off = rng.integers(0, (48 << 20) - int(ln.max()) - 1, size=n)
        cin = rng.integers(0, 1 << 32, size=n, dtype=np.uint64).astype(np.uint32) if it % 3 == 0 else None
        grid = int(rng.choice([0, 0, 1, 5, 77]))
        window = int(rng.choice([32 << 30, 1 << 20, 4 << 20]))
        gpu.set_grid(0, grid)
        gpu.set_window(0, window)
        try:
            got = run_batch(gpu, mem, off, ln, crc_in=cin)
        finally:
            gpu.set_grid(0, 0)
            gpu.set_window(0, 32 << 30)
        exp = oracle.batch(mem, off, ln, crc_in=cin, threads=8)
        assert np.array_equal(got, exp), (it, n, mix, grid, window)


def test_shutdown_and_reinit(gpu, oracle):
    """ambrycrc_shutdown releases every context (tables, workspace, staging and message slabs,
    events); a new ambrycrc_init works as before."""
    from ambry_amd import lib

    mem = stream_bytes(31, 0, 4 << 20)
    chunks = [(mem.ctypes.data + 5, 3 << 20), (mem.ctypes.data, 1000)]
    before = gpu.crc32_batch_host(chunks)
    assert lib().ambrycrc_shutdown() == 0
    assert lib().ambrycrc_batch_host((ctypes.c_void_p * 1)(mem.ctypes.data), (ctypes.c_uint64 * 1)(10), None,
                                     (ctypes.c_uint32 * 1)(), 1, 0, 0) == -4  # ENOINIT
    gpu.init(0)
    gpu.set_host_policy(0, gpu.HOST_GPU)  # a new context starts at the auto policy (conftest's gpu fixture)
    assert gpu.crc32_batch_host(chunks) == before == list(oracle.batch(mem, [5, 0], [3 << 20, 1000]))
    assert gpu.last_host_path(0) == 1


def test_timing_with_host_paths(gpu, oracle):
    """Kernel timing stays usable while host-path calls run (they hold the context lock across the
    call; the timing events have their own): batch_host and the device batch both record."""
    torch = _torch()
    mem = stream_bytes(41, 0, 8 << 20)
    gpu.timing_collect(0)
    gpu.timing_enable(0, True)
    try:
        got = gpu.crc32_batch_host([(mem.ctypes.data, 8 << 20)])
        base = dev_bytes(mem)
        out = gpu.crc32_batch(base, dev_u64([0]), dev_u64([8 << 20]))
        torch.cuda.synchronize()
    finally:
        gpu.timing_enable(0, False)
    each = gpu.timing_collect_each(0)
    assert len(each) >= 2 and all(x > 0 for x in each)
    assert got[0] == int(host_u32(out)[0]) == oracle.crc32(mem)


def _mixed_batch(seed, n=20000):
    rng = np.random.default_rng(seed)
    mem = stream_bytes(seed, 0, 8 << 20)
    ln = rng.integers(0, 20000, size=n)
    ln[::397] = rng.integers(20000, 1 << 20, size=len(ln[::397]))  # sweep-mode chunks mixed in
    ln[:8] = [0, 1, 3, 4, 5, 16, 17, 16385]
    off = rng.integers(0, (8 << 20) - (1 << 20), size=n)
    cin = rng.integers(0, 1 << 32, size=n, dtype=np.uint64).astype(np.uint32)
    cin[::5] = 0
    return mem, off, ln, cin


@pytest.mark.parametrize("variant", VARIANTS)
def test_in_place_continuation(gpu, oracle, variant):
    """d_out == d_crc_in (a streaming update in place): the plan copies crc_in before it
    initialises out, so every chunk continues from its own seed. 20,000 mixed chunks hit both
    the group phase and the sweep (aliased buffers used to compute from 0)."""
    torch = _torch()
    mem, off, ln, cin = _mixed_batch(4242)
    buf = torch.from_numpy(cin.view(np.int32).copy()).cuda()
    default = gpu.get_variant(0)
    gpu.set_variant(0, variant)
    try:
        out = gpu.crc32_batch(dev_bytes(mem), dev_u64(off), dev_u64(ln), crc_in=buf, out=buf)
        torch.cuda.synchronize()
    finally:
        gpu.set_variant(0, default)
    assert out.data_ptr() == buf.data_ptr()
    assert np.array_equal(host_u32(buf), oracle.batch(mem, off, ln, crc_in=cin, threads=8))


def test_partial_overlap_of_crc_in_and_out_rejected(gpu):
    torch = _torch()
    from ambry_amd._lib import AmbryCrcError

    buf = torch.zeros(17, dtype=torch.int32, device="cuda")
    mem = dev_bytes(stream_bytes(1, 0, 4096))
    with pytest.raises(AmbryCrcError):
        gpu.crc32_batch(mem, dev_u64([0] * 16), dev_u64([100] * 16), crc_in=buf[1:], out=buf[:16])


def test_default_workspace_concurrent_threads(gpu, oracle):
    """Six host threads call ambrycrc_batch_dev with ws = NULL and growing n, each on its own
    stream and on the shared default stream: a growing workspace is retired behind the work
    queued on it, never freed under it (ambrycrc.cpp resolve/ensure_ws)."""
    import threading

    torch = _torch()
    mem = stream_bytes(77, 0, 4 << 20)
    base = dev_bytes(mem)
    errors, results = [], {}

    def work(t):
        try:
            rng = np.random.default_rng(t)
            s = torch.cuda.Stream() if t % 2 else torch.cuda.current_stream()
            for it in range(12):
                n = int(64 * (2 ** (it % 9)) + t)  # 65 .. 16,390 chunks: crosses the group threshold
                ln = rng.integers(0, 9000, size=n)
                off = rng.integers(0, (4 << 20) - 9000, size=n)
                with torch.cuda.stream(s):
                    o, l = dev_u64(off), dev_u64(ln)
                    out = gpu.crc32_batch(base, o, l, stream=s)
                    got = out.cpu().numpy().view(np.uint32)
                results[(t, it)] = (off, ln, got)
        except Exception as e:  # pragma: no cover - reported below
            errors.append(repr(e))

    ths = [threading.Thread(target=work, args=(t,)) for t in range(6)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    torch.cuda.synchronize()
    assert not errors, errors
    assert len(results) == 72
    for off, ln, got in results.values():
        assert np.array_equal(got, oracle.batch(mem, off, ln, threads=8))


def test_many_short_lived_streams_default_workspace(gpu, oracle):
    """Default workspaces (d_ws NULL) are kept per stream up to a cap (kMaxStreamWs = 16), the least
    recently used retired behind its last call's event: 40 short-lived streams, each running a batch
    (some while earlier streams' work is still queued), every result right."""
    torch = _torch()
    rng = np.random.default_rng(31)
    mem = stream_bytes(31, 0, 8 << 20)
    base = dev_bytes(mem)
    jobs = []
    for k in range(40):
        n = int(rng.integers(1, 3000))
        ln = rng.integers(0, 40000, size=n)
        off = rng.integers(0, (8 << 20) - 40000, size=n)
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            out = gpu.crc32_batch(base, dev_u64(off), dev_u64(ln), stream=s)
        jobs.append((off, ln, out, s))
        if k % 5 == 4:  # drop some streams early (their buffers may be evicted while others queue)
            jobs[-3][3].synchronize()
    torch.cuda.synchronize()
    for off, ln, out, _ in jobs:
        assert np.array_equal(host_u32(out), oracle.batch(mem, off, ln))


def test_diagnostic_variants_not_selectable(gpu):
    """Variants 100-102 (timing builds that return wrong CRCs) and 32 (the split group kernel, which
    lost everywhere) are not in the product library."""
    from ambry_amd._lib import AmbryCrcError

    before = gpu.get_variant(0)
    for v in (1, 22, 28, 30, 31, 32, 33, 100, 101, 102, -1):
        with pytest.raises(AmbryCrcError):
            gpu.set_variant(0, v)
    assert gpu.get_variant(0) == before


@pytest.mark.parametrize("value,expect", [("0", 0), ("29", 29), ("32", 29), ("101", 29), ("abc", 29), ("29x", 29),
                                          ("-5", 29)])
def test_variant_environment_validated(value, expect):
    """AMBRYCRC_VARIANT selects only a built-in shape; anything else is ignored."""
    import os
    import subprocess
    import sys

    code = ("import sys; sys.path.insert(0, %r); from ambry_amd import device as D; D.init(0); "
            "print(D.get_variant(0))" % os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    env = dict(os.environ, AMBRYCRC_VARIANT=value)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert int(r.stdout.strip().splitlines()[-1]) == expect


def test_binding_rejects_bad_tensors(gpu):
    """ambry_amd.device checks every tensor before the ABI sees it (device.py:45)."""
    torch = _torch()
    base = dev_bytes(stream_bytes(3, 0, 4096))
    off, ln = dev_u64([0, 16]), dev_u64([10, 20])
    bad = [
        dict(crc_in=torch.zeros(2, dtype=torch.int32)),                       # CPU tensor
        dict(crc_in=torch.zeros(2, dtype=torch.int64, device="cuda")),        # wrong dtype
        dict(out=torch.zeros(3, dtype=torch.int32, device="cuda")),           # wrong size
        dict(out=torch.zeros(4, dtype=torch.int32, device="cuda")[::2]),      # non-contiguous
        dict(workspace=torch.zeros(16, dtype=torch.uint8)),                   # CPU workspace
    ]
    for kw in bad:
        with pytest.raises(TypeError):
            gpu.crc32_batch(base, off, ln, **kw)
    with pytest.raises(TypeError):
        gpu.crc32_verify(base, off, ln, torch.zeros(2, dtype=torch.int16, device="cuda"))
    # a workspace is sized in bytes whatever its dtype
    ws = torch.empty((gpu.workspace_bytes(2) + 7) // 8, dtype=torch.int64, device="cuda")
    out = gpu.crc32_batch(base, off, ln, workspace=ws)
    torch.cuda.synchronize()
    assert out.numel() == 2
