"""CRC-trailered store files: the LogSegment header on the host loop (CPU), and batched
trailer verify of index-segment-style files and device items (GPU).

Reference semantics: IndexSegment.checkDataIntegrityInByteBufferWithCRC
(ambry-store/.../IndexSegment.java:727-735) -- CRC32 of bytes [0, cap - 8) == the big-endian
long in the last 8 bytes; LogSegment's header (LogSegment.java:130-140, 603-607)."""
import struct
import zlib

import numpy as np
import pytest

from ambry_amd import store_files as sf
from datagen import stream_bytes


def _trailed(payload: bytes) -> bytes:
    return payload + struct.pack(">q", zlib.crc32(payload))


def _expect_bad(item: bytes) -> bool:
    if len(item) < 8:
        return True
    return zlib.crc32(item[:-8]) != struct.unpack(">q", item[-8:])[0]


def test_log_segment_header_roundtrip():
    for cap in (0, 1, 4 << 30, (1 << 63) - 1):
        h = sf.log_segment_header(cap)
        assert len(h) == sf.LOG_SEGMENT_HEADER_SIZE
        assert h[:10] == struct.pack(">hq", 0, cap)
        assert sf.log_segment_header_intact(h)
        for i in range(18):
            bad = bytearray(h)
            bad[i] ^= 0x10
            assert not sf.log_segment_header_intact(bytes(bad)), i
    assert not sf.log_segment_header_intact(sf.log_segment_header(5)[:17])


def _items(n, seed, max_len):
    rng = np.random.default_rng(seed)
    items = []
    for i in range(n):
        if i < 10:
            ln = i  # 0..7: too short (the reference throws); 8, 9: empty and 1-B payloads
            items.append(bytes(stream_bytes(seed, i, ln)) if ln < 8 else _trailed(bytes(stream_bytes(seed, i, ln - 8))))
            continue
        ln = int(rng.integers(0, max_len))
        item = bytearray(_trailed(stream_bytes(seed * 7919 + i, 0, ln).tobytes()))
        kind = rng.integers(0, 10)
        if kind == 0:  # payload bit flip
            if ln:
                item[int(rng.integers(0, ln))] ^= 1 << int(rng.integers(0, 8))
        elif kind == 1:  # high word of the stored long
            item[-8 + int(rng.integers(0, 4))] ^= 1 << int(rng.integers(0, 8))
        elif kind == 2:  # low word
            item[-4 + int(rng.integers(0, 4))] ^= 1 << int(rng.integers(0, 8))
        items.append(bytes(item))
    return items


@pytest.mark.gpu
@pytest.mark.parametrize("n,max_len", [(500, 200000), (20000, 20000)])
def test_verify_trailed_device(gpu, n, max_len):
    """Device items packed at arbitrary offsets; 20,000 items engage the group phase, which reads
    the stored CRCs of items up to 16 KiB itself (SweepArgs::exp_fill)."""
    import torch

    items = _items(n, n, max_len)
    offs, blob = [], bytearray()
    for i, it in enumerate(items):
        blob += bytes(i % 13)
        offs.append(len(blob))
        blob += it
    base = torch.from_numpy(np.frombuffer(bytes(blob), dtype=np.uint8).copy()).cuda()
    off = torch.tensor(offs, dtype=torch.int64, device="cuda")
    ln = torch.tensor([len(x) for x in items], dtype=torch.int64, device="cuda")
    mism, count = gpu.verify_trailed(base, off, ln)
    torch.cuda.synchronize()
    exp = [_expect_bad(x) for x in items]
    assert [bool(x) for x in mism.cpu().numpy()] == exp
    assert int(count.item()) == sum(exp)
    assert 0 < sum(exp) < n


@pytest.mark.gpu
def test_index_segments_intact_files(gpu, tmp_path):
    """index_segments_intact over files on disk (mmap -> ambrycrc_verify_trailed_host)."""
    items = _items(60, 3, 3 << 20)
    paths = []
    for i, it in enumerate(items):
        p = tmp_path / f"{i}_index"
        p.write_bytes(it)
        paths.append(str(p))
    got = sf.index_segments_intact(paths)
    assert got == [not _expect_bad(x) for x in items]
    with pytest.raises(FileNotFoundError):
        sf.index_segments_intact([str(tmp_path / "missing_index")])
