"""§8f row 3 -- FileStore.getChecksumsForRanges on libambrycrc (ambry_amd/filestore.py).

Reference semantics restated for the checker (FileStore.java:567-595): range (first, second)
covers [first, second), truncated at EOF; invalid ranges raise; values are Long.toString of
java.util.zip.CRC32 (zlib.crc32 here)."""
import zlib

import numpy as np
import pytest

from datagen import stream_bytes


def ref_checksums(data: bytes, ranges):
    out = []
    for a, b in ranges:
        if a < 0 or b < 0 or a > b:
            raise ValueError("Invalid byte range")
        out.append(str(zlib.crc32(data[a:b])))
    return out


def test_invalid_ranges_raise_before_device_work(ambry):
    from ambry_amd.filestore import checksums_for_ranges

    for bad in ([(-1, 5)], [(5, -1)], [(10, 5)], [(0, 3), (9, 2)]):
        with pytest.raises(ValueError):
            checksums_for_ranges(b"x" * 100, bad)
    assert checksums_for_ranges(b"x" * 100, []) == []


def test_checksum_ranges_generator():
    from ambry_amd.filestore import checksum_ranges

    rng = np.random.default_rng(0)
    size = (5 << 20) + 123
    r = checksum_ranges(size, 3, 1, rng)
    assert len(r) == 3 and r == sorted(r)
    for a, b in r:
        assert a % (1 << 20) == 0 and b == min(a + (1 << 20) - 1, size - 1)
    assert len(checksum_ranges(size, 100, 1, rng)) == 6
    with pytest.raises(ValueError):
        checksum_ranges(0, 1, 1, rng)


@pytest.mark.gpu
def test_get_checksums_for_ranges_matches_reference(gpu, tmp_path):
    from ambry_amd.filestore import checksum_ranges, get_checksums_for_ranges

    size = (40 << 20) + 777
    data = stream_bytes(0xF11E, 0, size).tobytes()
    path = tmp_path / "0_0_log"
    path.write_bytes(data)
    rng = np.random.default_rng(4)
    ranges = checksum_ranges(size, 10, 2, rng)
    ranges += [(0, 0), (5, 5), (3, 4), (size - 10, size + 100), (size + 5, size + 10), (1, size)]
    assert get_checksums_for_ranges(str(path), ranges) == ref_checksums(data, ranges)
