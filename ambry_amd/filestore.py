"""Mirror of FileStore.getChecksumsForRanges (ambry-store/src/main/java/com/github/ambry/store/FileStore.java:567-595)
over libambrycrc's range-checksum entry point (§8f row 3).

Same inputs (a file path inside the partition, a list of (first, second) integer
pairs), same output (decimal strings of the CRC values, Long.toString), same
semantics: range i covers [first, second), truncated at EOF; an invalid range
raises ValueError (the reference's IllegalArgumentException, wrapped there as a
FileStoreException with FileStoreErrorCode.UnknownError). The CRCs are computed
on the GPU (ambrycrc_range_checksums_host: pinned staging + hipMemcpyAsync + the
gfx950 kernels); the file is read once.
"""
from __future__ import annotations

import ctypes
import mmap
import os
from typing import Sequence

from ._lib import AMBRYCRC_EINVAL, AmbryCrcError, check, lib


def checksums_for_ranges(data, ranges: Sequence[tuple[int, int]], device: int = 0) -> list[int]:
    """uint32 CRCs of data[first:second] (clamped to len(data)) for each (first, second)."""
    n = len(ranges)
    if n == 0:
        return []
    first = (ctypes.c_int64 * n)(*[int(a) for a, _ in ranges])
    second = (ctypes.c_int64 * n)(*[int(b) for _, b in ranges])
    out = (ctypes.c_uint32 * n)()
    import numpy as np

    arr = np.frombuffer(data, dtype=np.uint8) if not isinstance(data, np.ndarray) else data.view(np.uint8)
    size = arr.nbytes
    buf = arr  # keeps the (possibly mmap-backed, read-only) buffer alive; no copy
    ptr = ctypes.c_void_p(arr.ctypes.data) if size else None
    rc = lib().ambrycrc_range_checksums_host(ptr, size, first, second, n, out, device)
    if rc == AMBRYCRC_EINVAL:
        bad = next(((a, b) for a, b in ranges if a < 0 or b < 0 or a > b), None)
        if bad is not None:
            raise ValueError(f"Invalid byte range: [{bad[0]}, {bad[1]}]")
    check(rc, "ambrycrc_range_checksums_host")
    del buf
    return list(out)


def get_checksums_for_ranges(file_path: str, ranges: Sequence[tuple[int, int]], device: int = 0) -> list[str]:
    """FileStore.getChecksumsForRanges: decimal-string CRCs of [first, second) of the file."""
    if not os.path.isfile(file_path):
        raise FileNotFoundError(file_path)
    with open(file_path, "rb") as f:
        size = os.fstat(f.fileno()).st_size
        if size == 0:
            return [str(c) for c in checksums_for_ranges(b"", ranges, device)]
        with mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ) as mm:
            return [str(c) for c in checksums_for_ranges(memoryview(mm), ranges, device)]


def checksum_ranges(file_size: int, ranges_count: int, range_size_mb: int, rng) -> list[tuple[int, int]]:
    """StoreFileCopyHandler.getChecksumRanges (ambry-file-transfer/.../StoreFileCopyHandler.java:404-434):
    `ranges_count` distinct range_size_mb-sized chunks, sorted; second = start + size - 1 (clamped)."""
    if file_size <= 0 or ranges_count <= 0 or range_size_mb <= 0:
        raise ValueError("file size, ranges count and range size must be > 0")
    rsz = range_size_mb * 1024 * 1024
    total = -(-file_size // rsz)
    chosen = sorted(rng.permutation(total)[: min(total, ranges_count)].tolist())
    return [(c * rsz, min(c * rsz + rsz - 1, file_size - 1)) for c in chosen]
