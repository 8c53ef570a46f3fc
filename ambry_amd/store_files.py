"""CRC-trailered store files over the GPU engine (widening past SURVEY §8f: the persisted-file
checks either side of the log).

Ambry persists several files as ``payload || CRC32(payload) as a big-endian long``:
- index segment files, checked whole at store start-up
  (ambry-store/.../IndexSegment.java:727-735 ``checkDataIntegrityInByteBufferWithCRC``,
  called from ``checkFileDataIntegrity`` :743-758);
- the log segment header ``version(2) | capacity(8) | crc(8)`` (LogSegment.java:130-140, 603-607).

``index_segments_intact`` checks many index segment files in one device batch
(``ambrycrc_verify_trailed_host``) and returns, per file, what the reference's check returns.
``log_segment_header_intact`` is 10 bytes: it runs on the host loop (``ambrycrc_update``).
"""
from __future__ import annotations

import mmap
import os
import struct
from typing import Sequence

from . import device as _device
from .crc32 import crc32 as _crc32

LOG_SEGMENT_HEADER_SIZE = 18  # LogSegment.java:49-53: version 2 + capacity 8 + crc 8


def index_segments_intact(paths: Sequence[str], device: int = 0) -> list[bool]:
    """True per file whose trailing CRC matches (IndexSegment.checkDataIntegrityInByteBufferWithCRC).
    A file shorter than 8 bytes is not intact (the reference's limit(capacity - 8) throws).
    Missing files raise FileNotFoundError, as checkFileDataIntegrity raises FileNotFound."""
    maps, bufs = [], []
    try:
        for p in paths:
            size = os.path.getsize(p)
            if size == 0:
                bufs.append(b"")
                continue
            with open(p, "rb") as f:
                m = mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ)
            maps.append(m)
            bufs.append(memoryview(m))
        bad = _device.verify_trailed_host(bufs, device=device)
        return [not b for b in bad]
    finally:
        del bufs
        for m in maps:
            m.close()


def log_segment_header_intact(header: bytes) -> bool:
    """LogSegment's header check (LogSegment.java:130-140): version 0, CRC of the first 10 bytes
    equals the big-endian long that follows."""
    if len(header) < LOG_SEGMENT_HEADER_SIZE or struct.unpack_from(">h", header, 0)[0] != 0:
        return False
    return _crc32(header[:10]) == struct.unpack_from(">q", header, 10)[0]


def log_segment_header(capacity: int) -> bytes:
    """LogSegment.writeHeader (LogSegment.java:602-609): version 0, capacity, CRC."""
    body = struct.pack(">hq", 0, capacity)
    return body + struct.pack(">q", _crc32(body))
