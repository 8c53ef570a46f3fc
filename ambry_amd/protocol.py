"""PUT-path compositions over libambrycrc (§8f rows 2 and 4).

Row 2 -- one pass over the blob for both PUT CRCs: the PutRequest wire CRC
(ambry-protocol/.../PutRequest.java:238-283, checked on receive at :497-521) and
the Blob_Format_V3 record CRC the server writes (MessageFormatRecord.java:1789-1795,
PutMessageFormatInputStream.java:116-120) both end in the same blob bytes, so
crc(fields || blob) and crc(prefix || blob) come from crc(blob) by GF(2) combine
(ambrycrc_put_crcs).

Row 4 -- router chunk CRC (PutOperation.PutChunk, ambry-router/.../PutOperation.java:
1228 chunkCrc32, 1700-1703 fillFrom, 2033-2054 verifyCRC): slices are CRC'd as
they arrive and merged with combine; verifyCRC for every chunk in flight is one
device batch instead of a host re-scan per chunk.
"""
from __future__ import annotations

import ctypes
import struct
from typing import Sequence

from ._lib import check, lib
from .crc32 import combine, crc32


def blob_record_prefix_v3(blob_size: int, blob_type: int = 0, compressed: bool = False) -> bytes:
    """Blob_Format_V3.serializePartialBlobRecord (MessageFormatRecord.java:1789-1795): 13 bytes."""
    return struct.pack(">hhbq", 3, blob_type, 1 if compressed else 0, blob_size)


def put_crcs(fields: Sequence[bytes], prefixes: Sequence[bytes], blob_crcs: Sequence[int],
             blob_lens: Sequence[int]) -> tuple[list[int], list[int]]:
    """(wire CRCs, blob-record CRCs) from per-request field bytes, record prefixes and blob CRCs."""
    n = len(blob_crcs)
    keep = []

    def arr(items):
        ptrs = (ctypes.c_void_p * n)()
        lens = (ctypes.c_uint64 * n)()
        for i, b in enumerate(items):
            buf = ctypes.create_string_buffer(bytes(b), max(1, len(b)))
            keep.append(buf)
            ptrs[i] = ctypes.cast(buf, ctypes.c_void_p)
            lens[i] = len(b)
        return ptrs, lens

    fp, fl = arr(fields)
    pp, pl = arr(prefixes)
    bc = (ctypes.c_uint32 * n)(*[int(c) & 0xFFFFFFFF for c in blob_crcs])
    bl = (ctypes.c_uint64 * n)(*[int(x) for x in blob_lens])
    wire = (ctypes.c_uint32 * n)()
    rec = (ctypes.c_uint32 * n)()
    check(lib().ambrycrc_put_crcs(fp, fl, pp, pl, bc, bl, n, wire, rec), "ambrycrc_put_crcs")
    return list(wire), list(rec)


class ChunkCrc:
    """PutChunk.chunkCrc32 (PutOperation.java:1228): streaming CRC of a router chunk's slices.

    fill_from(slice) mirrors `chunkCrc32.update(slice.nioBuffer())` (:1700-1703); each slice
    may be CRC'd anywhere (host, or a device batch) and merged in order with combine.
    """

    def __init__(self) -> None:
        self.value = 0
        self.length = 0

    def fill_from(self, data) -> None:
        self.add_slice_crc(crc32(data), memoryview(data).nbytes)

    def add_slice_crc(self, slice_crc: int, slice_len: int) -> None:
        self.value = combine(self.value, slice_crc, slice_len)
        self.length += slice_len

    def getValue(self) -> int:
        return self.value & 0xFFFFFFFF


def verify_chunks_device(base, off, length, stored_crcs):
    """verifyCRC (PutOperation.java:2033-2054) for many chunks at once on the GPU.

    Returns a bool list `matches` (False -> RouterErrorCode.BlobCorrupted)."""
    import numpy as np
    import torch

    from . import device as D

    exp = torch.from_numpy(np.asarray(stored_crcs, dtype=np.uint32).view(np.int32)).to(base.device)
    _, mismatch, _ = D.crc32_verify(base, off, length, exp)
    return [not bool(x) for x in mismatch.cpu().tolist()]


# ---- hard delete (HardDeleteMessageFormatInputStream, ambry-messageformat/.../
# HardDeleteMessageFormatInputStream.java:58-124): the user-metadata record is rewritten with
# `userMetadataSize` zero bytes and the blob record with `blobStreamSize` zero bytes
# (ZeroBytesInputStream), each with a fresh CRC. The zero runs are never scanned: the CRC of
# `prefix || 0^n` is ambrycrc_zeros(crc(prefix), n), a GF(2) shift (log2 n multiplies).


def _crc_long(v: int) -> bytes:
    return struct.pack(">q", v & 0xFFFFFFFF)


def hard_delete_records(usermeta_size: int, blob_size: int, blob_version: int = 3, blob_type: int = 0,
                        zero_fill: bool = True) -> tuple[bytes, bytes]:
    """(user-metadata record, blob record) as the hard-delete stream writes them.

    UserMetadata_Format_V1 (MessageFormatRecord.java:1603-1635): version(2) size(4) zeros crc(8).
    Blob_Format_V2/V3 (:1717-1755, :1777-1795): prefix, zeros, crc(8); V3 isCompressed = false.
    zero_fill=False returns the records without their zero bodies: (prefix || crc) pairs, for
    callers that write the zeros themselves (a 4 MiB blob needs no 4 MiB buffer to get its CRC)."""
    from .crc32 import zeros

    um_prefix = struct.pack(">hi", 1, usermeta_size)
    um_crc = zeros(crc32(um_prefix), usermeta_size)
    if blob_version == 2:
        bl_prefix = struct.pack(">hhq", 2, blob_type, blob_size)
    elif blob_version == 3:
        bl_prefix = struct.pack(">hhbq", 3, blob_type, 0, blob_size)
    else:
        raise ValueError(f"blob record version {blob_version}: the hard-delete stream writes V2 or V3 here")
    bl_crc = zeros(crc32(bl_prefix), blob_size)
    if not zero_fill:
        return um_prefix + _crc_long(um_crc), bl_prefix + _crc_long(bl_crc)
    return (um_prefix + bytes(usermeta_size) + _crc_long(um_crc),
            bl_prefix + bytes(blob_size) + _crc_long(bl_crc))
