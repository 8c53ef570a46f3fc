"""Host-side mirror of Ambry's checksum interface over libambrycrc.

``Crc32`` mirrors ``com.github.ambry.utils.Crc32`` (ambry-utils/src/main/java/
com/github/ambry/utils/Crc32.java), which implements ``java.util.zip.Checksum``:
same method names, same argument meaning, same ``getValue()`` range
(unsigned 32-bit in a Python int, Java's ``long``). Small updates run on the
host through ``ambrycrc_update``; device batches go through
``crc32_batch`` / ``crc32_verify`` (the gfx950 kernels).
"""
from __future__ import annotations

import ctypes

from ._lib import check, lib

_MASK = 0xFFFFFFFF


def _buffer_ptr(data, off: int, length: int):
    """(pointer, keepalive) for bytes/bytearray/memoryview/numpy data."""
    mv = memoryview(data).cast("B")
    if off < 0 or length < 0 or off + length > mv.nbytes:
        raise IndexError(f"off={off} len={length} outside buffer of {mv.nbytes} bytes")
    if length == 0:
        return None, None
    if mv.readonly:
        buf = (ctypes.c_char * length).from_buffer_copy(mv[off:off + length])
        return ctypes.cast(buf, ctypes.c_void_p), buf
    buf = (ctypes.c_char * mv.nbytes).from_buffer(mv)
    return ctypes.c_void_p(ctypes.addressof(buf) + off), buf


class Crc32:
    """Drop-in mirror of com.github.ambry.utils.Crc32 (Crc32.java:34-149).

    The Java class keeps the bit-flipped register (``crc``, Crc32.java:37);
    this one keeps the finalized value, which is what the C ABI passes around.
    """

    def __init__(self) -> None:  # Crc32.java:40-42
        self._value = 0

    def getValue(self) -> int:  # Crc32.java:44-47
        return self._value & _MASK

    def reset(self) -> None:  # Crc32.java:49-52
        self._value = 0

    def update(self, b, off: int | None = None, length: int | None = None) -> None:
        """update(int b) (Crc32.java:146-148) or update(byte[] b, int off, int len) (:55-98)."""
        if isinstance(b, int):
            self._value = lib().ambrycrc_update_byte(self._value, b)
            return
        if off is None:
            off, length = 0, memoryview(b).nbytes
        ptr, keep = _buffer_ptr(b, off, length)
        if ptr is not None:
            self._value = lib().ambrycrc_update(self._value, ptr, length)
        del keep

    def update_buffers(self, buffers) -> None:
        """update(ByteBuffer) over every buffer in order (PutOperation.java:2041-2043), one native call."""
        bufs = list(buffers)
        n = len(bufs)
        ptrs = (ctypes.c_void_p * n)()
        lens = (ctypes.c_size_t * n)()
        keep = []
        for i, b in enumerate(bufs):
            data = b.array_view()
            ptr, k = _buffer_ptr(data, b.position, b.remaining())
            keep.append(k)
            ptrs[i], lens[i] = ptr, b.remaining()
        self._value = lib().ambrycrc_update_iov(self._value, ptrs, lens, n)
        for b in bufs:
            b.position = b.limit  # each buffer is consumed, as update(ByteBuffer) does
        del keep

    def update_buffer(self, buffer: "ByteBufferLike") -> None:
        """update(ByteBuffer) (Crc32.java:100-143): consumes position..limit."""
        if buffer.remaining() == 0:  # Crc32.java:101-103
            return
        data = buffer.array_view()
        self.update(data, buffer.position, buffer.remaining())
        buffer.position = buffer.limit


class ByteBufferLike:
    """Minimal java.nio.ByteBuffer stand-in (position/limit over a bytes-like)."""

    def __init__(self, data, position: int = 0, limit: int | None = None) -> None:
        self._data = data
        self.position = position
        self.limit = memoryview(data).nbytes if limit is None else limit

    def remaining(self) -> int:
        return self.limit - self.position

    def array_view(self):
        return self._data


def crc32(data, crc: int = 0) -> int:
    """zlib-style crc32(data, crc) on the host path."""
    c = Crc32()
    c._value = crc & _MASK
    c.update(data)
    return c.getValue()


def combine(crc1: int, crc2: int, len2: int) -> int:
    return lib().ambrycrc_combine(crc1 & _MASK, crc2 & _MASK, len2)


def zeros(crc: int, n: int) -> int:
    return lib().ambrycrc_zeros(crc & _MASK, n)
