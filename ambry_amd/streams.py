"""CRC-on-the-fly streams over the native checksum.

Mirrors ``com.github.ambry.utils.CrcInputStream`` / ``CrcOutputStream``
(ambry-utils/src/main/java/com/github/ambry/utils/CrcInputStream.java:27-96,
CrcOutputStream.java:24-62): same method names, argument meaning and results.
The reference types their checksum field as the final class
``java.util.zip.CRC32``; the drop-in retypes it to
``Checksum``, which is what these take: any object with ``update`` /
``getValue`` (by default :class:`ambry_amd.crc32.Crc32`, i.e. ``ambrycrc_update``).

Reference behaviour kept on purpose:
- ``read()`` at end of stream returns -1 and still feeds ``(byte) -1`` (0xFF) to
  the checksum (CrcInputStream.java:47-51);
- ``read(b, off, len)`` at end of stream passes ``len = -1`` to the checksum,
  which the JDK rejects with ``ArrayIndexOutOfBoundsException``; here
  ``IndexError`` (CrcInputStream.java:59-63).
"""
from __future__ import annotations

from .crc32 import ByteBufferLike, Crc32


class CrcInputStream:
    """CrcInputStream(in) / CrcInputStream(crc, in) (CrcInputStream.java:36-43)."""

    def __init__(self, *args) -> None:
        if len(args) == 1:
            self._crc, self._stream = Crc32(), args[0]
        elif len(args) == 2:
            self._crc, self._stream = args
        else:
            raise TypeError("CrcInputStream(in) or CrcInputStream(crc, in)")

    def read(self, b=None, off: int | None = None, length: int | None = None) -> int:
        """read() (:46-51), read(byte[] b) (:53-56), read(b, off, len) (:58-63)."""
        if b is None:
            val = self._stream.read()
            self._crc.update(val & 0xFF)
            return val
        if off is None:
            off, length = 0, len(b)
        ret = self._stream.read(b, off, length)
        if ret < 0:
            raise IndexError("checksum update with len = -1 (end of stream)")
        self._crc.update(b, off, ret)
        return ret

    def updateCrc(self, buffer: ByteBufferLike) -> None:  # :70-72 (consumes the buffer)
        self._crc.update_buffer(buffer)

    def available(self) -> int:  # :74-79
        return self._stream.available()

    def close(self) -> None:  # :81-84
        self._stream.close()

    def getValue(self) -> int:  # :86-88
        return self._crc.getValue()

    def getUnderlyingInputStream(self):  # :94-96
        return self._stream


class CrcOutputStream:
    """CrcOutputStream(out) / CrcOutputStream(crc, out) (CrcOutputStream.java:32-39)."""

    def __init__(self, *args) -> None:
        if len(args) == 1:
            self._crc, self._stream = Crc32(), args[0]
        elif len(args) == 2:
            self._crc, self._stream = args
        else:
            raise TypeError("CrcOutputStream(out) or CrcOutputStream(crc, out)")

    def write(self, b, off: int | None = None, length: int | None = None) -> None:
        """write(int) (:41-45), write(byte[]) (:47-51), write(b, off, len) (:53-57)."""
        if isinstance(b, int):
            self._stream.write(b)
            self._crc.update(b & 0xFF)
            return
        if off is None:
            self._stream.write(b)
            self._crc.update(b, 0, len(b))
            return
        self._stream.write(b, off, length)
        self._crc.update(b, off, length)

    def close(self) -> None:  # :59-62
        self._stream.close()

    def getValue(self) -> int:  # :64-66
        return self._crc.getValue()


class ByteBufferInputStream:
    """Test-side stand-in for com.github.ambry.utils.ByteBufferInputStream over a bytes-like."""

    def __init__(self, data) -> None:
        self._data = bytes(data)
        self._pos = 0

    def read(self, b=None, off: int = 0, length: int | None = None) -> int:
        if b is None:
            if self._pos >= len(self._data):
                return -1
            self._pos += 1
            return self._data[self._pos - 1]
        if length is None:
            length = len(b) - off
        if length == 0:
            return 0
        if self._pos >= len(self._data):
            return -1
        n = min(length, len(self._data) - self._pos)
        b[off:off + n] = self._data[self._pos:self._pos + n]
        self._pos += n
        return n

    def available(self) -> int:
        return len(self._data) - self._pos

    def close(self) -> None:
        pass


class ByteBufferOutputStream:
    """Test-side stand-in for com.github.ambry.utils.ByteBufferOutputStream over a bytearray."""

    def __init__(self, buf: bytearray) -> None:
        self._buf = buf
        self._pos = 0

    def write(self, b, off: int | None = None, length: int | None = None) -> None:
        if isinstance(b, int):
            self._buf[self._pos] = b & 0xFF
            self._pos += 1
            return
        if off is None:
            off, length = 0, len(b)
        if self._pos + length > len(self._buf):
            raise IndexError("buffer overflow")
        self._buf[self._pos:self._pos + length] = bytes(b[off:off + length])
        self._pos += length

    def close(self) -> None:
        pass
