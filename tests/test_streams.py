"""CrcInputStream / CrcOutputStream over the native checksum: the reference's own tests
(CrcInputStreamTest.java:27-70, CrcOutputStreamTest.java:27-70) restated, plus the
end-of-stream behaviour of CrcInputStream.java:46-63. Host path only (no GPU)."""
import zlib

import numpy as np
import pytest

from ambry_amd.crc32 import ByteBufferLike, Crc32
from ambry_amd.streams import ByteBufferInputStream, ByteBufferOutputStream, CrcInputStream, CrcOutputStream


def _buf(seed, n=4000):
    return bytearray(np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8).tobytes())


def test_crc_input_stream():  # CrcInputStreamTest.testCrcInputStream
    buf = _buf(1)
    crc_stream = CrcInputStream(ByteBufferInputStream(buf))
    out = bytearray(4000)
    crc_stream.read(out)
    assert out == buf
    value1 = crc_stream.getValue()
    assert value1 == zlib.crc32(bytes(buf))

    crc_stream = CrcInputStream(ByteBufferInputStream(buf))
    out = bytearray(4000)
    crc_stream.read(out, 0, 3999)
    out[3999] = crc_stream.read()
    assert out == buf
    value2 = crc_stream.getValue()
    assert value1 == value2
    assert crc_stream.available() == 0

    buf[3999] = (~buf[3999]) & 0xFF
    crc_stream = CrcInputStream(ByteBufferInputStream(buf))
    out = bytearray(4000)
    crc_stream.read(out, 0, 3999)
    out[3999] = crc_stream.read()
    assert out == buf
    assert crc_stream.getValue() != value2
    crc_stream.close()


def test_crc_output_stream():  # CrcOutputStreamTest.testCrcOutputStream
    data = _buf(2)
    sink = bytearray(4000)
    crc_stream = CrcOutputStream(ByteBufferOutputStream(sink))
    crc_stream.write(data)
    assert sink == data
    value1 = crc_stream.getValue()
    assert value1 == zlib.crc32(bytes(data))

    sink = bytearray(4000)
    crc_stream = CrcOutputStream(ByteBufferOutputStream(sink))
    crc_stream.write(data[0])
    crc_stream.write(data, 1, 3999)
    assert sink == data
    value2 = crc_stream.getValue()
    assert value1 == value2

    data[0] = (~data[0]) & 0xFF
    sink = bytearray(4000)
    crc_stream = CrcOutputStream(ByteBufferOutputStream(sink))
    crc_stream.write(data[0])
    crc_stream.write(data, 1, 3999)
    assert sink == data
    assert crc_stream.getValue() != value2
    crc_stream.close()


def test_end_of_stream_matches_reference():
    """read() at EOF returns -1 and feeds 0xFF to the CRC (CrcInputStream.java:47-51);
    read(b, off, len) at EOF hands len=-1 to CRC32.update, which throws (:59-63)."""
    data = bytes(_buf(3, 100))
    s = CrcInputStream(ByteBufferInputStream(data))
    out = bytearray(100)
    assert s.read(out) == 100
    assert s.read() == -1
    assert s.getValue() == zlib.crc32(b"\xff", zlib.crc32(data))
    with pytest.raises(IndexError):
        s.read(out, 0, 10)


def test_explicit_checksum_and_update_crc():
    """CrcInputStream(crc, in) shares the caller's checksum; updateCrc consumes a buffer
    (the zero-copy Netty path, Utils.java:393,417)."""
    data = bytes(_buf(4, 10000))
    crc = Crc32()
    crc.update(data, 0, 5000)
    s = CrcInputStream(crc, ByteBufferInputStream(data[5000:]))
    out = bytearray(5000)
    assert s.read(out, 0, 5000) == 5000
    assert crc.getValue() == s.getValue() == zlib.crc32(data)
    bb = ByteBufferLike(data, position=1234)
    s2 = CrcInputStream(ByteBufferInputStream(b""))
    s2.updateCrc(bb)
    assert bb.position == bb.limit
    assert s2.getValue() == zlib.crc32(data[1234:])
    assert s2.getUnderlyingInputStream().available() == 0
