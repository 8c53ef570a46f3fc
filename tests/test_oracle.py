"""The CPU oracle (oracle/crc32_ref.c) pinned against the reference's table and the golden vectors.

Mirrors the reference's own CRC tests:
  Crc32Test.crcTest                 ambry-utils/src/test/java/com/github/ambry/utils/Crc32Test.java:26-41
  CrcInputStreamTest / CrcOutputStreamTest split-vs-bulk equivalence (:43-51 in each)
"""
import ctypes
import hashlib
import struct
import zlib

import numpy as np

from datagen import stream_bytes


def test_table_matches_reference_fingerprint(oracle, fingerprint):
    t = (ctypes.c_uint32 * 2048)()
    oracle.L.oracle_crc32_tables(t)
    packed = struct.pack("<2048I", *t)
    assert f"0x{zlib.crc32(packed):08x}" == fingerprint["zlib_crc32"]
    assert hashlib.sha256(packed).hexdigest() == fingerprint["sha256"]
    assert [f"0x{t[k * 256 + 1]:08x}" for k in range(8)] == fingerprint["T8_k_1"]
    assert [f"0x{t[k * 256 + 255]:08x}" for k in range(8)] == fingerprint["T8_k_255"]


def test_known_answers(oracle, vectors):
    for v in vectors["known_answers"] + vectors["message_headers"]:
        data = bytes.fromhex(v["hex"])
        assert oracle.crc32(data) == int(v["crc"], 16), v["name"]
        assert oracle.crc32_bytewise(data) == int(v["crc"], 16), v["name"]


def test_zero_runs(oracle, vectors):
    for v in vectors["zero_runs"]:
        assert oracle.crc32(bytes(v["len"])) == int(v["crc"], 16)


def test_random_vectors(oracle, vectors):
    for v in vectors["random"]:
        data = stream_bytes(int(v["seed"], 16), v["offset"], v["len"])
        assert oracle.crc32(data, int(v["crc_in"], 16)) == int(v["crc"], 16), v


def test_matches_zlib_all_small_lengths(oracle):
    data = stream_bytes(7, 0, 4096).tobytes()
    for n in range(0, 600):
        assert oracle.crc32(data[:n]) == zlib.crc32(data[:n])
        assert oracle.crc32(data[3:3 + n], 0xDEADBEEF) == zlib.crc32(data[3:3 + n], 0xDEADBEEF)


def test_object_model_crc_test(oracle):
    """Crc32Test.crcTest: same bytes -> same value; flipping the last byte changes it."""
    buf = bytearray(stream_bytes(42, 0, 4000).tobytes())
    state = ctypes.c_uint32()
    vals = []
    for flip in (False, False, True):
        if flip:
            buf[3999] = (~buf[3999]) & 0xFF
        oracle.L.oracle_crc32_reset(ctypes.byref(state))
        a = np.frombuffer(bytes(buf), dtype=np.uint8)
        oracle.L.oracle_crc32_update_bytes(ctypes.byref(state), a.ctypes.data_as(ctypes.c_void_p), 0, 4000)
        vals.append(oracle.L.oracle_crc32_get_value(ctypes.byref(state)))
    assert vals[0] == vals[1] == zlib.crc32(bytes(buf[:3999]) + bytes([(~buf[3999]) & 0xFF]))
    assert vals[2] != vals[0]


def test_split_updates_equal_bulk(oracle):
    """CrcInputStreamTest/CrcOutputStreamTest: split reads/writes give the bulk CRC."""
    data = stream_bytes(5, 0, 4000).tobytes()
    state = ctypes.c_uint32()
    oracle.L.oracle_crc32_reset(ctypes.byref(state))
    a = np.frombuffer(data, dtype=np.uint8)
    p = a.ctypes.data_as(ctypes.c_void_p)
    oracle.L.oracle_crc32_update_bytes(ctypes.byref(state), p, 0, 1000)
    for i in range(1000, 1010):
        oracle.L.oracle_crc32_update_byte(ctypes.byref(state), data[i])
    oracle.L.oracle_crc32_update_bytes(ctypes.byref(state), p, 1010, 2990)
    assert oracle.L.oracle_crc32_get_value(ctypes.byref(state)) == zlib.crc32(data)


def test_combine_restatement(oracle):
    data = stream_bytes(9, 0, 70000).tobytes()
    for cut in (0, 1, 17, 1024, 65536, 70000):
        a, b = data[:cut], data[cut:]
        assert oracle.combine(zlib.crc32(a), zlib.crc32(b), len(b)) == zlib.crc32(data)


def test_batch_threads(oracle):
    mem = stream_bytes(11, 0, 1 << 20)
    off = np.array([0, 5, 1000, 77777, 500000], dtype=np.uint64)
    ln = np.array([0, 100, 65536, 3, 500000], dtype=np.uint64)
    exp = [zlib.crc32(mem[o:o + n].tobytes()) for o, n in zip(off, ln)]
    for th in (1, 3):
        assert list(oracle.batch(mem, off, ln, threads=th)) == exp


def test_zlib_batch_matches_restatement(oracle):
    """oracle_zlib_batch (system zlib crc32_z, the java.util.zip.CRC32 stand-in timed by bench.py's
    cpu_baseline) and the Crc32.java restatement agree chunk for chunk, with and without crc_in."""
    import numpy as np

    from datagen import stream_bytes

    rng = np.random.default_rng(5)
    mem = stream_bytes(8, 0, 1 << 20)
    ln = rng.integers(0, 70000, size=200)
    off = rng.integers(0, (1 << 20) - 70000, size=200)
    cin = rng.integers(0, 1 << 32, size=200, dtype=np.uint64).astype(np.uint32)
    for c in (None, cin):
        for th in (1, 4):
            assert np.array_equal(oracle.batch(mem, off, ln, crc_in=c, threads=th, zlib=True),
                                  oracle.batch(mem, off, ln, crc_in=c, threads=th))
