"""C1 (BASELINE.json configs[0]): one 64 KiB-blob PUT message through the messageformat CRCs.

The fixture's record CRCs come from zlib (tests/golden/make_golden.py); the product's host path
(ambrycrc_update per record, ambrycrc_put_crcs deriving the blob record's CRC from the blob's,
PutMessageFormatInputStream.java:116-120), the oracle and the GPU message verify must all give
them. Shape of MessageFormatInputStreamTest.java:70-243 (serialize, then check every record)."""
import ctypes
import struct

import numpy as np
import pytest

from c1_message import c1_fixture, c1_message_bytes, c1_record_ranges


def test_c1_fixture_consistent():
    fx = c1_fixture()
    msg = c1_message_bytes()
    ranges = c1_record_ranges()
    assert [r[0] for r in ranges] == [0, 45, 139, 1153]
    # every record is followed by its stored CRC (a big-endian long, upper 32 bits zero)
    for (a, b), c in zip(ranges, fx["record_crcs"]):
        assert struct.unpack(">q", msg[b:b + 8])[0] == int(c, 16)
    assert struct.unpack(">h", msg[:2])[0] == 3 and msg[40:45] == b"\x00\x03id1"


def test_c1_product_host_path(ambry):
    """ambrycrc_update per record; the blob record from ambrycrc_put_crcs over the 13-B prefix."""
    L = ambry.lib()
    msg = c1_message_bytes()
    arr = np.frombuffer(msg, dtype=np.uint8)
    base = arr.ctypes.data
    ranges = c1_record_ranges()
    exp = [int(c, 16) for c in c1_fixture()["record_crcs"]]
    got = [L.ambrycrc_update(0, base + a, b - a) for a, b in ranges]
    assert got == exp
    a, b = ranges[-1]
    blob_crc = L.ambrycrc_update(0, base + a + 13, b - a - 13)
    rec = (ctypes.c_uint32 * 1)()
    rc = L.ambrycrc_put_crcs(None, None, (ctypes.c_void_p * 1)(base + a), (ctypes.c_uint64 * 1)(13),
                             (ctypes.c_uint32 * 1)(blob_crc), (ctypes.c_uint64 * 1)(b - a - 13), 1, None, rec)
    assert rc == 0 and rec[0] == exp[-1]
    # streaming in pieces (CrcInputStream reads) gives the same value
    c = 0
    for lo in range(a, b, 4093):
        c = L.ambrycrc_update(c, base + lo, min(4093, b - lo))
    assert c == exp[-1]
    # the host message chain (BlobStoreRecovery's hop) finds the one message
    from ambry_amd import device as D

    assert D.chain_messages_host(msg) == [0]


def test_c1_oracle(oracle):
    msg = c1_message_bytes()
    arr = np.frombuffer(msg, dtype=np.uint8)
    exp = [int(c, 16) for c in c1_fixture()["record_crcs"]]
    assert [oracle.crc32(arr[a:b]) for a, b in c1_record_ranges()] == exp


@pytest.mark.gpu
def test_c1_device_message_verify(gpu):
    """ambrycrc_verify_messages_dev on the C1 message: clean -> 0; a flipped byte in each record
    -> that record's status bit; the message end is its length."""
    import torch

    msg = c1_message_bytes()
    bits = [1 << 0, 1 << 2, 1 << 4, 1 << 5]  # header, properties, user metadata, blob
    regions = [msg]
    for (a, b), _ in zip(c1_record_ranges(), bits):
        m = bytearray(msg)
        m[(a + b) // 2] ^= 0x10
        regions.append(bytes(m))
    region = b"".join(regions)
    offs = [i * len(msg) for i in range(len(regions))]
    dev = torch.frombuffer(bytearray(region), dtype=torch.uint8).cuda()
    status, end = gpu.verify_messages(dev, torch.tensor(offs, dtype=torch.int64, device="cuda"))
    torch.cuda.synchronize()
    st = status.cpu().numpy().view(np.uint32).tolist()
    assert st == [0] + bits
    assert int(end[0]) == len(msg)
    # the host-staged form agrees
    st_h, end_h = gpu.verify_messages_host(region, offs)
    assert st_h.tolist() == st
