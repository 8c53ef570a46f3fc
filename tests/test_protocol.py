"""§8f rows 2 and 4: one-pass PUT CRCs (ambrycrc_put_crcs) and the router chunk CRC composition.

The PutRequest field layout is restated for the checker from
ambry-protocol/.../PutRequest.java:244-258 (prepareBuffer, version V5):
blobId bytes, BlobPropertiesSerDe, int umLen, um, short blobType, short keyLen,
key, byte isCompressed, long blobSize -- then the blob."""
import struct
import zlib

import numpy as np
import pytest

from datagen import stream_bytes
from test_message_format import MF


def put_request_fields(blob_id: bytes, props: bytes, um: bytes, blob_type: int, key: bytes, compressed: bool,
                       blob_size: int) -> bytes:
    return (blob_id + props + struct.pack(">i", len(um)) + um + struct.pack(">hh", blob_type, len(key)) + key +
            struct.pack(">bq", 1 if compressed else 0, blob_size))


def make_requests(n=20, seed=3):
    rng = np.random.default_rng(seed)
    reqs = []
    for i in range(n):
        size = int(rng.integers(0, 300000))
        blob = stream_bytes(seed * 7919 + i, 0, size).tobytes()
        key = stream_bytes(i, 1, 32 if i % 2 else 0).tobytes()
        fields = put_request_fields(stream_bytes(i, 2, 40).tobytes(), MF.blob_properties_bytes(size),
                                    stream_bytes(i, 3, int(rng.integers(0, 2000))).tobytes(), i % 3, key,
                                    bool(i % 4 == 0), size)
        reqs.append((fields, blob, bool(i % 4 == 0), i % 3))
    return reqs


def test_put_crcs_one_pass_host(ambry):
    from ambry_amd.protocol import blob_record_prefix_v3, put_crcs

    reqs = make_requests()
    prefixes = [blob_record_prefix_v3(len(b), t, c) for _, b, c, t in reqs]
    wire, rec = put_crcs([f for f, _, _, _ in reqs], prefixes, [zlib.crc32(b) for _, b, _, _ in reqs],
                         [len(b) for _, b, _, _ in reqs])
    assert wire == [zlib.crc32(f + b) for f, b, _, _ in reqs]
    assert rec == [zlib.crc32(p + b) for p, (_, b, _, _) in zip(prefixes, reqs)]
    # the record CRC is exactly what the message-format oracle stores for the blob record
    for (f, b, c, t), r in zip(reqs[:5], rec[:5]):
        assert struct.unpack(">q", MF.blob_record(b, 3, t, c)[-8:])[0] == r


def test_chunk_crc_slices_and_mutation(ambry):
    """PutOperationTest.java:575-679: CRC over slices == CRC of the chunk; a buffer mutated after
    the fill no longer verifies."""
    from ambry_amd.protocol import ChunkCrc

    data = bytearray(stream_bytes(99, 0, 4 << 20).tobytes())
    rng = np.random.default_rng(1)
    cuts = sorted(set([0, len(data)] + rng.integers(0, len(data), size=30).tolist()))
    cc = ChunkCrc()
    for a, b in zip(cuts, cuts[1:]):
        cc.fill_from(bytes(data[a:b]))
    assert cc.getValue() == zlib.crc32(bytes(data)) and cc.length == len(data)
    small = ChunkCrc()
    chunk = bytearray(b"0123456789")  # chunkSize = 10 (PutOperationTest.java:81)
    small.fill_from(bytes(chunk))
    chunk[3] ^= 0xFF
    assert small.getValue() != zlib.crc32(bytes(chunk))
    empty = ChunkCrc()
    assert empty.getValue() == 0  # empty content (PutOperationTest.java:1082-1108)


@pytest.mark.gpu
def test_put_crcs_with_device_blob_pass(gpu):
    import torch

    from ambry_amd.protocol import blob_record_prefix_v3, put_crcs

    reqs = make_requests(n=40, seed=5)
    blobs = [b for _, b, _, _ in reqs]
    off = np.concatenate([[0], np.cumsum([len(b) for b in blobs])[:-1]]).astype(np.int64)
    region = torch.from_numpy(np.frombuffer(b"".join(blobs) + b"\0", dtype=np.uint8).copy()).cuda()
    crcs = gpu.crc32_batch(region, torch.from_numpy(off).cuda(),
                           torch.tensor([len(b) for b in blobs], dtype=torch.int64, device="cuda"))
    blob_crcs = crcs.cpu().numpy().view(np.uint32).tolist()
    prefixes = [blob_record_prefix_v3(len(b), t, c) for _, b, c, t in reqs]
    wire, rec = put_crcs([f for f, _, _, _ in reqs], prefixes, blob_crcs, [len(b) for b in blobs])
    assert wire == [zlib.crc32(f + b) for f, b, _, _ in reqs]
    assert rec == [zlib.crc32(p + b) for p, b in zip(prefixes, blobs)]


@pytest.mark.gpu
def test_verify_chunks_device(gpu):
    import torch

    from ambry_amd.protocol import verify_chunks_device

    n, size = 64, 1 << 20
    data = bytearray(stream_bytes(7, 0, n * size).tobytes())
    stored = [zlib.crc32(bytes(data[i * size:(i + 1) * size])) for i in range(n)]
    for i in (3, 17, 40):
        data[i * size + 12345] ^= 0x08  # mutated after fill (PutOperationTest.java:664-668)
    base = torch.from_numpy(np.frombuffer(bytes(data), dtype=np.uint8).copy()).cuda()
    off = torch.arange(n, dtype=torch.int64, device="cuda") * size
    ln = torch.full((n,), size, dtype=torch.int64, device="cuda")
    ok = verify_chunks_device(base, off, ln, stored)
    assert [i for i, m in enumerate(ok) if not m] == [3, 17, 40]


def test_hard_delete_records_match_oracle(ambry):
    """HardDeleteMessageFormatInputStream.java:58-124: records rewritten with zero bytes and fresh
    CRCs; ambrycrc_zeros gives the same CRCs as scanning the zeros (oracle layouts + zlib), and a
    hard-deleted PUT message still verifies clean (oracle), as BlobStoreRecovery would see it."""
    import importlib.util
    import os

    from ambry_amd.protocol import hard_delete_records

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("mf", os.path.join(root, "oracle", "message_format.py"))
    mf = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mf)
    for um_size, blob_size in ((0, 0), (1, 1), (1000, 65536), (7, 4 << 20), (4096, 1 << 20)):
        for ver in (2, 3):
            um, bl = hard_delete_records(um_size, blob_size, blob_version=ver)
            assert um == mf.usermeta_record(bytes(um_size))
            assert bl == mf.blob_record(bytes(blob_size), version=ver)
            um2, bl2 = hard_delete_records(um_size, blob_size, blob_version=ver, zero_fill=False)
            assert um2[-8:] == um[-8:] and bl2[-8:] == bl[-8:]
    # a PUT message hard-deleted in place: same layout, zeroed user metadata and blob
    key = mf.store_key("hd")
    content = bytes(range(256)) * 300
    msg = bytearray(mf.put_message(key, mf.blob_properties_bytes(len(content)), b"meta" * 50, content))
    v, total, rel = mf.parse_header(bytes(msg), 0)
    um, bl = hard_delete_records(200, len(content))
    msg[rel[3]:rel[3] + len(um)] = um
    msg[rel[4]:rel[4] + len(bl)] = bl
    assert mf.verify_message(bytes(msg), 0) == (0, len(msg))
