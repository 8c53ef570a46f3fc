"""§8f next #1 -- message-level verify: oracle/message_format.py (CPU restatement of the
record layouts) pinned against the reference tests' deterministic headers, and the
host-side message chain of libambrycrc checked against it."""
import struct
import zlib

import numpy as np
import pytest

from datagen import stream_bytes

import importlib.util
import os

_spec = importlib.util.spec_from_file_location(
    "message_format", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle",
                                   "message_format.py"))
MF = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(MF)


def build_region(n=300, seed=7, corrupt_frac=0.1, big_every=17):
    """A log region of PUT (V1/V2/V3, +/- encryption key) and update messages, some corrupted.
    Returns (region bytes, message offsets, expected status list from the oracle)."""
    rng = np.random.default_rng(seed)
    out = bytearray()
    offs = []
    for i in range(n):
        key = MF.store_key(f"blob-{i:06d}-{seed}")
        kind = rng.integers(0, 10)
        if kind == 0:
            msg = MF.update_message(key, version=3, kind=["ttl", "delete", "undelete"][i % 3])
        else:
            ver = [1, 2, 3, 3][int(rng.integers(0, 4))]
            size = int(rng.integers(0, 5000)) if i % big_every else int(rng.integers(60000, 300000))
            content = stream_bytes(seed * 100003 + i, 0, size).tobytes()
            um = stream_bytes(seed + i, 7, int(rng.integers(0, 1200))).tobytes()
            enc = stream_bytes(i, 3, 100).tobytes() if (ver >= 2 and i % 2) else None
            msg = MF.put_message(key, MF.blob_properties_bytes(size), um, content, version=ver, enc_key=enc,
                                 life=int(i % 3), compressed=bool(i % 5 == 0))
        offs.append(len(out))
        out += msg
    region = bytearray(out)
    for i in rng.choice(n, size=int(n * corrupt_frac), replace=False):
        start = offs[i]
        end = offs[i + 1] if i + 1 < n else len(region)
        pos = int(rng.integers(start, end))
        region[pos] ^= 1 << int(rng.integers(0, 8))
    region = bytes(region)
    expect = [MF.verify_message(region, o) for o in offs]
    return region, offs, expect


def test_oracle_headers_match_golden(vectors):
    hv = {h["name"]: h for h in vectors["message_headers"]}
    h1 = MF.header(1, 1000, -1, 10, -1, 20, 30)
    assert h1[:26].hex() == hv["MessageHeader_Format_V1 (MessageFormatRecordTest.java:70)"]["hex"]
    assert struct.unpack(">q", h1[26:])[0] == int(hv["MessageHeader_Format_V1 (MessageFormatRecordTest.java:70)"]["crc"], 16)
    h3 = MF.header(3, 1000, 5, 10, -1, 20, 30, life=2)
    assert h3[:32].hex() == hv["MessageHeader_Format_V3 (MessageFormatRecordTest.java:115)"]["hex"]
    assert struct.unpack(">q", h3[32:])[0] == 0xA4893031


def test_clean_messages_verify_and_chain(ambry):
    region, offs, expect = build_region(n=120, corrupt_frac=0.0)
    assert all(s == 0 for s, _ in expect)
    ends = [e for _, e in expect]
    assert ends[:-1] == offs[1:] and ends[-1] == len(region)
    from ambry_amd.device import chain_messages_host

    assert chain_messages_host(region, 0) == offs


def test_oracle_detects_every_single_bit_flip():
    """MessageFormatRecordTest.deserializeTest / BlobStoreRecoveryTest.crcErrorRecoveryTest: one corrupted byte
    anywhere in a message is reported (header bit, a record bit, or a layout error) -- except inside the
    store key, which Ambry's format does not cover with any CRC (the key is validated by StoreKeyFactory)."""
    key = MF.store_key("id1")
    msg = MF.put_message(key, MF.blob_properties_bytes(4096), b"u" * 1000, stream_bytes(1, 0, 4096).tobytes(),
                         version=3, enc_key=b"k" * 100)
    assert MF.verify_message(msg, 0) == (0, len(msg))
    rng = np.random.default_rng(0)
    key_span = range(40, 40 + len(key))
    for pos in list(range(0, 200)) + list(rng.integers(200, len(msg), size=200)):
        bad = bytearray(msg)
        bad[pos] ^= 0x10
        st, _ = MF.verify_message(bytes(bad), 0)
        assert (st == 0) == (pos in key_span), pos


def test_chain_stops_at_corrupt_header(ambry):
    region, offs, _ = build_region(n=40, corrupt_frac=0.0)
    bad = bytearray(region)
    bad[offs[25] + 3] ^= 0xFF
    from ambry_amd.device import chain_messages_host

    assert chain_messages_host(bytes(bad), 0) == offs[:25]


def _seal(body: bytes) -> bytes:
    return body + struct.pack(">q", zlib.crc32(body))


def _assemble(version, key, enc, pr, um, bl, upd=None):
    """A message from already-sealed records (header offsets from their lengths, header CRC valid)."""
    h = MF.HEADER_SIZE[version]
    if upd is not None:
        return MF.header(version, len(upd), MF.INVALID, MF.INVALID, h + len(key), MF.INVALID, MF.INVALID) + key + upd
    enc = enc or b""
    bp = h + len(key) + len(enc)
    total = len(enc) + len(pr) + len(um) + len(bl)
    return MF.header(version, total, h + len(key) if enc else MF.INVALID, bp, MF.INVALID, bp + len(pr),
                     bp + len(pr) + len(um)) + key + enc + pr + um + bl


def record_level_cases():
    """(message, expected status) pairs whose every CRC is valid but whose record fields are not
    what the reference's deserializers accept (MessageFormatRecord.java:147-239, 1588-1833):
    unknown record versions -> BAD_VERSION; size fields that disagree with the header's record
    span, blob type ordinals >= 2, blob sizes > Integer.MAX_VALUE -> BAD_RECORD."""
    key = MF.store_key("rec-level")
    props = MF.blob_properties_bytes(300)
    content = bytes(range(200)) + bytes(100)
    ek = b"e" * 32
    pr, um = MF.props_record(props), MF.usermeta_record(b"meta" * 5)
    bl, enc = MF.blob_record(content), MF.enckey_record(ek)
    cases = [
        (_assemble(3, key, enc, pr, um, bl), 0),
        (_assemble(2, key, None, pr, um, MF.blob_record_v1(content)), 0),
        (_assemble(3, key, None, pr, um, MF.blob_record(content, version=2, blob_type=1)), 0),
        (_assemble(3, key, _seal(struct.pack(">hi", 2, len(ek)) + ek), pr, um, bl), MF.BAD_VERSION),
        (_assemble(3, key, _seal(struct.pack(">hi", 1, len(ek) + 1) + ek), pr, um, bl), MF.BAD_RECORD),
        (_assemble(3, key, None, _seal(struct.pack(">h", 2) + props), um, bl), MF.BAD_VERSION),
        (_assemble(3, key, None, pr, _seal(struct.pack(">hi", 0, 20) + b"meta" * 5), bl), MF.BAD_VERSION),
        (_assemble(3, key, None, pr, _seal(struct.pack(">hi", 1, 19) + b"meta" * 5), bl), MF.BAD_RECORD),
        (_assemble(3, key, None, pr, _seal(struct.pack(">hi", 1, -4) + b"meta" * 5), bl), MF.BAD_RECORD),
        (_assemble(3, key, None, pr, um, _seal(struct.pack(">hhbq", 3, 2, 0, len(content)) + content)),
         MF.BAD_RECORD),
        (_assemble(3, key, None, pr, um, _seal(struct.pack(">hhbq", 4, 0, 0, len(content)) + content)),
         MF.BAD_VERSION),
        (_assemble(3, key, None, pr, um, _seal(struct.pack(">hhbq", 3, 0, 0, len(content) - 1) + content)),
         MF.BAD_RECORD),
        (_assemble(3, key, None, pr, um, _seal(struct.pack(">hhbq", 3, 0, 0, len(content) + (1 << 32)) + content)),
         MF.BAD_RECORD),
        (_assemble(1, key, None, pr, um, _seal(struct.pack(">hq", 1, len(content) + 3) + content)), MF.BAD_RECORD),
        (_assemble(3, key, None, pr, um, _seal(struct.pack(">hhq", 2, 7, len(content)) + content)), MF.BAD_RECORD),
    ]
    upd = bytearray(MF.update_record_v3())
    upd[0:2] = struct.pack(">h", 4)
    cases.append((_assemble(3, key, None, None, None, None, upd=_seal(bytes(upd[:-8]))), MF.BAD_VERSION))
    cases.append((_assemble(3, key, None, None, None, None, upd=MF.update_record_v3(kind="delete")), 0))
    cases += props_level_cases(key, um, bl) + update_level_cases(key)
    return cases


def _props_msg(key, um, bl, serde: bytes, version=3):
    return _assemble(version, key, None, _seal(struct.pack(">h", 1) + serde), um, bl)


def props_level_cases(key, um, bl):
    """CRC-valid BlobProperties records through BlobPropertiesSerDe.getBlobPropertiesFromStream
    (BlobPropertiesSerDe.java:56-77) under deserializeBlobPropertiesRecord's catch-all
    (MessageFormatRecord.java:1179-1195: any exception -> DataCorrupt = BAD_RECORD)."""
    cases = []
    for v in (1, 2, 3, 4, 5):  # every stored version reads clean
        cases.append((_props_msg(key, um, bl, MF.blob_properties_bytes(
            300, serde_version=v, content_encoding="gzip", filename="f", reserved="r")), 0))
    good = MF.blob_properties_bytes(300, content_encoding="gzip", filename="name.bin")
    for bad_v in (0, 6, 9, -1):  # "stream has unknown blob property version"
        cases.append((_props_msg(key, um, bl, struct.pack(">h", bad_v) + good[2:]), MF.BAD_RECORD))
    # contentType's int size: past the span / negative / one short (the fields end early)
    ct = 27
    for n, want in ((1 << 20, MF.BAD_RECORD), (-2, MF.BAD_RECORD), (0x7FFFFFFF, MF.BAD_RECORD)):
        b = bytearray(good)
        b[ct:ct + 4] = struct.pack(">i", n)
        cases.append((_props_msg(key, um, bl, bytes(b)), want))
    cases.append((_props_msg(key, um, bl, good + b"\0"), MF.BAD_RECORD))  # trailing byte: CRC read early
    cases.append((_props_msg(key, um, bl, good[:-1]), MF.BAD_RECORD))      # last string cut: EOF
    cases.append((_props_msg(key, um, bl, good[:20]), MF.BAD_RECORD))      # inside the fixed fields
    v4 = MF.blob_properties_bytes(300, serde_version=4, filename="abc")
    cases.append((_props_msg(key, um, bl, v4[:-7] + struct.pack(">i", -1) + b"abc"), MF.BAD_RECORD))
    # non-canonical private / encrypted bytes and non-ASCII strings still verify (decoding never throws)
    cases.append((_props_msg(key, um, bl, MF.blob_properties_bytes(300, private=7, encrypted=2)), 0))
    cases.append((_props_msg(key, um, bl, MF.blob_properties_bytes(300, owner_id=b"\xc3\xa9t\xff")), 0))
    return cases


def update_level_cases(key):
    """CRC-valid update records through deserializeUpdateRecord (MessageFormatRecord.java:158-172,
    1217-1228, 1253-1266, 1388-1464)."""
    def upd_msg(body):
        return _assemble(3, key, None, None, None, None, upd=_seal(body))

    base = struct.pack(">hhhq", 3, 101, 5, 1_700_000_000_123)
    return [
        (upd_msg(struct.pack(">hb", 1, 1)), 0),                                  # V1: a delete flag
        (upd_msg(struct.pack(">hb", 1, 1) + b"x"), MF.BAD_RECORD),
        (upd_msg(struct.pack(">hhhq", 2, 101, 5, 7)), 0),                          # V2
        (upd_msg(struct.pack(">hhhq", 2, 101, 5, 7)[:-1]), MF.BAD_RECORD),
        (upd_msg(base + struct.pack(">hhq", 1, 1, 99)), 0),                        # V3 TTL_UPDATE
        (upd_msg(base + struct.pack(">hh", 2, 1)), 0),                             # V3 UNDELETE
        (upd_msg(base + struct.pack(">hh", 3, 1)), MF.BAD_RECORD),                 # Type.values()[3]
        (upd_msg(base + struct.pack(">hh", -1, 1)), MF.BAD_RECORD),
        (upd_msg(base + struct.pack(">hh", 0, 2)), MF.BAD_VERSION),                # delete sub-record v2
        (upd_msg(base + struct.pack(">hhq", 1, 0, 99)), MF.BAD_VERSION),           # ttl sub-record v0
        (upd_msg(base + struct.pack(">hh", 0, 1) + bytes(8)), MF.BAD_RECORD),      # delete + 8 stray bytes
        (upd_msg(base + struct.pack(">hh", 1, 1)), MF.BAD_RECORD),                 # TTL without its expiry
        (upd_msg(base), MF.BAD_RECORD),                                          # no type
        (upd_msg(struct.pack(">hhhq", 0, 1, 1, 1) + bytes(2)), MF.BAD_VERSION),
    ]


def test_blob_properties_versions_match_reference_test():
    """BlobPropertiesTest.basicTest (ambry-messageformat/src/test/.../BlobPropertiesTest.java:68-202)
    restated over the layouts its serializeBlobPropertiesInVersion writes (:209-275): what
    getBlobPropertiesFromStream must return at each version -- account/container UNKNOWN (-1) at
    V1, `encrypted` only from V3, contentEncoding/filename only from V4, the reserved metadata id
    only at V5, null owner/contentType read back as "" (readIntString) and null nullable strings
    as null -- and the V5 re-serialization (serializeBlobProperties, BlobPropertiesSerDe.java:83-103)."""
    acct, cont, ttl, ctime = 1234, -77, 144, 1_700_000_000_555
    for v in (1, 2, 3, 4, 5):
        for enc in (False, True):
            ce, fn = ("gzip", "filename") if v >= 4 else (None, None)
            raw = MF.blob_properties_bytes(100, service_id="ServiceId", owner_id="OwnerId", content_type="ContentType",
                                           ttl=ttl, private=True, creation_ms=ctime, account=acct, container=cont,
                                           encrypted=enc, content_encoding=ce, filename=fn, reserved="blobid",
                                           serde_version=v)
            f, end = MF.parse_blob_properties(raw, 0, len(raw))
            assert end == len(raw)
            assert (f["size"], f["service"], f["owner"], f["content_type"]) == (100, b"ServiceId", b"OwnerId",
                                                                                b"ContentType")
            assert (f["private"], f["ttl"], f["creation"]) == (True, ttl, ctime)
            assert (f["account"], f["container"]) == ((acct, cont) if v > 1 else (-1, -1))
            assert f["encrypted"] == (v >= 3 and enc)
            assert (f["content_encoding"], f["filename"]) == ((b"gzip", b"filename") if v >= 4 else (None, None))
            assert f["reserved"] == (b"blobid" if v == 5 else None)
            v5 = MF.serialize_blob_properties_v5(f)
            g, _ = MF.parse_blob_properties(v5, 0, len(v5))
            assert {k: x for k, x in g.items() if k != "version"} == {k: x for k, x in f.items() if k != "version"}
            assert v5 == MF.blob_properties_bytes(100, service_id="ServiceId", owner_id="OwnerId",
                                                  content_type="ContentType", ttl=ttl, private=True, creation_ms=ctime,
                                                  account=f["account"], container=f["container"],
                                                  encrypted=f["encrypted"], content_encoding=ce, filename=fn,
                                                  reserved="blobid" if v == 5 else None)
    # null owner / contentType serialize as int 0 and read back as "" (not null): the same bytes
    raw = MF.blob_properties_bytes(100, owner_id=None, content_type=None, serde_version=2)
    f, _ = MF.parse_blob_properties(raw, 0, len(raw))
    assert f["owner"] == b"" and f["content_type"] == b""
    assert MF.serialize_blob_properties_v5(f)[27:35] == bytes(8)


def test_props_not_encodable():
    for s in (b"\x80", b"caf\xc3\xa9", b"\xf0\x9f\x98\x80"):
        raw = MF.blob_properties_bytes(1, filename=s)
        f, _ = MF.parse_blob_properties(raw, 0, len(raw))
        with pytest.raises(MF.NotEncodable):
            MF.serialize_blob_properties_v5(f)


def test_oracle_record_level_checks():
    for i, (msg, want) in enumerate(record_level_cases()):
        assert MF.verify_message(msg, 0) == (want, len(msg)), i
