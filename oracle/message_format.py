"""oracle/message_format.py -- TEST INFRASTRUCTURE ONLY (never imported by the product).

CPU restatement of Ambry's on-disk/on-wire message record layouts, used to
build fixture log regions and to decide, per message, what
deserializeBlobAll / update-record deserialization would report. It is the
parity checker for ambrycrc_verify_messages_dev.

Restated from ambry-messageformat/src/main/java/com/github/ambry/messageformat/:
  MessageFormatRecord.java
    :44-61     Version_Field_Size_In_Bytes = 2, Crc_Size = 8, header/record versions,
               Message_Header_Invalid_Relative_Offset = -1
    :467-486   MessageHeader_Format_V1.serializeHeader (version, totalSize, 4 relative offsets, CRC)
    :696-725   MessageHeader_Format_V2.serializeHeader (+ encryption-key relative offset)
    :951-981   MessageHeader_Format_V3.serializeHeader (+ lifeVersion)
    :985-1030  checkHeaderConstraints (totalSize > 0, lifeVersion >= 0, put vs update offsets)
    :1132-1145 verifyHeader / verifyCrc: CRC32 over header minus trailing 8 B
    :1162-1195 BlobProperties_Format_V1 (version, BlobPropertiesSerDe bytes, CRC)
    :1322-1379 Update_Format_V3 (version, account, container, updateTime, type, sub-record, CRC)
    :1568-1601 BlobEncryptionKey_Format_V1 (version, int size, key, CRC)
    :1619-1650 UserMetadata_Format_V1 (version, int size, content, CRC)
    :1717-1755 Blob_Format_V2 (version, blobType, long size, content, CRC)
    :1777-1833 Blob_Format_V3 (version, blobType, isCompressed, long size, content, CRC)
    :257-303   deserializeBlobAll: header verified first (corrupt header -> no record parsed),
               then encryption key (if present), blob properties, user metadata, blob.
  PutMessageFormatInputStream.java:76-124,133-162 (record order and relative offsets)
  ValidatingTransformer.java:46-104 (transform: verify, deserialize, re-serialize a PUT)
  BlobPropertiesSerDe.java:43-103 (VERSION_1..5 read, VERSION_5 written)
  Utils.java:233-283,860-892 (int-length strings)
Every record's CRC covers [record start, record end - 8) and is stored as a
big-endian long with the upper 32 bits zero. CRCs come from zlib.crc32, the
function java.util.zip.CRC32 computes.
"""
from __future__ import annotations

import struct
import zlib

CRC_SIZE = 8
INVALID = -1
HEADER_SIZE = {1: 34, 2: 38, 3: 40}

# status bits (mirrors include/ambrycrc.h AMBRYCRC_MSG_*)
HEADER_CRC = 1 << 0
ENCKEY_CRC = 1 << 1
PROPS_CRC = 1 << 2
UPDATE_CRC = 1 << 3
USERMETA_CRC = 1 << 4
BLOB_CRC = 1 << 5
BAD_VERSION = 1 << 8
BAD_LAYOUT = 1 << 9
NOT_PUT = 1 << 10      # transform only: an update record
BAD_RECORD = 1 << 11   # a record's size field disagrees with its span, bad blob type/size, record too short
NOT_ENCODABLE = 1 << 13  # transform only: the properties cannot be re-serialized (serialize_blob_properties_v5)

RECORD_BITS = (ENCKEY_CRC, PROPS_CRC, UPDATE_CRC, USERMETA_CRC, BLOB_CRC)  # slot order enc, bp, upd, um, blob


def _crc_long(b: bytes) -> bytes:
    return struct.pack(">q", zlib.crc32(b))


def header(version, total, enc, bp, upd, um, blob, life=0):
    if version == 1:
        body = struct.pack(">hqiiii", 1, total, bp, upd, um, blob)
    elif version == 2:
        body = struct.pack(">hqiiiii", 2, total, enc, bp, upd, um, blob)
    else:
        body = struct.pack(">hhqiiiii", 3, life, total, enc, bp, upd, um, blob)
    return body + _crc_long(body)


def store_key(blob_id: str) -> bytes:
    """MockId-style key bytes: short length + id (ambry-test-utils/.../store/MockId.java:47-77)."""
    raw = blob_id.encode()
    return struct.pack(">h", len(raw)) + raw


def _int_string(s):
    if s is None:
        return struct.pack(">i", 0)
    raw = s if isinstance(s, bytes) else s.encode()
    return struct.pack(">i", len(raw)) + raw


def blob_properties_bytes(blob_size, service_id="servid", owner_id="owner", content_type="application/octet",
                          ttl=-1, private=False, creation_ms=1_700_000_000_000, account=101, container=5,
                          encrypted=False, content_encoding=None, filename=None, reserved=None, serde_version=5):
    """BlobPropertiesSerDe bytes at `serde_version` 1..5: serializeBlobProperties writes VERSION_5
    (BlobPropertiesSerDe.java:83-103); versions 1..4 are the layouts getBlobPropertiesFromStream
    still reads (:56-77) -- older servers wrote them: V1 has no account/container, V1-V2 no
    `encrypted` byte, V1-V3 no contentEncoding/filename, V1-V4 no reservedMetadataBlobId.
    `private` / `encrypted` may be an int to store a non-canonical byte (the reader tests `== 1`)."""
    v = serde_version
    out = struct.pack(">hqbqq", v, ttl, int(private), creation_ms, blob_size)
    out += _int_string(content_type) + _int_string(owner_id) + _int_string(service_id)
    if v > 1:
        out += struct.pack(">hh", account, container)
    if v > 2:
        out += struct.pack(">b", int(encrypted))
    if v > 3:
        out += _int_string(content_encoding) + _int_string(filename)
    if v > 4:
        out += _int_string(reserved)
    return out


class PropsParseError(Exception):
    """getBlobPropertiesFromStream threw (IllegalArgumentException / EOFException): the record
    deserializer maps every such exception to DataCorrupt (MessageFormatRecord.java:1192-1195)."""


class NotEncodable(Exception):
    """serializeBlobProperties cannot re-write these properties: see serialize_blob_properties_v5."""


UNKNOWN_ACCOUNT_ID = -1    # Account.UNKNOWN_ACCOUNT_ID (ambry-api/.../account/Account.java:111)
UNKNOWN_CONTAINER_ID = -1  # Container.UNKNOWN_CONTAINER_ID (Container.java:97)


def parse_blob_properties(b: bytes, pos: int, end: int):
    """BlobPropertiesSerDe.getBlobPropertiesFromStream (BlobPropertiesSerDe.java:56-77) over
    b[pos:end): (fields dict, parsed end). Big-endian DataInputStream reads; a read past `end`
    is the EOFException; strings are Utils.readIntString (Utils.java:265-283: a negative size
    throws) and, from V4, readNullableIntString (:253-256: empty -> null). Strings are kept as
    their raw bytes (decoding is a separate question: serialize_blob_properties_v5)."""
    def take(n):
        nonlocal pos
        if n < 0 or pos + n > end:
            raise PropsParseError("EOF")
        s = b[pos:pos + n]
        pos += n
        return s

    def int_string(nullable=False):
        n = struct.unpack(">i", take(4))[0]
        if n < 0:
            raise PropsParseError("readIntString: the size cannot be negative")
        s = take(n)
        return None if (nullable and n == 0) else s

    v = struct.unpack(">h", take(2))[0]
    if v < 1 or v > 5:
        raise PropsParseError("stream has unknown blob property version %d" % v)
    ttl, priv, ctime, size = struct.unpack(">qbqq", take(25))
    f = {"version": v, "ttl": ttl, "private": priv == 1, "creation": ctime, "size": size}
    f["content_type"] = int_string()
    f["owner"] = int_string()
    f["service"] = int_string()
    f["account"], f["container"] = (struct.unpack(">hh", take(4)) if v > 1
                                    else (UNKNOWN_ACCOUNT_ID, UNKNOWN_CONTAINER_ID))
    f["encrypted"] = v > 2 and struct.unpack(">b", take(1))[0] == 1
    f["content_encoding"] = int_string(True) if v > 3 else None
    f["filename"] = int_string(True) if v > 3 else None
    f["reserved"] = int_string(True) if v > 4 else None
    return f, pos


_PROPS_STRINGS = ("content_type", "owner", "service", "content_encoding", "filename", "reserved")


def serialize_blob_properties_v5(f) -> bytes:
    """BlobPropertiesSerDe.serializeBlobProperties at CURRENT_VERSION = VERSION_5
    (BlobPropertiesSerDe.java:41,83-103), of properties parse_blob_properties read.

    Each string was decoded as UTF-8 (Utils.readIntString, Utils.java:265-283) and is re-encoded
    with Charset.defaultCharset() (Utils.serializeNullableString / serializeString, :860-866,
    888-892) -- UTF-8 assumed (the JDK 18+ default, JEP 400; a UTF-8 locale before). ASCII bytes
    round-trip unchanged. Any other byte makes the encoded string longer than String.length(),
    which is what getBlobPropertiesSerDeSize (:43-54, Utils.getIntStringLength :233-235) budgets:
    PutMessageFormatInputStream sizes its buffer from that budget (PutMessageFormatInputStream.java
    :83-90), so the extra bytes overrun it (BufferOverflowException) and the transform fails
    (ValidatingTransformer.java:100-102). NotEncodable models that."""
    for k in _PROPS_STRINGS:
        s = f[k]
        if s is not None and any(c >= 0x80 for c in s):
            raise NotEncodable(k)
    out = struct.pack(">hqbqq", 5, f["ttl"], 1 if f["private"] else 0, f["creation"], f["size"])
    for k in _PROPS_STRINGS[:3]:
        out += struct.pack(">i", len(f[k])) + f[k]
    out += struct.pack(">hhb", f["account"], f["container"], 1 if f["encrypted"] else 0)
    for k in _PROPS_STRINGS[3:]:
        s = f[k] or b""  # serializeNullableString: null -> int 0
        out += struct.pack(">i", len(s)) + s
    return out


UPDATE_TYPES = 3  # SubRecord.Type: DELETE, TTL_UPDATE, UNDELETE (SubRecord.java:26-28)


def _update_check(rec: bytes) -> int:
    """deserializeUpdateRecord (MessageFormatRecord.java:158-172) over a record span, stored CRC
    included: Update_Format_V1 (:1217-1228) reads a byte, V2 (:1253-1266) account, container and
    update time, V3 (:1388-1413) those, a short type indexing SubRecord.Type.values() (out of range
    throws), then the sub-record -- a short version that must be 1 (:1422-1464, UnknownFormatVersion
    otherwise) and, for TTL_UPDATE, a long expiry -- before the CRC. The parsed end must be the span's
    CRC position (else the reference reads its CRC elsewhere)."""
    v = _be16(rec, 0)
    body = len(rec) - CRC_SIZE
    if v == 1:
        return 0 if body == 3 else BAD_RECORD
    if v == 2:
        return 0 if body == 14 else BAD_RECORD
    if v != 3:
        return BAD_VERSION
    if body < 16:
        return BAD_RECORD
    t = _be16(rec, 14)
    if not 0 <= t < UPDATE_TYPES:
        return BAD_RECORD
    if body < 18:
        return BAD_RECORD
    if _be16(rec, 16) != 1:
        return BAD_VERSION
    return 0 if body == (26 if t == 1 else 18) else BAD_RECORD


def props_record(props: bytes) -> bytes:
    body = struct.pack(">h", 1) + props
    return body + _crc_long(body)


def enckey_record(key: bytes) -> bytes:
    body = struct.pack(">hi", 1, len(key)) + key
    return body + _crc_long(body)


def usermeta_record(um: bytes) -> bytes:
    body = struct.pack(">hi", 1, len(um)) + um
    return body + _crc_long(body)


def blob_record(content: bytes, version=3, blob_type=0, compressed=False) -> bytes:
    if version == 2:
        body = struct.pack(">hhq", 2, blob_type, len(content)) + content
    else:
        body = struct.pack(">hhbq", 3, blob_type, 1 if compressed else 0, len(content)) + content
    return body + _crc_long(body)


def update_record_v3(account=101, container=5, update_ms=1_700_000_000_123, kind="ttl", expiry=1_800_000_000_000):
    """Update_Format_V3 (MessageFormatRecord.java:1322-1379): TTL update / delete / undelete sub-records."""
    types = {"delete": 0, "ttl": 1, "undelete": 2}
    body = struct.pack(">hhhqh", 3, account, container, update_ms, types[kind])
    if kind == "ttl":
        body += struct.pack(">hq", 1, expiry)
    else:
        body += struct.pack(">h", 1)
    return body + _crc_long(body)


def put_message(key: bytes, props: bytes, usermeta: bytes, content: bytes, version=3, enc_key=None, life=0,
                blob_version=None, compressed=False, blob_type=0) -> bytes:
    """PutMessageFormatInputStream: header, key, [encryption key], properties, user metadata, blob."""
    h = HEADER_SIZE[version]
    enc = enckey_record(enc_key) if (enc_key is not None and version >= 2) else b""
    pr = props_record(props)
    um = usermeta_record(usermeta)
    bl = blob_record(content, version=blob_version or (3 if version != 1 else 3), blob_type=blob_type,
                     compressed=compressed)
    total = len(enc) + len(pr) + len(um) + len(bl)
    enc_off = h + len(key) if enc else INVALID
    bp_off = h + len(key) + len(enc)
    um_off = bp_off + len(pr)
    blob_off = um_off + len(um)
    return header(version, total, enc_off, bp_off, INVALID, um_off, blob_off, life) + key + enc + pr + um + bl


def update_message(key: bytes, version=3, life=1, **kw) -> bytes:
    h = HEADER_SIZE[version]
    rec = update_record_v3(**kw)
    return header(version, len(rec), INVALID, INVALID, h + len(key), INVALID, INVALID, life) + key + rec


def _be16(b, o):
    return struct.unpack_from(">h", b, o)[0]


def _be32(b, o):
    return struct.unpack_from(">i", b, o)[0]


def _be64(b, o):
    return struct.unpack_from(">q", b, o)[0]


def parse_header(region: bytes, off: int):
    """(version, total, [enc, bp, upd, um, blob]) or None when the version is unknown."""
    v = _be16(region, off)
    if v == 1:
        total = _be64(region, off + 2)
        rel = [INVALID] + [_be32(region, off + 10 + 4 * i) for i in range(4)]
    elif v == 2:
        total = _be64(region, off + 2)
        rel = [_be32(region, off + 10 + 4 * i) for i in range(5)]
    elif v == 3:
        total = _be64(region, off + 4)
        rel = [_be32(region, off + 12 + 4 * i) for i in range(5)]
    else:
        return None
    return v, total, rel


def _record_check(k: int, rec: bytes) -> int:
    """What record k's deserializer reads before its CRC (MessageFormatRecord.java): the version
    (deserializeAndGet*WithVersion :147-239 throw UnknownFormatVersion), then the size fields that
    decide where the stream reads the CRC -- BlobEncryptionKey_Format_V1 (:1588-1600) and
    UserMetadata_Format_V1 (:1637-1649): int size + bytes; Blob_Format_V1..V3 (:1681-1833): type
    ordinal < 2, long size <= Integer.MAX_VALUE. BlobProperties_Format_V1 (:1179-1195): the
    BlobPropertiesSerDe fields (parse_blob_properties), any exception -> DataCorrupt. Update
    records: _update_check. `rec` is the record's span from the header, stored CRC included; a
    parsed end other than the span's CRC position is BAD_RECORD (the reference would read its CRC
    from other bytes)."""
    if len(rec) < 10:
        return BAD_RECORD
    v = _be16(rec, 0)
    if k in (0, 3):
        if v != 1:
            return BAD_VERSION
        if len(rec) < 14:
            return BAD_RECORD
        n = _be32(rec, 2)
        return 0 if n >= 0 and n + 14 == len(rec) else BAD_RECORD
    if k == 1:
        if v != 1:
            return BAD_VERSION
        try:
            _, end = parse_blob_properties(rec, 2, len(rec) - CRC_SIZE)
        except PropsParseError:
            return BAD_RECORD
        return 0 if end == len(rec) - CRC_SIZE else BAD_RECORD
    if k == 2:
        return _update_check(rec)
    if not 1 <= v <= 3:
        return BAD_VERSION
    head = {1: 10, 2: 12, 3: 13}[v]
    if len(rec) < head + 8:
        return BAD_RECORD
    btype = 0 if v == 1 else struct.unpack_from(">H", rec, 2)[0]  # a negative ordinal fails too (index error)
    size = struct.unpack_from(">Q", rec, {1: 2, 2: 4, 3: 5}[v])[0]
    return 0 if btype < 2 and size <= 0x7FFFFFFF and size + head + 8 == len(rec) else BAD_RECORD


def verify_message(region: bytes, off: int):
    """(status bits, message end offset or 0) -- deserializeBlobAll / update-record semantics."""
    if off + 2 > len(region):
        return BAD_LAYOUT, 0
    v = _be16(region, off)
    if v not in HEADER_SIZE:
        return BAD_VERSION, 0
    h = HEADER_SIZE[v]
    if off + h > len(region):
        return BAD_LAYOUT, 0
    stored = _be64(region, off + h - CRC_SIZE)
    if zlib.crc32(region[off:off + h - CRC_SIZE]) != stored:
        return HEADER_CRC, 0  # verifyHeader throws before any record is read
    _, total, rel = parse_header(region, off)
    if v == 3 and _be16(region, off + 2) < 0:  # lifeVersion >= 0 (checkHeaderConstraints, :990-1003)
        return BAD_LAYOUT, 0
    enc, bp, upd, um, blob = rel
    is_put = bp != INVALID and upd == INVALID and um != INVALID and blob != INVALID
    is_upd = upd != INVALID and bp == INVALID and um == INVALID and blob == INVALID and enc == INVALID
    if total <= 0 or not (is_put or is_upd):
        return BAD_LAYOUT, 0
    present = [(k, r) for k, r in enumerate(rel) if r != INVALID]
    starts = [r for _, r in present]
    if starts[0] < h or any(b <= a for a, b in zip(starts, starts[1:])):
        return BAD_LAYOUT, 0
    end = starts[0] + total
    if off + end > len(region):
        return BAD_LAYOUT, 0
    status = 0
    for i, (k, s) in enumerate(present):
        e = starts[i + 1] if i + 1 < len(present) else end
        if e - s < CRC_SIZE:
            return BAD_LAYOUT, 0
        stored = _be64(region, off + e - CRC_SIZE)
        if zlib.crc32(region[off + s:off + e - CRC_SIZE]) != stored:
            status |= RECORD_BITS[k]
        status |= _record_check(k, region[off + s:off + e])
    return status, off + end


def blob_record_v1(content: bytes) -> bytes:
    """Blob_Format_V1 (MessageFormatRecord.java:1668-1716): short 1, long size, content, CRC."""
    body = struct.pack(">hq", 1, len(content)) + content
    return body + _crc_long(body)


def transform_message(region: bytes, off: int, life=None, version: int = 3):
    """ValidatingTransformer.transform (ValidatingTransformer.java:46-104): (status, bytes or None).

    Verify every CRC (verify_message); refuse update records ("Message cannot be anything rather
    than put record"); deserialize the encryption key, properties, user metadata and blob
    (deserializeBlob* :1568-1833: blob record V1/V2/V3, type ordinal < 2, size <= MAX_INT, the
    fields consistent with the record spans); re-serialize with PutMessageFormatInputStream at
    header `version` (V1 drops the encryption key) and lifeVersion `life` (msgInfo's; None: the
    stored header's, 0 for V1/V2)."""
    status, end = verify_message(region, off)
    if status:
        return status, None
    v, total, rel = parse_header(region, off)
    enc, bp, upd, um, blob = rel
    if upd != INVALID or bp == INVALID or um == INVALID or blob == INVALID:
        return NOT_PUT, None
    h = HEADER_SIZE[v]
    first = enc if enc != INVALID else bp
    key = region[off + h:off + first]
    enc_key = None
    if enc != INVALID:
        n = _be32(region, off + enc + 2)
        if n < 0 or enc + 6 + n + 8 != bp:
            return BAD_RECORD, None
        enc_key = region[off + enc + 6:off + enc + 6 + n]
    if um - 8 < bp + 2:
        return BAD_RECORD, None
    # deserializeBlobProperties, then serializeBlobProperties at VERSION_5 (ValidatingTransformer.java
    # :77,87-89 -> PutMessageFormatInputStream.java:114 -> BlobPropertiesSerDe.java:83-103)
    fields, _ = parse_blob_properties(region, off + bp + 2, off + um - 8)  # verify_message parsed it
    try:
        props = serialize_blob_properties_v5(fields)
    except NotEncodable:
        return NOT_ENCODABLE, None
    n = _be32(region, off + um + 2)
    if n < 0 or um + 6 + n + 8 != blob:
        return BAD_RECORD, None
    usermeta = region[off + um + 6:off + um + 6 + n]
    bv = _be16(region, off + blob)
    btype, comp = 0, False
    if bv == 1:
        size, head = _be64(region, off + blob + 2), 10
    elif bv == 2:
        btype, size, head = _be16(region, off + blob + 2), _be64(region, off + blob + 4), 12
    elif bv == 3:
        btype = _be16(region, off + blob + 2)
        comp = region[off + blob + 4] == 1
        size, head = _be64(region, off + blob + 5), 13
    else:
        return BAD_RECORD, None
    if not (0 <= btype < 2) or not (0 <= size <= 0x7FFFFFFF) or blob + head + size + 8 != first + total:
        return BAD_RECORD, None
    content = region[off + blob + head:off + blob + head + size]
    stored_life = _be16(region, off + 2) if v == 3 else 0
    out = put_message(key, props, usermeta, content, version=version,
                      enc_key=enc_key if version >= 2 else None, life=stored_life if life is None else life,
                      compressed=comp, blob_type=btype)
    return 0, out
