"""Write side of the message path: PUT messages laid out and every CRC
trailer filled by libambrycrc, byte-exact against oracle/message_format.py's restatement of
PutMessageFormatInputStream (PutMessageFormatInputStream.java:76-124, header V1 :133-162) and
the record formats of MessageFormatRecord.java, with zlib CRCs. Shape of
MessageFormatInputStreamTest.java:70-243: serialize, then every record must verify."""
import importlib.util
import itertools
import os
import zlib

import numpy as np
import pytest

from c1_message import c1_fixture, c1_message_bytes
from datagen import stream_bytes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def mf():
    spec = importlib.util.spec_from_file_location("message_format", os.path.join(ROOT, "oracle", "message_format.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def random_messages(mf, n, seed, max_blob=70000):
    from ambry_amd.messages import PutMessage

    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        v = int(rng.choice([1, 2, 3], p=[0.15, 0.15, 0.7]))
        enc = None
        if v >= 2 and rng.random() < 0.4:
            enc = stream_bytes(seed + i, 5, int(rng.choice([0, 1, 16, 32, 300]))).tobytes()
        blen = int(rng.choice([0, 1, 3, 13, 100, 1000, 4096, 4109, int(rng.integers(0, max_blob))]))
        um = stream_bytes(seed + i, 7 << 20, int(rng.choice([0, 1, 5, 1000, int(rng.integers(0, 3000))]))).tobytes()
        key = mf.store_key("blob-%d-%s" % (i, "x" * int(rng.integers(0, 40))))
        props = mf.blob_properties_bytes(blen, service_id="svc%d" % i, ttl=int(rng.integers(-1, 10**6)))
        out.append(PutMessage(key=key, props=props, usermeta=um, blob=stream_bytes(seed ^ i, 0, blen).tobytes(),
                              enckey=enc, header_version=v, life_version=int(rng.integers(0, 5)) if v == 3 else 0,
                              blob_type=int(rng.integers(0, 3)), compressed=bool(rng.random() < 0.3)))
    return out


def expected(mf, m):
    """oracle/message_format.py lays out blob type 0; other types differ only in the blob record's
    type field (and so in its CRC): patch and re-CRC that record."""
    import struct

    b = bytearray(mf.put_message(m.key, m.props, m.usermeta, m.blob, version=m.header_version, enc_key=m.enckey,
                                 life=m.life_version, compressed=m.compressed))
    v, total, rel = mf.parse_header(bytes(b), 0)
    blob_rel = rel[4]
    struct.pack_into(">h", b, blob_rel + 2, m.blob_type)
    end = len(b) - 8
    struct.pack_into(">q", b, end, zlib.crc32(bytes(b[blob_rel:end])))
    return bytes(b)


def test_host_serializer_matches_layout_oracle(ambry, mf):
    from ambry_amd.messages import layout, serialize_host

    for m in random_messages(mf, 300, seed=11):
        got, crcs = serialize_host(m)
        exp = expected(mf, m)
        assert got == exp
        # BlobType has two values (DataBlob, MetadataBlob): a type-2 record fails the reader's check
        assert mf.verify_message(got, 0) == (mf.BAD_RECORD if m.blob_type >= 2 else 0, len(got))
        n, offs = layout(m)
        assert n == len(got)
        assert got[offs["key"]:offs["key"] + len(m.key)] == m.key
        assert got[offs["blob"]:offs["blob"] + len(m.blob)] == m.blob
        assert got[offs["usermeta"]:offs["usermeta"] + len(m.usermeta)] == m.usermeta
        assert got[offs["props"]:offs["props"] + len(m.props)] == m.props
        if m.enckey is not None:
            assert got[offs["enckey"]:offs["enckey"] + len(m.enckey)] == m.enckey
        assert crcs[0] == zlib.crc32(got[:{1: 26, 2: 30, 3: 32}[m.header_version]])


def test_every_version_and_option(ambry, mf):
    from ambry_amd.messages import PutMessage, serialize_host

    blob = stream_bytes(3, 0, 777).tobytes()
    for v, enc, comp, life in itertools.product((1, 2, 3), (None, b"", b"k" * 32), (False, True), (0, 7)):
        if v == 1 and enc is not None:
            continue
        m = PutMessage(key=mf.store_key("id1"), props=mf.blob_properties_bytes(777), usermeta=b"meta" * 9, blob=blob,
                       enckey=enc, header_version=v, life_version=life if v == 3 else 0, compressed=comp)
        assert serialize_host(m)[0] == expected(mf, m)


def test_c1_message_serialized_by_the_product(ambry):
    """The C1 fixture's exact bytes come out of ambrycrc_serialize_put_host."""
    from ambry_amd.messages import PutMessage, serialize_host

    fx = c1_fixture()
    msg = c1_message_bytes()
    ko, kl = fx["key_offset"], fx["key_bytes"]
    (_, _), (p0, p1), (u0, u1), (b0, b1) = [tuple(r) for r in fx["record_ranges"]]
    m = PutMessage(key=msg[ko:ko + kl], props=msg[p0 + 2:p1], usermeta=msg[u0 + 6:u1], blob=msg[b0 + 13:b1])
    got, crcs = serialize_host(m)
    assert got == msg
    assert [f"0x{c:08x}" for c in (crcs[0], crcs[2], crcs[3], crcs[4])] == fx["record_crcs"]


def test_invalid_descriptors_rejected(ambry, mf):
    import ctypes

    from ambry_amd.messages import PutMessage

    L = ambry.lib()
    for v, enc in ((0, None), (4, None), (1, b"k")):
        m = PutMessage(key=b"\x00\x01a", props=b"", usermeta=b"", blob=b"", enckey=enc, header_version=v)
        assert L.ambrycrc_put_layout(ctypes.byref(m.desc()), None) == 0
        out = ctypes.create_string_buffer(4096)
        assert L.ambrycrc_serialize_put_host(ctypes.byref(m.desc()), None, None, out, 4096, None) == -1
    m = PutMessage(key=b"\x00\x01a", props=b"", usermeta=b"", blob=b"x" * 100)
    out = ctypes.create_string_buffer(64)
    assert L.ambrycrc_serialize_put_host(ctypes.byref(m.desc()), None, None, out, 64, None) == -1  # too small
    big = PutMessage(key=b"", props=b"", usermeta=b"", blob=b"")
    d = big.desc()
    d.usermeta_len = 0x7FFFFFF0  # relative offsets past a Java int
    assert L.ambrycrc_put_layout(ctypes.byref(d), None) == 0
