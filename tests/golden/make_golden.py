#!/usr/bin/env python3
"""Generates the golden fixtures in tests/golden/ (run in the build container).

The reference (Java) cannot run here (no JDK), so parity is
pinned by:
  1. crc32_table_fingerprint.json -- the 2048 table words of
     ambry-utils/src/main/java/com/github/ambry/utils/Crc32.java:154-179,
     parsed from the source *as text* (only read when /root/reference exists),
     reduced to a fingerprint + a few entries. No source text is stored.
  2. crc32_vectors.json -- known answers computed with Python's zlib.crc32,
     the same CRC-32 that java.util.zip.CRC32 (zlib-backed) computes and that
     Ambry's messageformat/protocol layers call: the standard check value,
     the reference tests' empty/zero-run cases, the deterministic message
     headers of MessageFormatRecordTest.java:70,92,115 and
     MessageFormatSendTest.java:621-630 serialized per MessageFormatRecord.java
     :467-486 (V1), :696-725 (V2), :951-981 (V3), and seeded random vectors
     over tests/datagen.py's splitmix stream (seed, offset, length, crc only).
  3. c1_message.bin + c1_message.json -- BASELINE.json configs[0] (C1): one PUT message with a
     V3 header (MessageFormatRecord.java:951-981), MockId("id1") key (MockId.java:47-77),
     BlobProperties VERSION_5 (BlobPropertiesSerDe.java:80-103), 1000 B user metadata and a
     64 KiB blob record (Blob_Format_V3, :1777-1833), laid out by PutMessageFormatInputStream
     (:76-124) through oracle/message_format.py; every record CRC from zlib.crc32 (the JDK
     CRC32's function), with the record byte ranges. Shape of MessageFormatInputStreamTest.java:70-243.
"""
from __future__ import annotations

import hashlib
import json
import os
import re
import struct
import sys
import zlib

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from datagen import stream_bytes  # noqa: E402

REF_CRC32_JAVA = "/root/reference/ambry-utils/src/main/java/com/github/ambry/utils/Crc32.java"


def table_fingerprint():
    if not os.path.exists(REF_CRC32_JAVA):
        return None
    text = open(REF_CRC32_JAVA).read()
    body = text[text.index("private static final int[] T = new int[]{"):]
    words = [int(h, 16) for h in re.findall(r"0x([0-9A-Fa-f]{8})", body)]
    assert len(words) == 2048, len(words)
    packed = struct.pack("<2048I", *words)
    return {
        "source": "ambry-utils/src/main/java/com/github/ambry/utils/Crc32.java:154-179",
        "words": 2048,
        "packing": "little-endian uint32, T8_0 first",
        "zlib_crc32": f"0x{zlib.crc32(packed):08x}",
        "sha256": hashlib.sha256(packed).hexdigest(),
        "T8_k_1": [f"0x{words[k * 256 + 1]:08x}" for k in range(8)],
        "T8_k_255": [f"0x{words[k * 256 + 255]:08x}" for k in range(8)],
    }


def header_v1(total, bp, upd, um, blob, version=1):
    return struct.pack(">hqiiii", version, total, bp, upd, um, blob)


def header_v2(total, enc, bp, upd, um, blob):
    return struct.pack(">hqiiiii", 2, total, enc, bp, upd, um, blob)


def header_v3(life, total, enc, bp, upd, um, blob):
    return struct.pack(">hhqiiiii", 3, life, total, enc, bp, upd, um, blob)


def vectors():
    kat = [
        {"name": "check_123456789", "hex": b"123456789".hex(), "crc": "0xcbf43926"},
        {"name": "empty (PutOperationTest.java:1106 empty content)", "hex": "", "crc": "0x00000000"},
        {"name": "a", "hex": b"a".hex(), "crc": f"0x{zlib.crc32(b'a'):08x}"},
        {"name": "bytes_0_255", "hex": bytes(range(256)).hex(), "crc": f"0x{zlib.crc32(bytes(range(256))):08x}"},
    ]
    zero_runs = [{"len": n, "crc": f"0x{zlib.crc32(bytes(n)):08x}"} for n in (1, 15, 16, 1000, 65536, 4 << 20)]
    headers = [
        {"name": "MessageHeader_Format_V1 (MessageFormatRecordTest.java:70)",
         "hex": header_v1(1000, 10, -1, 20, 30).hex()},
        {"name": "MessageHeader_Format_V2 (MessageFormatRecordTest.java:92)",
         "hex": header_v2(1000, 5, 10, -1, 20, 30).hex()},
        {"name": "MessageHeader_Format_V3 (MessageFormatRecordTest.java:115)",
         "hex": header_v3(2, 1000, 5, 10, -1, 20, 30).hex()},
        {"name": "V1 header (MessageFormatSendTest.java:621-630)",
         "hex": header_v1(950, 60, -1, 81, 191).hex()},
    ]
    for h in headers:
        h["crc"] = f"0x{zlib.crc32(bytes.fromhex(h['hex'])):08x}"
    lengths = list(range(0, 18)) + [31, 32, 33, 63, 64, 65, 127, 1000, 1023, 1024, 1025, 4000, 4096, 16383,
                                     65536, 65539, 262143, 262144, 262161, 1 << 20, (4 << 20) - 3, 4 << 20]
    rnd = []
    seed = 0xA3B1C2D3
    for i, n in enumerate(lengths):
        off = (i * 7919) % 61  # odd / unaligned starts
        data = stream_bytes(seed, off, n).tobytes()
        cin = (i * 0x9E3779B9) & 0xFFFFFFFF if i % 3 == 2 else 0
        rnd.append({"seed": f"0x{seed:x}", "offset": off, "len": n, "crc_in": f"0x{cin:08x}",
                    "crc": f"0x{zlib.crc32(data, cin):08x}"})
    return {"generator": "tests/golden/make_golden.py (zlib %s)" % zlib.ZLIB_RUNTIME_VERSION,
            "known_answers": kat, "zero_runs": zero_runs, "message_headers": headers, "random": rnd}


C1_SEED = 0xA3B1C2D3


def c1_message():
    """(message bytes, fixture dict) for config C1."""
    import importlib.util

    spec = importlib.util.spec_from_file_location(
        "message_format", os.path.join(os.path.dirname(os.path.dirname(HERE)), "oracle", "message_format.py"))
    mf = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mf)
    content = stream_bytes(C1_SEED, 0, 64 << 10).tobytes()
    usermeta = stream_bytes(C1_SEED, 1 << 20, 1000).tobytes()
    key = mf.store_key("id1")
    msg = mf.put_message(key, mf.blob_properties_bytes(len(content)), usermeta, content, version=3)
    version, total, rel = mf.parse_header(msg, 0)
    starts = [r for r in rel if r != -1]
    ends = starts[1:] + [starts[0] + total]
    ranges = [(0, mf.HEADER_SIZE[version] - 8)] + [(a, e - 8) for a, e in zip(starts, ends)]
    crcs = [zlib.crc32(msg[a:b]) for a, b in ranges]
    for (a, b), c in zip(ranges, crcs):  # the stored trailer of every record is that CRC
        assert struct.unpack(">q", msg[b:b + 8])[0] == c
    fx = {"generator": "tests/golden/make_golden.py (zlib %s)" % zlib.ZLIB_RUNTIME_VERSION,
          "what": "C1: one 64 KiB-blob PUT message, V3 header, MockId(\"id1\") key, BlobProperties V5, "
                  "1000 B user metadata, Blob_Format_V3 record",
          "seed": f"0x{C1_SEED:x}", "content": "datagen.stream_bytes(seed, 0, 65536)",
          "user_metadata": "datagen.stream_bytes(seed, 1 << 20, 1000)",
          "message_bytes": len(msg), "sha256": hashlib.sha256(msg).hexdigest(),
          "records": ["header", "blob_properties", "user_metadata", "blob"],
          "record_ranges": [[a, b] for a, b in ranges],
          "record_crcs": [f"0x{c:08x}" for c in crcs],
          "blob_prefix_bytes": 13, "key_offset": mf.HEADER_SIZE[version], "key_bytes": len(key)}
    return msg, fx


def main():
    msg, fx = c1_message()
    with open(os.path.join(HERE, "c1_message.bin"), "wb") as f:
        f.write(msg)
    with open(os.path.join(HERE, "c1_message.json"), "w") as f:
        json.dump(fx, f, indent=1)
    fp = table_fingerprint()
    if fp is not None:
        with open(os.path.join(HERE, "crc32_table_fingerprint.json"), "w") as f:
            json.dump(fp, f, indent=1)
    with open(os.path.join(HERE, "crc32_vectors.json"), "w") as f:
        json.dump(vectors(), f, indent=1)


if __name__ == "__main__":
    main()
