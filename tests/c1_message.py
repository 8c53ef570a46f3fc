"""Config C1 (BASELINE.json configs[0]): the committed 64 KiB-blob PUT message fixture
(tests/golden/c1_message.bin / .json, made by tests/golden/make_golden.py) and its record ranges.
Data only: nothing here computes a CRC."""
from __future__ import annotations

import hashlib
import json
import os

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def c1_fixture() -> dict:
    with open(os.path.join(GOLDEN, "c1_message.json")) as f:
        return json.load(f)


def c1_message_bytes() -> bytes:
    with open(os.path.join(GOLDEN, "c1_message.bin"), "rb") as f:
        msg = f.read()
    fx = c1_fixture()
    if len(msg) != fx["message_bytes"] or hashlib.sha256(msg).hexdigest() != fx["sha256"]:
        raise ValueError("tests/golden/c1_message.bin does not match c1_message.json")
    return msg


def c1_record_ranges(msg: bytes | None = None):
    """[start, end) of the bytes each record CRC covers: header, properties, user metadata, blob."""
    return [tuple(r) for r in c1_fixture()["record_ranges"]]
