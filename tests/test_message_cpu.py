"""One message on the CPU (ambrycrc_verify_message_cpu / ambrycrc_transform_message_cpu): the
per-message form of the device verify and ValidatingTransformer paths, byte- and bit-exact
against oracle/message_format.py (verify_message restating deserializeBlobAll,
MessageFormatRecord.java:257-303; transform_message restating ValidatingTransformer.java:46-104)
on corrupted regions, the record-level cases, every header version and life version."""
import numpy as np
import pytest

from test_message_format import MF, build_region, record_level_cases


def test_verify_matches_oracle(ambry):
    from ambry_amd.messages import verify_message_cpu

    for seed in (1, 2, 3):
        region, offs, expect = build_region(n=300, seed=seed, corrupt_frac=0.15)
        for o, e in zip(offs, expect):
            assert verify_message_cpu(region, o) == e, (seed, o)
    for msg, want in record_level_cases():
        region = bytes(5) + msg
        assert verify_message_cpu(region, 5) == (want, len(region))


def test_verify_truncated_and_out_of_range(ambry):
    from ambry_amd.messages import verify_message_cpu

    region, offs, _ = build_region(n=40, seed=9, corrupt_frac=0.0)
    cut = region[:offs[-1] + 57]  # the last message cut inside its records
    for o in offs:
        assert verify_message_cpu(cut, o) == MF.verify_message(cut, o), o
    assert verify_message_cpu(region, len(region)) == (MF.BAD_LAYOUT, 0)
    assert verify_message_cpu(region, len(region) + 10) == (MF.BAD_LAYOUT, 0)
    assert verify_message_cpu(region, len(region) - 1) == (MF.BAD_LAYOUT, 0)


@pytest.mark.parametrize("version", [3, 2, 1])
@pytest.mark.parametrize("life", [None, 5])
def test_transform_matches_oracle(ambry, version, life):
    from test_gpu_transform import build_region as transform_region

    from ambry_amd.messages import transform_message_cpu

    region, offs = transform_region(MF, 300, seed=50 + version)
    kinds = set()
    for o in offs:
        exp_st, exp = MF.transform_message(region, o, life=life, version=version)
        st, got = transform_message_cpu(region, o, header_version=version, life=life)
        assert st == exp_st, o
        assert got == exp, o
        kinds.add(st)
    assert 0 in kinds and MF.NOT_PUT in kinds and MF.BAD_RECORD in kinds and MF.NOT_ENCODABLE in kinds


@pytest.mark.parametrize("life", [None, 0, 7])
def test_transform_fast_form_matches_oracle(ambry, life):
    """The CPU transform's fast form (V3 header, V3 blob record, properties already canonical
    VERSION_5 bytes: the message's own bytes with the life version and header CRC rewritten, as the
    GPU fast path does) against the oracle's full re-serialization, message by message."""
    from test_gpu_transform import dense_v3_region

    from ambry_amd.messages import transform_message_cpu

    region, offs = dense_v3_region(MF, 200, seed=61)
    for o in offs:
        exp_st, exp = MF.transform_message(region, o, life=life, version=3)
        st, got = transform_message_cpu(region, o, header_version=3, life=life)
        assert exp_st == 0 and st == 0 and got == exp, o


def test_transform_no_room_and_args(ambry):
    from ambry_amd._lib import AmbryCrcError
    from ambry_amd.messages import MSG_NO_ROOM, transform_message_cpu

    msg = MF.put_message(MF.store_key("k"), MF.blob_properties_bytes(100), b"um", bytes(100))
    st, out = transform_message_cpu(msg, 0, out_cap=len(msg) - 1)
    assert st == MSG_NO_ROOM and out is None
    assert transform_message_cpu(msg, 0, out_cap=len(msg)) == (0, msg)
    with pytest.raises(AmbryCrcError):
        transform_message_cpu(msg, 0, header_version=4)


def test_verdict_probes_props(ambry):
    """Round-2 review probes: a CRC-valid properties record at SerDe version 9 is DataCorrupt
    (BlobPropertiesSerDe.java:58-60 under MessageFormatRecord.java:1192-1195), and a message whose
    properties are stored at SerDe V1 comes out of the transform re-encoded at V5
    (ValidatingTransformer.java:77,87-89 -> BlobPropertiesSerDe.java:83-103): new bytes, new CRC."""
    import struct

    from ambry_amd.messages import transform_message_cpu, verify_message_cpu

    key, um, content = MF.store_key("probe"), b"meta", bytes(range(50))
    v5 = MF.blob_properties_bytes(50, content_encoding="gzip")
    bad = MF.put_message(key, struct.pack(">h", 9) + v5[2:], um, content)
    assert verify_message_cpu(bad, 0) == (MF.BAD_RECORD, len(bad))
    v1 = MF.blob_properties_bytes(50, serde_version=1, private=True)
    msg = MF.put_message(key, v1, um, content)
    st, out = transform_message_cpu(msg, 0)
    assert st == 0 and out != msg
    want = MF.put_message(key, MF.blob_properties_bytes(50, serde_version=5, private=True, account=-1, container=-1),
                          um, content)
    assert out == want and MF.transform_message(msg, 0) == (0, want)
    assert verify_message_cpu(out, 0) == (0, len(out))


def test_transform_dense_old_region_bound(ambry):
    """Each old message (header V1/V2, SerDe V1-V3 properties, Blob_Format_V1) fits the ABI's
    bound for its own length (ambrycrc_transform_out_bound(len, 1)); the bound is tight for the
    worst case (V1 header + V1 props + blob V1 -> V3: exactly +26 B)."""
    from test_gpu_transform import dense_old_region

    from ambry_amd.messages import TRANSFORM_GROWTH_MAX, out_bound, transform_message_cpu

    region, offs = dense_old_region(MF, 200, seed=5)
    ends = offs[1:] + [len(region)]
    worst = 0
    for o, e in zip(offs, ends):
        exp_st, exp = MF.transform_message(region, o, version=3)
        assert exp_st == 0
        msg = region[o:e]
        assert transform_message_cpu(msg, 0, out_cap=out_bound(len(msg), 1)) == (0, exp)
        assert transform_message_cpu(region, o) == (0, exp)  # the default cap
        worst = max(worst, len(exp) - len(msg))
    assert worst == TRANSFORM_GROWTH_MAX
    assert out_bound(2**64 - 10, 1) == 2**64 - 1  # saturates


def test_transform_host_argument_errors(ambry):
    """ambrycrc_transform_messages_host rejects bad arguments before touching a device, and reports
    ENOINIT for a device with no context (no GPU in the build container)."""
    import ctypes

    from ambry_amd._lib import lib

    region = (ctypes.c_uint8 * 64)()
    offs = (ctypes.c_uint64 * 1)(0)
    st = (ctypes.c_uint32 * 1)()
    ol = (ctypes.c_uint64 * 1)()
    out = (ctypes.c_uint8 * 128)()
    f = lib().ambrycrc_transform_messages_host
    assert f(region, 64, offs, 0, None, 3, out, 128, None, ol, st, 0, 0) == 0  # m == 0: nothing to do
    assert f(region, 64, offs, 1, None, 4, out, 128, None, ol, st, 0, 0) == -1  # header version
    assert f(region, 64, None, 1, None, 3, out, 128, None, ol, st, 0, 0) == -1
    assert f(region, 64, offs, 1, None, 3, out, 128, None, None, st, 0, 0) == -1
    assert f(region, 64, offs, 1, None, 3, None, 128, None, ol, st, 0, 0) == -1  # out NULL with a capacity
    assert f(region, 64, offs, 1, None, 3, out, 128, None, ol, st, 63, 0) == -4  # no context


def test_transform_host_cpu_leg_writes_negative_life_versions(ambry):
    """The CPU leg of ambrycrc_transform_messages_host (device -1) writes each index life version as given,
    -1 (MessageInfo.LIFE_VERSION_FROM_FRONTEND) included, as ValidatingTransformer.java:90 writes
    msgInfo.getLifeVersion() and the device batch does: dense clean V3 messages (the CPU fast form) and
    the mixed region (the general form), against the oracle."""
    from test_gpu_transform import build_region, dense_v3_region

    from ambry_amd.messages import transform_host

    for region, offs in (dense_v3_region(MF, 60, seed=21), build_region(MF, 120, seed=22)):
        life = np.random.default_rng(8).integers(-2, 4, size=len(offs)).astype(np.int16)
        life[::5] = -1
        out, oo, ol, st = transform_host(region, offs, header_version=3, life_version=life, device=-1)
        pos = 0
        for i, o in enumerate(offs):
            exp_st, exp = MF.transform_message(region, o, life=int(life[i]), version=3)
            assert int(st[i]) == exp_st, i
            if exp is not None:
                assert oo[i] == pos and out[pos:pos + len(exp)] == exp, i
                pos += len(exp)
