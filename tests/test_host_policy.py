"""Host-resident dispatch (include/ambrycrc.h ambrycrc_set_host_policy): the
*_host entries' CPU leg. device = -1 runs it without any GPU context, so this file runs on the CPU:
ambrycrc_batch_host, _verify_messages_host and _transform_messages_host on the CPU leg against
zlib and oracle/message_format.py (the same outputs the GPU leg's tests check), and the argument
rules of the policy calls."""
import zlib

import numpy as np
import pytest

from datagen import stream_bytes
from test_message_format import MF, build_region


@pytest.fixture(scope="module")
def ambry():
    from conftest import _build_if_missing

    _build_if_missing()
    import ambry_amd

    return ambry_amd


def test_batch_host_cpu_leg(ambry):
    """ambrycrc_batch_host(device = -1): every chunk's CRC (with and without crc_in) equals zlib's,
    empty chunks included -- Crc32.update over each buffer (Crc32.java:55-98)."""
    from ambry_amd import device as D

    mem = stream_bytes(3, 0, 6 << 20)
    rng = np.random.default_rng(4)
    offs = rng.integers(0, (6 << 20) - (1 << 20), size=300)
    lens = rng.integers(0, 1 << 20, size=300)
    lens[:3] = [0, 1, 4095]
    chunks = [(mem.ctypes.data + int(o), int(n)) for o, n in zip(offs, lens)]
    got = D.crc32_batch_host(chunks, device=-1)
    assert got == [zlib.crc32(mem[o:o + n].tobytes()) for o, n in zip(offs, lens)]
    cin = rng.integers(0, 1 << 32, size=300, dtype=np.uint64).astype(np.uint32)
    got = D.crc32_batch_host(chunks, device=-1, crc_in=cin)
    assert got == [zlib.crc32(mem[o:o + n].tobytes(), int(c)) for o, n, c in zip(offs, lens, cin)]


@pytest.mark.parametrize("seed", [1, 2])
def test_verify_messages_host_cpu_leg(ambry, seed):
    """ambrycrc_verify_messages_host(device = -1) over a region of PUT / update messages (headers
    V1-V3, corrupt bytes, a bad version, a truncated tail): every status and message end equals the
    oracle's deserializeBlobAll reading, as the GPU leg's test_verify_messages_host_matches_oracle."""
    from ambry_amd import device as D

    region, offs, expect = build_region(n=400, seed=seed, corrupt_frac=0.1)
    st, end = D.verify_messages_host(region, offs, device=-1)
    assert list(st) == [s for s, _ in expect]
    assert list(end) == [e for _, e in expect]


def test_transform_messages_host_cpu_leg(ambry):
    """ambrycrc_transform_messages_host(device = -1): ValidatingTransformer.transform over a batch
    (ValidatingTransformer.java:46-104) -- clean PUTs of every header version re-serialized at V3
    with index life versions, corrupt ones and update records refused -- packed in message order;
    then a cap that holds only the first 20 outputs gives NO_ROOM after them, as the device batch."""
    from ambry_amd.messages import transform_host

    region, offs, _ = build_region(n=300, seed=9, corrupt_frac=0.1)
    life = np.random.default_rng(2).integers(0, 7, size=len(offs)).astype(np.int16)
    out, oo, ol, st = transform_host(region, offs, life_version=life, device=-1)
    pos = 0
    for i, o in enumerate(offs):
        exp_st, exp = MF.transform_message(region, o, life=int(life[i]), version=3)
        assert int(st[i]) == exp_st, i
        if exp is None:
            assert ol[i] == 0 and oo[i] == -1
            continue
        assert oo[i] == pos and ol[i] == len(exp) and out[pos:pos + len(exp)] == exp, i
        pos += len(exp)
    ok = [i for i in range(len(offs)) if st[i] == 0]
    cap = int(oo[ok[20]])
    _, oo2, ol2, st2 = transform_host(region, offs, life_version=life, device=-1, out_cap=cap)
    assert all(st2[i] == 0 for i in ok[:20]) and all(st2[i] == (1 << 12) for i in ok[20:])  # AMBRYCRC_MSG_NO_ROOM
    assert all(oo2[i] == -1 and ol2[i] == 0 for i in ok[20:])


def test_policy_calls_without_context(ambry):
    """Policy calls need a context (ENOINIT without one); the CPU leg does not."""
    from ambry_amd._lib import lib

    L = lib()
    dev = 63  # never initialised here
    assert L.ambrycrc_set_host_policy(dev, 1) == -4
    assert L.ambrycrc_last_host_path(dev) == -4
    assert L.ambrycrc_host_rates(dev, None, None, None) == -4
    assert L.ambrycrc_host_msg_rates(dev, 0, None, None) == -4


def test_transform_messages_host_cpu_leg_fast_form(ambry):
    """The CPU leg over a dense region of canonical V3 PUTs (every message takes the fast form: its own
    bytes, life version and header CRC rewritten), with index life versions, against the oracle;
    then with no life versions, where the output is the region itself."""
    from test_gpu_transform import dense_v3_region

    from ambry_amd.messages import transform_host

    region, offs = dense_v3_region(MF, 300, seed=19)
    life = np.random.default_rng(4).integers(0, 9, size=len(offs)).astype(np.int16)
    out, oo, ol, st = transform_host(region, offs, life_version=life, device=-1)
    assert list(st) == [0] * len(offs)
    for i, o in enumerate(offs):
        exp_st, exp = MF.transform_message(region, o, life=int(life[i]), version=3)
        assert exp_st == 0 and oo[i] == o - offs[0] and out[oo[i]:oo[i] + ol[i]] == exp, i
    out2, _, _, st2 = transform_host(region, offs, device=-1)
    assert list(st2) == [0] * len(offs) and out2 == region[offs[0]:]


def test_cpu_budget_process_default_and_calibration(ambry):
    """The CPU leg's budget (ambrycrc_set_host_cpu_threads): the default is half this process's CPU share
    (the rest stays with the server's own threads), a process budget set with device -1 is what device -1
    calls and ambrycrc_host_rates report, the calibration is per budget (run once per thread count, then cached),
    and the CPU leg's results do not depend on it."""
    import os

    from ambry_amd import device as D

    share = len(os.sched_getaffinity(0))
    if os.environ.get("OMP_NUM_THREADS", "").isdigit() and int(os.environ["OMP_NUM_THREADS"]) > 0:
        share = min(share, int(os.environ["OMP_NUM_THREADS"]))
    prev = D.set_host_cpu_threads(-1, 0)
    try:
        default = D.host_rates(-1)["cpu_threads"]
        if "AMBRYCRC_CPU_THREADS" not in os.environ:
            assert 1 <= default <= max(1, share // 2)
        assert D.set_host_cpu_threads(-1, 1) == 0
        one = D.host_calibrate(-1)
        r1 = D.host_rates(-1)
        assert r1["cpu_threads"] == 1 and r1["gpu_gibps"] == 0 and r1["auto_leg"] == "cpu" and one > 0
        assert r1["cpu_gibps"] == one  # the calibration at this budget is what auto compares
        mem = stream_bytes(5, 0, 4 << 20)
        chunks = [(mem.ctypes.data + 997 * i, 30000 + i) for i in range(64)]
        want = [zlib.crc32(mem[997 * i:997 * i + 30000 + i].tobytes()) for i in range(64)]
        assert D.crc32_batch_host(chunks, device=-1) == want
        if share >= 4:
            assert D.set_host_cpu_threads(-1, 4) == 1
            four = D.host_calibrate(-1)
            assert four > 0 and D.host_calibrate(-1) == four  # one calibration per budget, then cached
            assert D.host_rates(-1)["cpu_gibps"] == four
            assert D.crc32_batch_host(chunks, device=-1) == want
        with pytest.raises(Exception):
            D.set_host_cpu_threads(-1, -2)
        with pytest.raises(Exception):
            D.set_host_cpu_threads(-1, 257)
        with pytest.raises(Exception):
            D.set_host_cpu_threads(63, 2)  # no context for device 63
    finally:
        D.set_host_cpu_threads(-1, prev)
