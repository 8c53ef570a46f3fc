"""Host-resident dispatch on a GPU box (include/ambrycrc.h ambrycrc_set_host_policy): auto takes the
leg ambrycrc_host_rates names for pageable bytes and the GPU for pinned ones; the forced policies
take theirs; every leg gives zlib's CRCs and the oracle's message statuses."""
import zlib

import numpy as np
import pytest

from datagen import stream_bytes
from test_message_format import build_region

pytestmark = pytest.mark.gpu


def test_auto_policy_legs(gpu):
    import torch

    mem = stream_bytes(11, 0, 8 << 20)
    chunks = [(mem.ctypes.data + 4096 * i, 65536 + i) for i in range(100)]
    want = [zlib.crc32(mem[4096 * i:4096 * i + 65536 + i].tobytes()) for i in range(100)]
    rates = gpu.host_rates(0)
    assert rates["cpu_threads"] >= 1 and rates["cpu_gibps"] > 0 and rates["gpu_gibps"] > 0
    prev = gpu.set_host_policy(0, gpu.HOST_AUTO)
    try:
        assert gpu.crc32_batch_host(chunks) == want
        assert gpu.last_host_path(0) == (1 if rates["auto_leg"] == "gpu" else 0)
        pinned = torch.from_numpy(mem).pin_memory()
        pc = [(pinned.data_ptr() + 4096 * i, 65536 + i) for i in range(100)]
        assert gpu.crc32_batch_host(pc, pinned=True) == want
        assert gpu.last_host_path(0) == 1  # pinned bytes: the GPU's DMA
        gpu.set_host_policy(0, gpu.HOST_CPU)
        assert gpu.crc32_batch_host(pc, pinned=True) == want and gpu.last_host_path(0) == 0
        gpu.set_host_policy(0, gpu.HOST_GPU)
        assert gpu.crc32_batch_host(chunks) == want and gpu.last_host_path(0) == 1
    finally:
        gpu.set_host_policy(0, prev)


@pytest.mark.parametrize("policy", ["cpu", "gpu"])
def test_verify_messages_host_both_legs(gpu, policy):
    region, offs, expect = build_region(n=500, seed=31, corrupt_frac=0.1)
    prev = gpu.set_host_policy(0, gpu.HOST_CPU if policy == "cpu" else gpu.HOST_GPU)
    try:
        st, end = gpu.verify_messages_host(region, offs)
        assert gpu.last_host_path(0) == (0 if policy == "cpu" else 1)
    finally:
        gpu.set_host_policy(0, prev)
    assert list(st) == [s for s, _ in expect] and list(end) == [e for _, e in expect]


@pytest.mark.parametrize("op", ["verify", "transform"])
def test_auto_policy_message_legs(gpu, op):
    """The message entries under auto take the leg ambrycrc_host_msg_rates names for their own op
    (not the CRC batch's rates: a CPU leg parses, and for the transform copies, each message);
    results equal the oracle's either way."""
    from test_gpu_transform import dense_v3_region
    from test_message_format import MF

    from ambry_amd.messages import transform_host

    region, offs = dense_v3_region(MF, 400, seed=71)
    rates = gpu.host_msg_rates(0, op)
    assert rates["cpu_gibps"] > 0 and rates["gpu_gibps"] > 0
    prev = gpu.set_host_policy(0, gpu.HOST_AUTO)
    try:
        if op == "verify":
            st, end = gpu.verify_messages_host(region, offs)
            assert list(st) == [0] * len(offs)
        else:
            out, oo, ol, st = transform_host(region, offs)
            assert list(st) == [0] * len(offs) and out == region  # V3 -> V3, no life versions: the same bytes
        assert gpu.last_host_path(0) == (1 if rates["auto_leg"] == "gpu" else 0)
    finally:
        gpu.set_host_policy(0, prev)
