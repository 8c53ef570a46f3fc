#!/usr/bin/env python3
"""Measure §8f next #1: GPU verify of a log region of PUT messages (ambrycrc_verify_messages_dev),
plus config C1 (one 64 KiB PUT message, per-record CRCs on the CPU oracle).

The region is built on the device: every message shares the template header / key /
properties / user-metadata records (V3 header, 1000 B user metadata, as C1), blob
contents are random device bytes, and each blob record's CRC is computed by the engine
and stored big-endian, exactly as PutMessageFormatInputStream would have written it.
Prints one JSON line per measurement.

The oracle (oracle/message_format.py, oracle/crc32_ref.c) appears here only as the fixture
builder, the checker and the C1 CPU baseline being timed -- the roles tests/ and bench.py's
cpu_baseline leg give it; the GPU verify it measures is libambrycrc alone.
"""
from __future__ import annotations

import argparse
import importlib.util
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def load_mf():
    spec = importlib.util.spec_from_file_location("message_format", os.path.join(ROOT, "oracle", "message_format.py"))
    mf = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mf)
    return mf


def c1_cpu(mf, reps=2000):
    """C1: one 64 KiB-blob PUT message (V3 header, MockId key, BlobProperties, 1000 B user metadata);
    per-record CRCs with the oracle (C restatement of Crc32.java), µs per message, one core."""
    import numpy as np

    from conftest import Oracle
    from datagen import stream_bytes

    orc = Oracle()
    content = stream_bytes(0xA3B1C2D3, 0, 64 << 10).tobytes()
    msg = mf.put_message(mf.store_key("id1"), mf.blob_properties_bytes(len(content)),
                         stream_bytes(0xA3B1C2D3, 1 << 20, 1000).tobytes(), content, version=3)
    v, total, rel = mf.parse_header(msg, 0)
    starts = [r for r in rel if r != -1]
    ranges = [(0, 32)] + [(s, (starts[i + 1] if i + 1 < len(starts) else starts[0] + total) - 8)
                          for i, s in enumerate(starts)]
    arr = np.frombuffer(msg, dtype=np.uint8)
    crcs = [orc.crc32(arr[a:b]) for a, b in ranges]
    t0 = time.perf_counter()
    for _ in range(reps):
        for a, b in ranges:
            orc.crc32(arr[a:b])
    us = (time.perf_counter() - t0) / reps * 1e6
    assert mf.verify_message(msg, 0) == (0, len(msg))
    return {"config": "C1", "us_per_message_cpu": round(us, 2), "crc_bytes": sum(b - a for a, b in ranges),
            "message_bytes": len(msg), "record_crcs": [f"0x{c:08x}" for c in crcs],
            "records": ["header", "blob_properties", "user_metadata", "blob"], "cores": 1,
            "note": "oracle/crc32_ref.c via ctypes (includes ~1 us/record call overhead)"}


def gpu_region(mf, m, blob_bytes, reps, variant=None, host=False, mode="region"):
    import numpy as np
    import torch

    from ambry_amd import device as D

    torch.cuda.set_device(0)
    D.init(0)
    if variant is not None:
        D.set_variant(0, variant)
    D.set_region_mode(0, {"region": 1, "region2": 2, "jobs": 0}[mode])
    tmpl = mf.put_message(mf.store_key("blob-00000000"), mf.blob_properties_bytes(blob_bytes), b"u" * 1000,
                          bytes(blob_bytes), version=3)
    L = len(tmpl)
    v, total, rel = mf.parse_header(tmpl, 0)
    blob_rec = rel[4]
    c0 = blob_rec + 13
    region = torch.empty(m * L, dtype=torch.uint8, device="cuda")
    view = region.view(m, L)
    view[:] = torch.from_numpy(np.frombuffer(tmpl, dtype=np.uint8).copy()).cuda()
    rnd = torch.empty(m * blob_bytes, dtype=torch.uint8, device="cuda")
    D.fill_random(rnd, 0xC1, 0)
    view[:, c0:c0 + blob_bytes] = rnd.view(m, blob_bytes)
    del rnd
    base = torch.arange(m, dtype=torch.int64, device="cuda") * L
    crc = D.crc32_batch(region, base + blob_rec, torch.full((m,), L - 8 - blob_rec, dtype=torch.int64,
                                                            device="cuda"))
    c = crc.to(torch.int64) & 0xFFFFFFFF
    be = torch.stack([(c >> s) & 0xFF for s in (24, 16, 8, 0)], dim=1).to(torch.uint8)
    view[:, L - 8:L - 4] = 0
    view[:, L - 4:] = be
    torch.cuda.synchronize()
    status, end = D.verify_messages(region, base)
    torch.cuda.synchronize()
    # AMBRYCRC_PROBE=1: a timing-only probe build (tools/ab_build.sh), whose CRCs are wrong by design
    probe = os.environ.get("AMBRYCRC_PROBE") == "1"
    assert probe or int(status.abs().sum().item()) == 0, "clean region must verify"
    # inject corruption into 1 % of blobs and check the flags
    bad = torch.randperm(m, device="cuda")[: max(1, m // 100)]
    view[bad, c0 + 7] ^= 0x20
    status, _ = D.verify_messages(region, base)
    flagged = (status != 0).nonzero().flatten().sort().values
    assert probe or torch.equal(flagged, bad.sort().values), "corruption flags"
    assert probe or bool((status[bad] == mf.BLOB_CRC).all())
    view[bad, c0 + 7] ^= 0x20
    t_pre = time.perf_counter()  # clock ramp (see bench.py)
    while time.perf_counter() - t_pre < 0.3:
        D.verify_messages(region, base, want_end=False)
        torch.cuda.synchronize()
    times = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        D.verify_messages(region, base, want_end=False)
        e1.record()
        torch.cuda.synchronize()
        times.append(e0.elapsed_time(e1))
    times.sort()
    med = times[len(times) // 2]
    res = {"config": f"verify {m} x PUT({blob_bytes} B blob)", "variant": variant,
           "mode": mode if L <= int(os.environ.get("AMBRYCRC_REGION_MAX_PER_MESSAGE", "6144")) else
                   "jobs (region > cut-off per message)", "messages": m, "region_bytes": m * L,
           "ms_median": round(med, 4), "GiBps": round(m * L / (med / 1e3) / 2**30, 1),
           "messages_per_s": round(m / (med / 1e3)), "parity": "clean=0, 1% injected flips flagged exactly",
           "mode_taken": {0: "jobs", 1: "region one-pass", 2: "region two-pass"}.get(D.last_message_mode(0))}
    if host and m * L <= (5 << 30):
        res["host"] = host_region_rate(D, region, base, m, L)
    return res


def host_region_rate(D, region, base, m, L):
    """The same region from host memory through ambrycrc_verify_messages_host (PCIe-inclusive):
    pageable (numpy) and pinned (pin_memory) sources, best of 3 after one untimed pass."""
    import numpy as np

    host = region.cpu().numpy()
    offs = base.cpu().numpy().astype(np.uint64)
    D.set_host_policy(0, D.HOST_GPU)  # the GPU host path itself (the auto policy may pick the CPU leg)
    out = {}
    for name, src, pinned in (("pageable", host, False), ("pinned", None, True)):
        if pinned:
            import torch

            src = torch.from_numpy(host).pin_memory()
        st, _ = D.verify_messages_host(src, offs, pinned=pinned)
        assert int(st.sum()) == 0, "host verify of the clean region"
        best = None
        for _ in range(3):
            t0 = time.perf_counter()
            D.verify_messages_host(src, offs, pinned=pinned)
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        out[name + "_GiBps"] = round(m * L / best / 2**30, 2)
        del src
    out["what"] = "ambrycrc_verify_messages_host, synchronous, host region staged through the pinned slabs"
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--no-gpu", action="store_true")
    ap.add_argument("--variants", default="29")
    ap.add_argument("--cases", default="64k,4m,4k", help="subset of 64k,4m,4k,3k,2k,1k,100")
    ap.add_argument("--modes", default="region2", help="message-verify modes: region2 (two passes, the default), region (one pass), jobs")
    ap.add_argument("--host", action="store_true", help="also time the host-region path (regions <= 5 GiB)")
    args = ap.parse_args()
    mf = load_mf()
    print(json.dumps(c1_cpu(mf)), flush=True)
    if args.no_gpu:
        return
    cases = {"64k": (65536, 64 << 10), "4m": (4096, 4 << 20), "4k": (262144, 4 << 10), "3k": (327680, 3 << 10),
             "2k": (393216, 2 << 10), "1k": (524288, 1 << 10), "100": (1048576, 100),
             # 4 KiB blobs over smaller regions (~87 / 175 / 350 MB: inside / around the 256 MB MALL)
             "4k16k": (16384, 4 << 10), "4k32k": (32768, 4 << 10), "4k64k": (65536, 4 << 10)}
    for m, s in (cases[c] for c in args.cases.split(",")):
        for v in [int(x) for x in args.variants.split(",")]:
            for mode in args.modes.split(","):
                print(json.dumps(gpu_region(mf, m, s, args.reps, v, args.host, mode)), flush=True)


if __name__ == "__main__":
    main()
