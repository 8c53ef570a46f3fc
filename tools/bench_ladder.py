#!/usr/bin/env python3
"""Per-size table on Crc32Benchmark's ladder (SURVEY.md §8a a14 / §8d "CPU baseline").

Crc32Benchmark.java:43-44 times one buffer per call at sizes 100 B ... 4 MiB
(10 buffers, 500 iterations) and reports µs per call. For each ladder size this prints:
  gpu_batch   chunks of that size packed at 16-B-aligned offsets, about --gib of them in
              HBM, one ambrycrc_batch_dev call (plan + sweep); sweep-kernel time (HIP
              events, ambrycrc timing hook) and stream wall time, median of --reps
  gpu_call    ONE chunk per ambrycrc_batch_dev call, µs per call (stream wall): the
              latency floor a Crc32Benchmark-style caller sees
  cpu         oracle/crc32_ref.c (C restatement of Crc32.java slice-by-8) and zlib.crc32
              (the java.util.zip.CRC32 stand-in), one thread, µs per call and GB/s, over
              10 buffers x enough iterations for ~0.3 s
One JSON line per size. --no-gpu runs the CPU columns only.

The oracle appears here only as the CPU baseline being timed (and as the checker of the GPU
results), the role bench.py's cpu_baseline leg gives it; nothing GPU-side calls it.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time
import zlib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

LADDER = [100, 1 << 10, 4 << 10, 16 << 10, 64 << 10, 256 << 10, 1 << 20, 4 << 20]


def cpu_row(size: int, target_s: float = 0.3):
    import numpy as np

    from conftest import Oracle
    from datagen import stream_bytes

    orc = Oracle()
    bufs = [stream_bytes(0xB0 + i, 0, size) for i in range(10)]
    raw = [b.tobytes() for b in bufs]
    ptrs = [(b, b.ctypes.data) for b in bufs]
    fn = orc.L.oracle_crc32
    for b, r in zip(bufs, raw):
        assert fn(0, b.ctypes.data, size) == zlib.crc32(r)
    out = {}
    for name, call in (("restatement", lambda i: fn(0, ptrs[i][1], size)), ("zlib", lambda i: zlib.crc32(raw[i]))):
        iters, el = 1, 0.0
        while True:
            t0 = time.perf_counter()
            for _ in range(iters):
                for i in range(10):
                    call(i)
            el = time.perf_counter() - t0
            if el > target_s:
                break
            iters *= 4
        us = el / (iters * 10) * 1e6
        out[name] = {"us_per_call": round(us, 3), "GBps": round(size / us / 1e3, 3)}
    # Python->C call overhead (measured with a 0-byte call) is included in the per-call numbers.
    t0 = time.perf_counter()
    for _ in range(100000):
        fn(0, ptrs[0][1], 0)
    out["call_overhead_us"] = round((time.perf_counter() - t0) / 100000 * 1e6, 3)
    return out


def gpu_rows(size: int, gib: float, reps: int, variant: int = 0, check: bool = True):
    import numpy as np
    import torch

    from ambry_amd import device as D

    stride = (size + 15) // 16 * 16
    n = max(1, int(gib * 2**30) // stride)
    buf = torch.empty(n * stride, dtype=torch.uint8, device="cuda")
    D.fill_random(buf, 0xA1 + size, 0)
    off = torch.arange(n, dtype=torch.int64, device="cuda") * stride
    ln = torch.full((n,), size, dtype=torch.int64, device="cuda")
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    ws = torch.empty(D.workspace_bytes(n), dtype=torch.uint8, device="cuda")
    default = D.get_variant(0)
    D.set_variant(0, variant)
    D.crc32_batch(buf, off, ln, out=out, workspace=ws)
    torch.cuda.synchronize()
    # spot-check a few chunks against zlib
    idx = [0, n // 2, n - 1]
    host = buf.view(n, stride)[idx, :size].cpu().numpy()
    got = out[idx].cpu().numpy().view(np.uint32)
    if check:
        assert [zlib.crc32(h.tobytes()) for h in host] == list(got), "ladder parity"
    t_pre = time.perf_counter()
    while time.perf_counter() - t_pre < 0.3:
        D.crc32_batch(buf, off, ln, out=out, workspace=ws)
        torch.cuda.synchronize()
    kt, wt = [], []
    D.timing_enable(0, True)
    try:
        for _ in range(reps):
            D.timing_collect(0)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            D.crc32_batch(buf, off, ln, out=out, workspace=ws)
            e1.record()
            torch.cuda.synchronize()
            wt.append(e0.elapsed_time(e1))
            ms, cnt = D.timing_collect(0)
            kt.append(ms)
    finally:
        D.timing_enable(0, False)
    k, w = statistics.median(kt), statistics.median(wt)
    batch = {"chunks": n, "bytes": n * size, "kernel_ms": round(k, 4), "wall_ms": round(w, 4),
             "kernel_GBps": round(n * size / k / 1e6, 1), "wall_GiBps": round(n * size / (w / 1e3) / 2**30, 1),
             "meta_bytes_per_chunk": 16 + 4}
    # single-chunk calls
    o1, l1 = off[:1].clone(), ln[:1].clone()
    out1 = torch.empty(1, dtype=torch.int32, device="cuda")
    ws1 = torch.empty(D.workspace_bytes(1), dtype=torch.uint8, device="cuda")
    for _ in range(50):
        D.crc32_batch(buf, o1, l1, out=out1, workspace=ws1)
    torch.cuda.synchronize()
    calls = 500
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(calls):
        D.crc32_batch(buf, o1, l1, out=out1, workspace=ws1)
    e1.record()
    torch.cuda.synchronize()
    host_us = (time.perf_counter() - t0) / calls * 1e6
    call = {"us_per_call_stream": round(e0.elapsed_time(e1) / calls * 1e3, 2), "us_per_call_host": round(host_us, 2)}
    # the same calls straight through the C ABI (ctypes, arguments prepared once): what a JNI
    # caller pays, without the torch wrapper's per-call tensor checks and stream lookup
    import ctypes

    from ambry_amd._lib import lib

    L = lib()
    args = (ctypes.c_void_p(buf.data_ptr()), ctypes.c_void_p(o1.data_ptr()), ctypes.c_void_p(l1.data_ptr()), None,
            ctypes.c_void_p(out1.data_ptr()), 1, ctypes.c_void_p(ws1.data_ptr()), ws1.numel(),
            ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    fn = L.ambrycrc_batch_dev
    for _ in range(50):
        fn(*args)
    torch.cuda.synchronize()
    e0.record()
    t0 = time.perf_counter()
    for _ in range(calls):
        fn(*args)
    e1.record()
    torch.cuda.synchronize()
    call["us_per_call_abi_host"] = round((time.perf_counter() - t0) / calls * 1e6, 2)
    call["us_per_call_abi_stream"] = round(e0.elapsed_time(e1) / calls * 1e3, 2)
    # the same call captured once in a HIP graph (torch.cuda.CUDAGraph) and replayed:
    # the launch-bound single-chunk case without per-launch submission cost
    g = torch.cuda.CUDAGraph()
    cap = torch.cuda.Stream()
    cap.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(cap):
        D.crc32_batch(buf, o1, l1, out=out1, workspace=ws1)  # warm on the capture stream
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=cap):
            D.crc32_batch(buf, o1, l1, out=out1, workspace=ws1)
    torch.cuda.synchronize()
    for _ in range(20):
        g.replay()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(calls):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    call["us_per_call_graph_stream"] = round(e0.elapsed_time(e1) / calls * 1e3, 2)
    D.set_variant(0, default)
    del buf, off, ln, out, ws
    torch.cuda.empty_cache()
    return batch, call


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=2.0)
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--no-gpu", action="store_true")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--variants", default="29", help="sweep variants (0 or 29; 100-102 only in a -DAMBRYCRC_DIAGNOSTICS build)")
    ap.add_argument("--sizes", default=None, help="subset of the ladder, comma separated bytes")
    args = ap.parse_args()
    if not args.no_gpu:
        import torch

        from ambry_amd import device as D

        torch.cuda.set_device(0)
        D.init(0)
    sizes = LADDER if not args.sizes else [int(x) for x in args.sizes.split(",")]
    for size in sizes:
        row = {"size": size}
        if not args.no_cpu:
            row["cpu_1thread"] = cpu_row(size)
        if not args.no_gpu:
            for v in [int(x) for x in args.variants.split(",")]:
                row["variant"] = v
                row["gpu_batch"], row["gpu_call"] = gpu_rows(size, args.gib, args.reps, v, check=v < 100)
                print(json.dumps(row), flush=True)
        else:
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
