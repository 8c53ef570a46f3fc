#!/usr/bin/env python3
"""Host-resident CRC path probes (SURVEY.md §8d "host-resident rate"), one process, MI355X.

Bytes of a PUT arrive in host memory (a Netty ByteBuf, NettyServerRequest.java:35,54) and
GET/scrub bytes in a FileChannel prefetch (StoreMessageReadSet.java:170-188). This tool
times the ways those bytes can reach the CRC kernels:

  h2d_copy        one hipMemcpyAsync of the whole pinned buffer (SDMA): the PCIe H2D roof
  h2d_copy_4m     the same in 4 MiB pieces on one stream
  batch_host      ambrycrc_batch_host(pinned=1): slab-staged copies + kernels + D2H of CRCs
  batch_host_pg   ambrycrc_batch_host(pinned=0): pageable host memory (memcpy into pinned slabs)
  zero_copy       ambrycrc_batch_dev with base = the device alias of the pinned buffer
                  (the sweep kernel reads host memory over PCIe; no staging copy)

Usage: python tools/bench_hostpath.py [--mib 2048] [--reps 3] [--out gpurun_out/hostpath.jsonl]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=2048)
    ap.add_argument("--chunk-kib", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out", default=None)
    ap.add_argument("--only", default="", help="comma list of probe names")
    args = ap.parse_args()

    import numpy as np
    import torch

    from ambry_amd import device as D
    from ambry_amd._lib import check, lib

    torch.cuda.set_device(0)
    D.init(0)
    D.set_host_policy(0, D.HOST_GPU)  # the GPU host path itself (the auto policy may pick the CPU leg)
    L = lib()
    total = args.mib << 20
    chunk = args.chunk_kib << 10
    n = total // chunk
    host = torch.empty(total, dtype=torch.uint8).pin_memory()
    host.view(torch.int64).random_(generator=torch.Generator().manual_seed(7))
    dev = torch.empty(total, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()

    # reference CRCs: copy to device, device batch
    dev.copy_(host)
    off_t = torch.arange(n, dtype=torch.int64, device="cuda") * chunk
    len_t = torch.full((n,), chunk, dtype=torch.int64, device="cuda")
    ref = D.crc32_batch(dev, off_t, len_t).cpu().numpy().view(np.uint32)

    hip = ctypes.CDLL("libamdhip64.so.7", mode=ctypes.RTLD_GLOBAL)
    dptr = ctypes.c_void_p()
    rc = hip.hipHostGetDevicePointer(ctypes.byref(dptr), ctypes.c_void_p(host.data_ptr()), 0)
    zero_copy_ok = rc == 0 and dptr.value is not None

    results = []
    only = set(x for x in args.only.split(",") if x)

    def record(name, secs, extra=None):
        gibs = total / secs / 2**30
        r = {"probe": name, "bytes": total, "chunk": chunk, "s": round(secs, 5), "GiBps": round(gibs, 2),
             "GBps": round(total / secs / 1e9, 2)}
        if extra:
            r.update(extra)
        results.append(r)
        print(json.dumps(r), flush=True)

    def timeit(fn):
        fn()
        torch.cuda.synchronize()
        best = None
        for _ in range(args.reps):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            best = el if best is None else min(best, el)
        return best

    if not only or "h2d_copy" in only:
        record("h2d_copy", timeit(lambda: dev.copy_(host, non_blocking=True)))
    if not only or "h2d_copy_4m" in only:
        def pieces():
            for i in range(n):
                dev[i * chunk:(i + 1) * chunk].copy_(host[i * chunk:(i + 1) * chunk], non_blocking=True)
        record("h2d_copy_4m", timeit(pieces))
    if not only or "batch_host" in only:
        chunks = [(host.data_ptr() + i * chunk, chunk) for i in range(n)]
        got = None

        def bh():
            nonlocal got
            got = D.crc32_batch_host(chunks, device=0, pinned=True)
        record("batch_host", timeit(bh), {"parity": bool(np.array_equal(np.asarray(got, dtype=np.uint32), ref))})
    if not only or "batch_host_pg" in only:
        pg = host.numpy().copy()  # pageable
        chunks = [(pg.ctypes.data + i * chunk, chunk) for i in range(n)]
        got = None

        def bhp():
            nonlocal got
            got = D.crc32_batch_host(chunks, device=0, pinned=False)
        record("batch_host_pg", timeit(bhp), {"parity": bool(np.array_equal(np.asarray(got, dtype=np.uint32), ref))})
        del pg
    if (not only or "zero_copy" in only) and zero_copy_ok:
        out = torch.empty(n, dtype=torch.int32, device="cuda")

        def zc():
            check(L.ambrycrc_batch_dev(dptr, ctypes.c_void_p(off_t.data_ptr()), ctypes.c_void_p(len_t.data_ptr()),
                                       None, ctypes.c_void_p(out.data_ptr()), n, None, 0,
                                       ctypes.c_void_p(s.cuda_stream)), "zero-copy batch")
        secs = timeit(zc)
        record("zero_copy", secs, {"parity": bool(np.array_equal(out.cpu().numpy().view(np.uint32), ref)),
                                   "device_alias_equal_host_ptr": dptr.value == host.data_ptr()})
    elif not zero_copy_ok:
        print(json.dumps({"probe": "zero_copy", "skipped": f"hipHostGetDevicePointer rc={rc}"}), flush=True)

    if args.out:
        os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
        with open(args.out, "a") as f:
            for r in results:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
