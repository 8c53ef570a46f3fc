#!/usr/bin/env python3
"""C5 layout probe: is the read roof over 256 GiB resident set by the allocation (one 256 GiB
tensor) or by the bytes (footprint)? Times the read-only probe (sweep grid and access shape,
ambrycrc_debug_readbw_dev variant 1) and the CRC batch over
  (a) 8 separate 32 GiB tensors, one launch each, back to back;
  (b) one 256 GiB tensor, as one launch and as 8 launches over consecutive 32 GiB windows.
Prints one JSON line per measurement (GB/s, best of 3)."""
from __future__ import annotations

import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import torch

    from ambry_amd import device as D
    from ambry_amd._lib import check, lib

    torch.cuda.set_device(0)
    D.init(0)
    GiB = 1 << 30
    part = 32 * GiB
    scratch = torch.empty(D.grid_size(0) * 1024, dtype=torch.int32, device="cuda")

    def readbw(ptrs_sizes, reps=3):
        best = None
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for p, n in ptrs_sizes:
                check(lib().ambrycrc_debug_readbw_dev(p, n, scratch.data_ptr(), 1,
                                                      torch.cuda.current_stream().cuda_stream), "readbw")
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1)
            best = ms if best is None else min(best, ms)
        return sum(n for _, n in ptrs_sizes) / (best / 1e3) / 1e9

    def crc(bufs, reps=3):
        n = 8192
        off = torch.arange(n, dtype=torch.int64, device="cuda") * (4 << 20)
        ln = torch.full((n,), 4 << 20, dtype=torch.int64, device="cuda")
        best = None
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for b in bufs:
                D.crc32_batch(b, off, ln)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1)
            best = ms if best is None else min(best, ms)
        return len(bufs) * part / (best / 1e3) / 1e9

    def warm(fn):
        t = time.perf_counter()
        while time.perf_counter() - t < 0.5:
            fn()

    parts = [torch.empty(part, dtype=torch.uint8, device="cuda") for _ in range(8)]
    for i, p in enumerate(parts):
        D.fill_random(p, 0x5EED + i, 0)
    torch.cuda.synchronize()
    warm(lambda: readbw([(parts[0].data_ptr(), part)], 1))
    print(json.dumps({"layout": "8 x 32 GiB tensors", "what": "readbw, 8 launches",
                      "GBps": round(readbw([(p.data_ptr(), part) for p in parts]), 1)}), flush=True)
    print(json.dumps({"layout": "8 x 32 GiB tensors", "what": "crc32_batch, 8 launches",
                      "GBps": round(crc(parts), 1)}), flush=True)
    del parts, p
    torch.cuda.empty_cache()

    big = torch.empty(8 * part, dtype=torch.uint8, device="cuda")
    D.fill_random(big, 0x5EED, 0)
    torch.cuda.synchronize()
    warm(lambda: readbw([(big.data_ptr(), part)], 1))
    print(json.dumps({"layout": "1 x 256 GiB tensor", "what": "readbw, 1 launch",
                      "GBps": round(readbw([(big.data_ptr(), 8 * part)]), 1)}), flush=True)
    print(json.dumps({"layout": "1 x 256 GiB tensor", "what": "readbw, 8 launches over 32 GiB windows",
                      "GBps": round(readbw([(big.data_ptr() + i * part, part) for i in range(8)]), 1)}), flush=True)
    views = [big[i * part:(i + 1) * part] for i in range(8)]
    print(json.dumps({"layout": "1 x 256 GiB tensor", "what": "crc32_batch, 8 launches over 32 GiB windows",
                      "GBps": round(crc(views), 1)}), flush=True)


if __name__ == "__main__":
    main()
