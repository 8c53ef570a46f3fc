#!/usr/bin/env python3
"""A/B sweep of sweep-kernel variants / grid sizes and the read-bandwidth roof, in ONE process.

Interleaved rounds (cdna_hip_programming.md §5.4 rule 24): every configuration is
timed once per round, R rounds, and the median/min per configuration reported.
Times are HIP-event kernel durations (ambrycrc timing hook) and stream wall time.
Usage: python tools/sweep.py [--config c3|c2|c4] [--rounds 5] [--variants 0,29] [--grids 0,512]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=3, help="launches per measurement")
    ap.add_argument("--variants", default="0,29")
    ap.add_argument("--grids", default="0")
    ap.add_argument("--readbw", action="store_true")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()

    import numpy as np
    import torch

    from ambry_amd import device as D
    from ambry_amd._lib import check, lib

    torch.cuda.set_device(0)
    D.init(0)
    if args.config == "c3":
        n, chunk = 8192, 4 << 20
        sizes = np.full(n, chunk, dtype=np.int64)
    elif args.config == "c2":
        n, chunk = 65536, 64 << 10
        sizes = np.full(n, chunk, dtype=np.int64)
    else:
        from datagen import zipf_sizes

        sizes = zipf_sizes(32768)
        n = len(sizes)
    off = np.concatenate([[0], np.cumsum((sizes + 15) // 16 * 16)[:-1]]).astype(np.int64)
    total = int(off[-1] + sizes[-1])
    buf = torch.empty(total, dtype=torch.uint8, device="cuda")
    D.fill_random(buf, 0xA3B1C2D3, 0)
    off_t = torch.from_numpy(off).cuda()
    len_t = torch.from_numpy(sizes).cuda()
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    rb_out = torch.empty(D.grid_size(0) * 1024 * 32, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()

    configs = []
    if args.readbw:
        configs += [("readbw", v, None) for v in (0, 1, 2, 3, 4)]
    for v in [int(x) for x in args.variants.split(",") if x]:
        for t in [int(x) for x in args.grids.split(",") if x]:
            configs.append(("crc", v, t))

    # clock ramp (see bench.py): ~0.3 s of the default kernel before measuring
    t_pre = time.perf_counter()
    while time.perf_counter() - t_pre < 0.3:
        D.crc32_batch(buf, off_t, len_t, out=out)
        torch.cuda.synchronize()

    results = {c: [] for c in configs}
    ref = None
    for r in range(args.rounds):
        for c in configs:
            kind, v, t = c
            if kind == "readbw":
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.reps):
                    D.set_grid(0, 0)
                    check(lib().ambrycrc_debug_readbw_dev(buf.data_ptr(), total & ~((256 << 10) - 1),
                                                          rb_out.data_ptr(), v,
                                                          torch.cuda.current_stream().cuda_stream),
                          "readbw")
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / args.reps
                results[c].append({"kernel_ms": ms, "wall_ms": ms,
                                   "bytes": total & ~((256 << 10) - 1)})
                continue
            D.set_variant(0, v)
            D.set_grid(0, t)
            D.timing_enable(0, True)
            torch.cuda.synchronize()
            D.timing_collect(0)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                D.crc32_batch(buf, off_t, len_t, out=out)
            e1.record()
            torch.cuda.synchronize()
            kms, cnt = D.timing_collect(0)
            D.timing_enable(0, False)
            got = out.cpu().numpy().copy()
            if ref is None:
                ref = got
            ok = bool((got == ref).all())
            results[c].append({"kernel_ms": kms / cnt, "wall_ms": e0.elapsed_time(e1) / args.reps,
                               "bytes": total, "consistent": ok})
        print(f"[sweep] round {r + 1}/{args.rounds} done", file=sys.stderr, flush=True)

    lines = []
    for c, rs in results.items():
        kind, v, t = c
        k = [x["kernel_ms"] for x in rs]
        w = [x["wall_ms"] for x in rs]
        b = rs[0]["bytes"]
        rec = {"config": args.config, "kind": kind, "variant": v, "grid": t,
               "kernel_ms_med": round(statistics.median(k), 4), "kernel_ms_min": round(min(k), 4),
               "wall_ms_med": round(statistics.median(w), 4),
               "kernel_GBps_med": round(b / (statistics.median(k) / 1e3) / 1e9, 1),
               "wall_GiBps_med": round(b / (statistics.median(w) / 1e3) / 2**30, 1),
               "consistent": all(x.get("consistent", True) for x in rs)}
        lines.append(rec)
        print(json.dumps(rec), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            for rec in lines:
                f.write(json.dumps(rec) + "\n")


if __name__ == "__main__":
    main()
