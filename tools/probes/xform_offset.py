#!/usr/bin/env python3
"""Probe: does the large-blob transform's time depend on where the output sits relative to the region?

Round-to-round, `transform 4096 x PUT(4 MiB blob)` (the general path) measured either ~6.0 ms or
7.1-7.4 ms with nothing changed in between (profiles/r05ao_put, r06z_put vs r05aw_put, r05x_put).
The only thing a run does not fix is the allocator's choice of the output address. This probe builds
the region once and runs the transform (and a plain hipMemcpyAsync of the same bytes, as a control)
into one large buffer at a list of byte offsets, printing one JSON line per offset:
the output's distance from the region modulo a few powers of two, and the median times."""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=4096)
    ap.add_argument("--blob", type=int, default=4 << 20)
    ap.add_argument("--reps", type=int, default=9)
    ap.add_argument("--offsets", default="0,256,4096,65536,1048576,2097152,3145728,16777216,100663296,1073741824")
    ap.add_argument("--fresh", type=int, default=4, help="also this many fresh torch.empty outputs")
    ap.add_argument("--fresh-first", action="store_true", help="the fresh outputs before the big buffer")
    ap.add_argument("--windows", default="", help="also time the transform at each sweep window (bytes; 0 = one round)")
    ap.add_argument("--round-to", default="", help="fresh outputs of cap rounded up to each of these byte counts")
    args = ap.parse_args()

    import numpy as np
    import torch

    from bench_put import _props_tensor
    from ambry_amd import device as D
    from ambry_amd.messages import PUT_DESC_DTYPE, PutMessage, layout, out_bound, serialize_dev, transform_dev

    torch.cuda.set_device(0)
    D.init(0)
    m, blob_bytes = args.m, args.blob
    key_len, props_len, um_len = 24, 94, 1000
    L, fo = layout(PutMessage(key=bytes(key_len), props=bytes(props_len), usermeta=bytes(um_len),
                              blob=bytes(blob_bytes)))
    descs = np.zeros(m, dtype=PUT_DESC_DTYPE)
    idx = np.arange(m, dtype=np.uint64)
    descs["out_off"] = idx * L
    descs["blob_len"] = blob_bytes
    descs["key_len"], descs["props_len"], descs["usermeta_len"] = key_len, props_len, um_len
    descs["enckey_len"] = -1
    descs["header_version"] = 3
    region = torch.empty(m * L, dtype=torch.uint8, device="cuda")
    D.fill_random(region[: (m * L) // 16 * 16], 3, 0)
    p0 = fo["props"]
    region.view(m, L)[:, p0:p0 + props_len] = _props_tensor(torch)
    serialize_dev(torch.from_numpy(descs.view(np.uint8).copy()).cuda(), region)
    offs = torch.from_numpy((idx * L).astype(np.int64)).cuda()
    cap = out_bound(m * L, m)
    offsets = [int(x) for x in args.offsets.split(",") if x]
    big = torch.empty(cap + max(offsets) + 4096, dtype=torch.uint8, device="cuda")
    nbytes = m * L

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(args.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        ts.sort()
        return ts[len(ts) // 2]

    def case(out, label):
        delta = out.data_ptr() - region.data_ptr()
        _, _, _, st = transform_dev(region, offs, out=out)
        torch.cuda.synchronize()
        ok = int(st.abs().sum().item()) == 0 and bool(torch.equal(out[:nbytes], region))
        t_x = timed(lambda: transform_dev(region, offs, out=out))
        t_c = timed(lambda: out[:nbytes].copy_(region))
        rec = {"out": label, "delta": delta, "delta_mod_4k": delta % 4096, "delta_mod_64k": delta % 65536,
               "delta_mod_2m": delta % (2 << 20), "delta_mod_16m": delta % (16 << 20),
               "transform_ms": round(t_x, 4), "copy_ms": round(t_c, 4),
               "transform_GBps_hbm": round(2 * nbytes / t_x / 1e6, 1), "copy_GBps": round(2 * nbytes / t_c / 1e6, 1),
               "path": D.last_transform_path(0), "ok": ok}
        for wdw in [int(x) for x in args.windows.split(",") if x]:
            D.set_window(0, wdw)
            rec[f"transform_ms_window_{wdw >> 20}M"] = round(timed(lambda: transform_dev(region, offs, out=out)), 4)
        if args.windows:
            D.set_window(0, 32 << 30)
        print(json.dumps(rec), flush=True)

    def fresh():
        for k in range(args.fresh):
            out = torch.empty(cap + 4096 * k, dtype=torch.uint8, device="cuda")
            case(out[:cap], f"fresh{k}")
            del out
        for r in [int(x) for x in args.round_to.split(",") if x]:
            torch.cuda.empty_cache()
            size = (cap + r - 1) // r * r
            out = torch.empty(size, dtype=torch.uint8, device="cuda")
            case(out[:cap], f"fresh_round{r}")
            del out

    if args.fresh_first:
        big_keep = big
        del big
        torch.cuda.empty_cache()
        fresh()
        big = big_keep
    for o in offsets:
        case(big[o:o + cap], f"big+{o}")
    del big
    torch.cuda.empty_cache()
    if not args.fresh_first:
        fresh()


if __name__ == "__main__":
    main()
