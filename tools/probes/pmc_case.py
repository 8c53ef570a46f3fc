#!/usr/bin/env python3
"""One small-record workload, launched `--reps` times back to back, for rocprofv3 passes
(tools/pmc_cases.sh). Every case checks its first result against zlib, then repeats the call
untimed; the profiler's per-dispatch counters are the measurement.

  batch100   chunks of 100 B at 112-B stride (16-B aligned starts), 0.5 GiB   -- group class 0
  batch1k    1 KiB chunks, aligned, 0.5 GiB                                     -- group class 1
  batch4k    4 KiB chunks, aligned, 0.5 GiB                                     -- group class 2
  batch4109  4109-B chunks at 16-B offsets (the blob records of 4 KiB PUTs)     -- group class 3
  batch2000  2000-B chunks, packed (8-B offsets); batch3000: 3000 B at 16-B offsets -- class 2
  batch16k   16 KiB chunks, aligned                                               -- class 3
  msg4k      ambrycrc_verify_messages_dev over 262,144 x PUT(4 KiB blob), 1.29 GiB (the default: region
             mode, two passes)
  msg1k      the same over 524,288 x PUT(1 KiB blob); msg3k with 3000 B blobs; msg100: 1,048,576 x 100 B
  <msg>_1pass / <msg>_jobs   in region mode's one-pass form / in job mode (<msg>_2pass = <msg>)
  scatter16 / scatter4 / scatter8   FETCH_SIZE calibration: every 128-B line of 1 GiB read once in
             scattered order by one 16-B / 4-B / unaligned 8-B load (ambrycrc_debug_readbw_dev 60-62)
  put4k      ambrycrc_serialize_puts_dev, copy mode, 262,144 x PUT(4 KiB blob); put4k_inplace in place
  xform4k    ambrycrc_transform_messages_dev over 262,144 stored PUT(4 KiB blob) messages (fast path)
  xform64k   the same over 65,536 PUT(64 KiB blob) messages
  single100  one 100 B chunk per ambrycrc_batch_dev call
  single4m   one 4 MiB chunk per ambrycrc_batch_dev call
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import zlib

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

# message-verify regions: (messages, blob bytes); msg4k16k / 32k / 64k: 4 KiB blobs over ~87 / 175 / 350 MB
MSG_CASES = {"msg4k": (262144, 4096), "msg3k": (262144, 3000), "msg1k": (524288, 1024), "msg100": (1048576, 100),
             "msg4k16k": (16384, 4096), "msg4k32k": (32768, 4096), "msg4k64k": (65536, 4096)}
SIZES = {"batch100": (100, 112), "batch1k": (1024, 1024), "batch4k": (4096, 4096), "batch4109": (4109, 4112),
         "batch2000": (2000, 2000), "batch3000": (3000, 3008), "batch16k": (16384, 16384)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("case")
    ap.add_argument("--reps", type=int, default=5)
    # timing probes of deliberately wrong kernels (tools/ab_cases.sh with a probe build) skip the check
    ap.add_argument("--no-check", action="store_true", default=bool(os.environ.get("AB_NO_CHECK")))
    ap.add_argument("--gib", type=float, default=0.5)
    args = ap.parse_args()
    import numpy as np
    import torch

    from ambry_amd import device as D

    torch.cuda.set_device(0)
    D.init(0)
    info = {"case": args.case}
    if args.case in SIZES:
        size, stride = SIZES[args.case]
        n = int(args.gib * 2**30) // stride
        buf = torch.empty(n * stride, dtype=torch.uint8, device="cuda")
        D.fill_random(buf, 0xA1 + size, 0)
        off = torch.arange(n, dtype=torch.int64, device="cuda") * stride
        ln = torch.full((n,), size, dtype=torch.int64, device="cuda")
        out = torch.empty(n, dtype=torch.int32, device="cuda")
        ws = torch.empty(D.workspace_bytes(n), dtype=torch.uint8, device="cuda")
        D.crc32_batch(buf, off, ln, out=out, workspace=ws)
        torch.cuda.synchronize()
        idx = [0, n // 2, n - 1]
        host = buf.view(n, stride)[idx, :size].cpu().numpy()
        assert args.no_check or [zlib.crc32(h.tobytes()) for h in host] == list(out[idx].cpu().numpy().view(np.uint32))
        for _ in range(args.reps):
            D.crc32_batch(buf, off, ln, out=out, workspace=ws)
        info.update(chunks=n, chunk_bytes=size, alg_bytes_per_launch=n * size + 4 * n)
    elif args.case in ("single100", "single4m"):
        size = 100 if args.case == "single100" else 4 << 20
        buf = torch.empty(size + 64, dtype=torch.uint8, device="cuda")
        D.fill_random(buf, 7, 0)
        off = torch.zeros(1, dtype=torch.int64, device="cuda")
        ln = torch.full((1,), size, dtype=torch.int64, device="cuda")
        out = torch.empty(1, dtype=torch.int32, device="cuda")
        ws = torch.empty(D.workspace_bytes(1), dtype=torch.uint8, device="cuda")
        D.crc32_batch(buf, off, ln, out=out, workspace=ws)
        torch.cuda.synchronize()
        assert args.no_check or zlib.crc32(buf[:size].cpu().numpy().tobytes()) == int(out.cpu().numpy().view(np.uint32)[0])
        for _ in range(args.reps):
            D.crc32_batch(buf, off, ln, out=out, workspace=ws)
        info.update(chunks=1, chunk_bytes=size, alg_bytes_per_launch=size + 4)
    elif args.case.split("_")[0] in MSG_CASES and args.case.split("_")[-1] in tuple(MSG_CASES) + ("2pass", "1pass", "jobs"):
        from bench_messages import gpu_region, load_mf

        m, blob = MSG_CASES[args.case.split("_")[0]]
        mode = "region" if args.case.endswith("_1pass") else "jobs" if args.case.endswith("_jobs") else "region2"
        res = gpu_region(load_mf(), m, blob, args.reps, mode=mode)
        info.update(res)
        # CRC'd bytes per message: header 32 + props + usermeta 1006 + blob record 4109 (+ stored CRCs read)
        info["alg_bytes_per_launch"] = res["region_bytes"]
    elif args.case in ("put4k", "put4k_inplace"):
        # ambrycrc_serialize_puts_dev, 262,144 PUTs with a 4 KiB blob: copy mode (fields and blobs in their
        # own buffers; the copy-through sweep reads, writes and CRCs each field) or in place
        from bench_put import run

        res = run(262144, 4096, args.reps, args.case == "put4k_inplace")
        info.update(res)
        info["alg_bytes_per_launch"] = res["hbm_bytes_min"]  # fields + blobs read, messages written (copy)
    elif args.case in ("xform4k", "xform64k"):
        # ambrycrc_transform_messages_dev over stored 4 KiB / 64 KiB-blob PUTs (the one-pass fast path
        # reads each message once and writes it once into the output)
        from bench_put import run_transform

        res = run_transform(262144, 4096, args.reps) if args.case == "xform4k" else run_transform(65536, 65536,
                                                                                                  args.reps)
        info.update(res)
        info["alg_bytes_per_launch"] = 2 * res["message_bytes"]
    elif args.case in ("scatter16", "scatter4", "scatter8"):
        from ambry_amd._lib import check, lib

        nbytes = 1 << 30
        buf = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
        D.fill_random(buf, 3, 0)
        scratch = torch.zeros(1024, dtype=torch.int32, device="cuda")
        v = {"scatter16": 60, "scatter4": 61, "scatter8": 62}[args.case]
        for _ in range(args.reps + 1):
            check(lib().ambrycrc_debug_readbw_dev(buf.data_ptr(), nbytes, scratch.data_ptr(), v,
                                                  torch.cuda.current_stream().cuda_stream), "readbw")
        info.update(lines=nbytes // 128, line_bytes=128, alg_bytes_per_launch=nbytes,
                    what="every 128-B line read once by one %s load" % args.case[7:] + "-B")
    else:
        raise SystemExit(f"unknown case {args.case}")
    torch.cuda.synchronize()
    print(json.dumps(info), flush=True)


if __name__ == "__main__":
    main()
