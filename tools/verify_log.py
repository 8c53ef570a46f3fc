#!/usr/bin/env python3
"""Verify an Ambry log segment file on the GPU: the scan BlobStoreRecovery.recover runs
(ambry-store/.../BlobStoreRecovery.java:43-110), with every CRC checked the way
deserializeBlobAll checks it (MessageFormatRecord.java:257-303).

  1. the 18-byte LogSegment header (version 0, capacity, CRC; LogSegment.java:130-140), unless
     --no-header (a bare message region);
  2. the message chain from the first message (ambrycrc_chain_messages_host: header hops until a
     header fails or the data ends);
  3. every message's header and record CRCs (ambrycrc_verify_messages_host: the file is mapped,
     staged through pinned slabs, verified by the gfx950 kernels).

Prints one JSON line: messages found, messages with a CRC or layout error (offset and status
bits of the first few), where the chain stopped, bytes and GiB/s of the verify call.
"""
from __future__ import annotations

import argparse
import json
import mmap
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def verify_log(path: str, header: bool = True, device: int = 0, max_messages: int = 1 << 22, repeat: int = 1) -> dict:
    import numpy as np

    from ambry_amd import device as D
    from ambry_amd import store_files

    D.init(device)
    size = os.path.getsize(path)
    with open(path, "rb") as f:
        # MAP_POPULATE: the pages are mapped at once, not faulted in one by one by the header
        # pass and the copy threads (4 KiB faults held a 4 GiB file to ~20 GiB/s)
        flags = mmap.MAP_SHARED | getattr(mmap, "MAP_POPULATE", 0)
        m = mmap.mmap(f.fileno(), 0, flags=flags, prot=mmap.PROT_READ) if size else None
    try:
        region = np.frombuffer(m, dtype=np.uint8) if m is not None else np.zeros(0, dtype=np.uint8)
        start = 0
        result = {"file": path, "bytes": size}
        if header:
            hdr = bytes(region[:store_files.LOG_SEGMENT_HEADER_SIZE])
            result["log_header_intact"] = store_files.log_segment_header_intact(hdr)
            start = store_files.LOG_SEGMENT_HEADER_SIZE
        offs = D.chain_messages_host(region, start, max_messages) if size > start else []
        result["messages"] = len(offs)
        if offs:
            times = []
            for _ in range(max(1, repeat)):  # the first call also allocates the pinned slabs
                t0 = time.perf_counter()  # the verify call only (the map and the chain are before it)
                status, end = D.verify_messages_host(region, offs, device=device)
                times.append(time.perf_counter() - t0)
            dt = min(times)
            last_end = int(end[-1]) if end[-1] else int(offs[-1])
            bad = [(int(o), int(s)) for o, s in zip(offs, status) if s]
            result.update({
                "corrupt": len(bad),
                "first_corrupt": [{"offset": o, "status": hex(s)} for o, s in bad[:10]],
                "chain_end": last_end,
                "unscanned_tail_bytes": size - last_end,
                "verify_s": round(dt, 4),
                "first_call_s": round(times[0], 4),
                "verify_GiBps": round((last_end - start) / dt / 2**30, 2) if dt > 0 else None,
            })
        return result
    finally:
        del region
        if m is not None:
            m.close()


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("path")
    ap.add_argument("--no-header", action="store_true", help="the file is a bare message region")
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--repeat", type=int, default=1, help="verify N times, report the fastest (and the first)")
    args = ap.parse_args()
    print(json.dumps(verify_log(args.path, header=not args.no_header, device=args.device, repeat=args.repeat)))


if __name__ == "__main__":
    main()
