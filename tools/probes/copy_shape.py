"""Copy roof of the group phase's store shape (ambrycrc_debug_readbw_dev variants 32+): reads
nbytes/2 and writes them to the upper half, in the group phase's access shape (4 chunks per wave
round, 256-B runs per 16-lane group) against a contiguous per-wave copy (variant 48). Prints one
JSON line per variant: GB/s counting read + write bytes."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=4.0)
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    import torch

    from ambry_amd import device as D
    from ambry_amd._lib import check, lib

    torch.cuda.set_device(0)
    D.init(0)
    nbytes = int(args.gib * (1 << 30))
    buf = torch.zeros(nbytes, dtype=torch.uint8, device="cuda")
    scratch = torch.zeros(256 * 1024 * 4, dtype=torch.int32, device="cuda")
    moved = 2 * (nbytes // 2 - 4096)
    for v, name in [(49, "grid-stride"), (50, "grid-stride, nt stores"), (48, "contiguous"), (32, "group 1 KiB"), (34, "group 4 KiB"), (36, "group 16 KiB"),
                    (42, "group 4 KiB, dst +11 B")]:
        s = torch.cuda.current_stream()
        times = []
        for r in range(args.reps + 2):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            check(lib().ambrycrc_debug_readbw_dev(buf.data_ptr(), nbytes, scratch.data_ptr(), v, s.cuda_stream),
                  "readbw")
            e1.record(s)
            torch.cuda.synchronize()
            if r >= 2:
                times.append(e0.elapsed_time(e1))
        times.sort()
        ms = times[len(times) // 2]
        print(json.dumps({"variant": v, "shape": name, "ms": round(ms, 4), "GBps_read_plus_write": round(moved / ms / 1e6, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
