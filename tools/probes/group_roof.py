#!/usr/bin/env python3
"""Read roof of the group phase's access shape (ambrycrc_debug_readbw_dev variant 16 + k: chunks of
1 KiB << k, 16-lane groups, 4 chunks per wave round, loads as group_load_sb) beside the sweep's
(variant 1), over the same 1 GiB buffer: best of 7 launches, GB/s. Prints one JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch

    from ambry_amd import device as D
    from ambry_amd._lib import check, lib

    torch.cuda.set_device(0)
    D.init(0)
    nbytes = 1 << 30
    buf = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    D.fill_random(buf, 5, 0)
    out = torch.empty(D.grid_size(0) * 1024, dtype=torch.int32, device="cuda")
    res = {}
    for name, v in (("sweep_shares_nt", 1), ("group_1k", 16), ("group_2k", 17), ("group_4k", 18), ("group_8k", 19),
                    ("group_16k", 20)):
        best = None
        for _ in range(7):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            check(lib().ambrycrc_debug_readbw_dev(buf.data_ptr(), nbytes, out.data_ptr(), v,
                                                  torch.cuda.current_stream().cuda_stream), "readbw")
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1)
            best = ms if best is None else min(best, ms)
        res[name] = round(nbytes / (best / 1e3) / 1e9, 1)
    print(json.dumps({"probe": "read roof by access shape, 1 GiB, GB/s", **res}))


if __name__ == "__main__":
    main()
