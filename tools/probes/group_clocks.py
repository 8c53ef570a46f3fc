#!/usr/bin/env python3
"""Where a group-phase wave's time goes: run with AMBRYCRC_LIBRARY pointing at a probe build of
libambrycrc.so whose sweep kernel stamps s_memtime (tools/ab_build.sh over an instrumented
crc32_kernels.hip exporting ambrycrc_probe_clocks). Per wave the build records kernel entry,
after the LDS fill, after the group phase, and per group round the time to descriptors ready
(`meta`), through the chain (`crc`), and the store (`store`). Prints the averages over waves. The instrumented kernel is not kept in the tree (it is
the group phase with `s_memtime` stamps stored per wave into a `__device__` array, plus an
`ambrycrc_probe_clocks` reader); s_memtime counters are per XCD, so only differences within a
wave are meaningful.

  python tools/probes/group_clocks.py batch4k|batch1k|batch100 [--reps 3]
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

SIZES = {"batch100": (100, 112), "batch1k": (1024, 1024), "batch4k": (4096, 4096), "batch4109": (4109, 4112)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("case")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--gib", type=float, default=0.5)
    args = ap.parse_args()
    import numpy as np
    import torch

    from ambry_amd import _lib, device as D

    D.init(0)
    size, stride = SIZES[args.case]
    n = int(args.gib * (1 << 30)) // stride
    buf = torch.randint(0, 256, (n * stride,), dtype=torch.uint8, device="cuda")
    off = torch.arange(n, dtype=torch.int64, device="cuda") * stride
    ln = torch.full((n,), size, dtype=torch.int64, device="cuda")
    for _ in range(args.reps):
        D.crc32_batch(buf, off, ln)
    torch.cuda.synchronize()
    clk = (ctypes.c_uint64 * (8192 * 8))()
    rc = _lib.lib().ambrycrc_probe_clocks(clk, ctypes.c_size_t(8192 * 8))
    assert rc == 0, rc
    a = np.frombuffer(clk, dtype=np.uint64).reshape(8192, 8).astype(np.float64)
    live = a[:, 7] > 0
    k0 = a[live, 0].min()
    res = {
        "case": args.case, "waves_with_group_work": int(live.sum()),
        "lds_fill": float(np.mean(a[live, 1] - a[live, 0])),
        "group_phase": float(np.mean(a[live, 2] - a[live, 1])),
        "start_spread": float(np.max(a[live, 0] - k0)),
        "group_end_max_from_first_start": float(np.max(a[live, 2] - k0)),
        "rounds_per_wave": float(np.mean(a[live, 7])),
        "meta_per_round": float(np.mean(a[live, 4] / a[live, 7])),
        "crc_per_round": float(np.mean(a[live, 5] / a[live, 7])),
        "store_per_round": float(np.mean(a[live, 6] / a[live, 7])),
        "unit": "s_memtime ticks",
    }
    print(json.dumps(res))


if __name__ == "__main__":
    main()
