#!/usr/bin/env python3
"""A/B probe (a library built with -DAMBRY_FUSED_PROBE=2, loaded through AMBRYCRC_LIBRARY): per
workgroup of the one-pass region kernel, when its streamers and its processors finished, relative
to its start (s_memrealtime, 100 MHz), for the message-verify case given (tools/bench_messages.py's
gpu_region), or the transform case given as x4k / x64k / x4m (tools/bench_put.py's run_transform: the
copy form). Prints the distribution over workgroups."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import numpy as np

    from ambry_amd._lib import lib
    from bench_messages import gpu_region, load_mf

    case = sys.argv[1] if len(sys.argv) > 1 else "4k"
    if case.startswith("x"):
        import torch
        from ambry_amd import device as D
        from bench_put import run_transform

        torch.cuda.set_device(0)
        D.init(0)
        m, blob = {"x4k": (262144, 4096), "x64k": (65536, 65536), "x4m": (4096, 4 << 20)}[case]
        res = run_transform(m, blob, 5)
        res["config"] = res["case"]
    else:
        m, blob = {"4k": (262144, 4096), "1k": (524288, 1024), "100": (1048576, 100)}[case]
        res = gpu_region(load_mf(), m, blob, 5)
    n = 256
    buf = (ctypes.c_ulonglong * (3 * 2048))()
    fn = lib().ambrycrc_debug_fused_times
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    assert fn(buf, 2048) == 0
    t = np.frombuffer(buf, dtype=np.uint64).reshape(2048, 3)[:n].astype(np.int64)
    s_end = (t[:, 1] - t[:, 0]) / 100.0  # us
    p_end = (t[:, 2] - t[:, 0]) / 100.0
    start = (t[:, 0] - t[:, 0].min()) / 100.0
    q = lambda a: [round(float(np.percentile(a, x)), 1) for x in (0, 50, 90, 100)]  # noqa: E731
    print(json.dumps({"case": res["config"], "ms_median": res["ms_median"], "wg_start_spread_us": q(start),
                      "stream_end_us": q(s_end), "proc_end_us": q(p_end), "proc_after_stream_us": q(p_end - s_end)}))


if __name__ == "__main__":
    main()
