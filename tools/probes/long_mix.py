#!/usr/bin/env python3
"""Message verify of a region of small PUTs with a few multi-MiB blobs among them (the
region-mode cliff): 240,000 PUTs with a 4 KiB blob and 8 with a 4 MiB blob spread through them
(~5.5 KiB of region per message: region mode). Times ambrycrc_verify_messages_dev in each form and
checks every status is 0 and that a flipped byte in one long blob is flagged."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    import numpy as np
    import torch

    from ambry_amd import device as D
    from bench_messages import load_mf

    mf = load_mf()
    torch.cuda.set_device(0)
    D.init(0)
    small = mf.put_message(mf.store_key("s"), mf.blob_properties_bytes(4096), b"u" * 1000, bytes(range(256)) * 16,
                           version=3)
    big = mf.put_message(mf.store_key("b"), mf.blob_properties_bytes(4 << 20), b"u" * 1000,
                         np.random.default_rng(1).integers(0, 256, 4 << 20, dtype=np.uint8).tobytes(), version=3)
    n_small, n_big = 240000, 8
    every = n_small // n_big
    parts, offs, pos = [], [], 0
    ts, tb = torch.frombuffer(bytearray(small), dtype=torch.uint8), torch.frombuffer(bytearray(big), dtype=torch.uint8)
    big_at = []
    for j in range(n_big):
        parts.append(ts.repeat(every))
        offs += [pos + len(small) * q for q in range(every)]
        pos += len(small) * every
        parts.append(tb)
        big_at.append(pos)
        offs.append(pos)
        pos += len(big)
    region = torch.cat(parts).cuda()
    off = torch.tensor(offs, dtype=torch.int64, device="cuda")
    out = {"case": f"verify {n_small} x PUT(4 KiB blob) + {n_big} x PUT(4 MiB blob)", "region_bytes": pos,
           "bytes_per_message": round(pos / len(offs))}
    for name, mode in (("region2", 2), ("region", 1), ("jobs", 0)):
        D.set_region_mode(0, mode)
        st, _ = D.verify_messages(region, off)
        torch.cuda.synchronize()
        assert int(st.abs().sum().item()) == 0, name
        times = []
        for _ in range(5):
            t0 = time.perf_counter()
            D.verify_messages(region, off)
            torch.cuda.synchronize()
            times.append((time.perf_counter() - t0) * 1e3)
        out[name + "_ms"] = round(sorted(times)[2], 3)
        out[name + "_taken"] = D.last_message_mode(0)
    region[big_at[3] + 5000] ^= 1
    for mode in (2, 1, 0):
        D.set_region_mode(0, mode)
        st, _ = D.verify_messages(region, off)
        bad = (st != 0).nonzero().flatten().cpu().tolist()
        assert bad == [offs.index(big_at[3])], (mode, bad[:5])
    D.set_region_mode(0, 2)
    out["flip_flagged"] = True
    print(json.dumps(out))


if __name__ == "__main__":
    main()
