#!/usr/bin/env python3
"""Debug probe: one two-pass region verify of build_region(n, seed) (tests/test_message_format.py),
status compared with the oracle; argv: n seed big_every."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import numpy as np
    import torch

    from ambry_amd import device as D
    from test_message_format import build_region

    n, seed, big = int(sys.argv[1]), int(sys.argv[2]), int(float(sys.argv[3]))
    region, offs, expect = build_region(n=n, seed=seed, corrupt_frac=0.08, big_every=big)
    torch.cuda.set_device(0)
    D.init(0)
    D.set_region_mode(0, 2)
    r = torch.from_numpy(np.frombuffer(region, dtype=np.uint8).copy()).cuda()
    o = torch.tensor(np.asarray(offs, dtype=np.int64), device="cuda")
    print("launch", flush=True)
    st, end = D.verify_messages(r, o)
    torch.cuda.synchronize()
    st = st.cpu().numpy().view(np.uint32).tolist()
    bad = [i for i, (s, (es, _)) in enumerate(zip(st, expect)) if s != es]
    print("mode", D.last_message_mode(0), "mismatches", len(bad), bad[:5], flush=True)


if __name__ == "__main__":
    main()
