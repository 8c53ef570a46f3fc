"""Summarize tools/pmc_cache.sh: per case and region kernel, each counter averaged over the kernel's
dispatches (the first, warm-up, dispatch dropped), plus the L2 hit rate and HBM read requests per
L2 request."""
import collections
import csv
import glob
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "pmc_cache")
for f in sorted(glob.glob(os.path.join(src, "*.p*.csv"))):
    case = os.path.basename(f).split(".")[0]
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].split("<")[0].split("::")[-1]
        if not k.startswith("region_"):
            continue
        per[(k, int(r["Dispatch_Id"]))][r["Counter_Name"]] += float(r["Counter_Value"])
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    seen = collections.Counter()
    for (k, d), cs in sorted(per.items(), key=lambda x: x[0][1]):
        seen[k] += 1
        if seen[k] == 1:
            continue
        for c, v in cs.items():
            agg[k][c].append(v)
    for k, cs in agg.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        extra = ""
        if "TCC_HIT_sum" in m and "TCC_MISS_sum" in m:
            tot = m["TCC_HIT_sum"] + m["TCC_MISS_sum"]
            extra = f" l2_hit={m['TCC_HIT_sum'] / tot:.3f}" if tot else ""
        print(f"{case:8s} {k:24s} " + " ".join(f"{c}={v:.4g}" for c, v in sorted(m.items())) + extra)
