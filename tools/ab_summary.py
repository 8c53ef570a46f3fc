"""Summarize tools/ab_cases.sh: per case and library build, the average duration of the batch's
CRC kernels (crc32_sweep_kernel, plus crc32_group_kernel where it runs; AB_MATCH=comma-separated
name substrings for other kernels) over the interleaved rounds, and each build's ratio to the
first."""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "ab")
res = {}
for f in sorted(glob.glob(os.path.join(src, "*", "*", "r*", "kt_kernel_stats.csv"))):
    tag, case, rnd = f.split(os.sep)[-4:-1]
    # the batch's CRC kernels: the sweep, plus the group kernel of variant 31 (one call each per batch)
    match = os.environ.get("AB_MATCH", "sweep_kernel,group_kernel").split(",")
    us = sum(float(r["AverageNs"]) / 1e3 for r in csv.DictReader(open(f)) if any(m in r["Name"] for m in match))
    res.setdefault(case, {}).setdefault(tag, []).append(us)
out = {}
for case, by in res.items():
    tags = sorted(by)
    base = None
    for t in tags:
        us = sum(by[t]) / len(by[t])
        base = base or us
        out.setdefault(case, {})[t] = {"us_per_round": [round(x, 1) for x in by[t]], "avg_us": round(us, 1),
                                       "vs_first": round(base / us, 3)}
        print(f"{case:10s} {t:12s} {us:9.1f} us  {base / us:6.3f}x  {by[t]}")
json.dump(out, open(os.path.join(src, "summary.json"), "w"), indent=1)
