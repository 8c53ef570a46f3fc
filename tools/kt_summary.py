#!/usr/bin/env python3
"""Median kernel durations per case from tools/kt_cases.sh output: prints, per case, each kernel's
median and call count and the case's JSON line (mode taken, ms per call)."""
import collections
import csv
import glob
import json
import os
import sys


def main(root):
    for d in sorted(glob.glob(os.path.join(root, "*", ""))):
        case = os.path.basename(os.path.dirname(d))
        kt = os.path.join(d, "kt_kernel_trace.csv")
        if not os.path.exists(kt):
            continue
        per = collections.defaultdict(list)
        for r in csv.DictReader(open(kt)):
            name = r["Kernel_Name"].split("(")[0].split("<")[0].replace("ambrycrc::", "")
            per[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
        info = {}
        for line in open(os.path.join(d, "kt.log")):
            if line.startswith("{"):
                info = json.loads(line)
        print(case, info.get("mode_taken"), info.get("ms_median"), info.get("GiBps"))
        for k, v in sorted(per.items(), key=lambda kv: -sorted(kv[1])[len(kv[1]) // 2]):
            v.sort()
            print("   %-32s med %9.1f us  n=%d" % (k, v[len(v) // 2], len(v)))


if __name__ == "__main__":
    main(sys.argv[1])
