"""Summarize tools/pmc_ab.sh: per library build, case and CRC kernel, each SQ counter averaged over
the kernel's dispatches (the first, warm-up, dispatch of each run dropped), and the ratios that
name a bound: waits and issue as fractions of wave cycles, LDS-array busy and bank-conflict
cycles, instructions per wave."""
import collections
import csv
import glob
import json
import os
import re
import sys

# kernels summarized (regex on the short name; KMATCH=region_ for the message verify kernels)
KMATCH = os.environ.get("KMATCH", "sweep_kernel|group_kernel")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "pmc_ab")
res = {}
for f in sorted(glob.glob(os.path.join(src, "*", "*", "p*.csv"))):
    tag, case = f.split(os.sep)[-3:-1]
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    rows = list(csv.DictReader(open(f)))
    for r in rows:
        k = r["Kernel_Name"].split("(")[0].split("<")[0].split("::")[-1]
        if not re.search(KMATCH, k):
            continue
        per[(k, r["Dispatch_Id"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    seen = collections.Counter()
    for (k, d), cs in sorted(per.items(), key=lambda x: int(x[0][1])):
        seen[k] += 1
        if seen[k] == 1:
            continue  # warm-up dispatch
        for c, v in cs.items():
            agg[k][c].append(sum(v))
    for k, cs in agg.items():
        dst = res.setdefault(tag, {}).setdefault(case, {}).setdefault(k, {})
        for c, v in cs.items():
            dst[c] = sum(v) / len(v)
for tag, cases in res.items():
    for case, ks in cases.items():
        for k, c in ks.items():
            wc = c.get("SQ_WAVE_CYCLES") or 1
            waves = c.get("SQ_WAVES") or 1
            line = {"valu/wave": c.get("SQ_INSTS_VALU", 0) / waves, "lds/wave": c.get("SQ_INSTS_LDS", 0) / waves,
                    "salu/wave": c.get("SQ_INSTS_SALU", 0) / waves,
                    "wait_any": c.get("SQ_WAIT_ANY", 0) / wc, "active_inst": c.get("SQ_ACTIVE_INST_ANY", 0) / wc,
                    "wait_inst_lds": c.get("SQ_WAIT_INST_LDS", 0) / wc, "wait_inst_any": c.get("SQ_WAIT_INST_ANY", 0) / wc,
                    "lds_idx_active": c.get("SQ_LDS_IDX_ACTIVE"), "lds_bank_conflict": c.get("SQ_LDS_BANK_CONFLICT"),
                    "busy_cycles": c.get("SQ_BUSY_CYCLES"), "waves": c.get("SQ_WAVES")}
            if os.environ.get("RAW"):
                print(f"{tag:8s} {case:9s} {k:22s} RAW " + " ".join(f"{n}={v:.4g}" for n, v in sorted(c.items())))
            print(f"{tag:8s} {case:9s} {k:22s} " + " ".join(
                f"{n}={v:.4g}" if isinstance(v, float) else f"{n}={v}" for n, v in line.items()))
json.dump(res, open(os.path.join(src, "summary.json"), "w"), indent=1)
