#!/usr/bin/env python3
"""Condense tools/pmc_cases.sh outputs (gpurun_out/pmc_cases/<case>/) into profiles/<tag>_small_cases.json.

Dispatch pairing (round 6). Each run -- the kernel trace and each counter pass -- is
the same program, so its library dispatches come in the same order. The timed calls are the periodic
tail of that order: the last `reps` calls, each the same sequence of (kernel, grid) dispatches. The
summary finds that period P in every run, checks that all runs agree on it, and indexes each dispatch
of a call by its role j in 0..P-1. A role's duration (median over the reps, from the trace) and its
counters (mean over the reps, from each counter pass) come from the same dispatches of the same
calls -- the untimed setup (the region build's sweep, the check call) never enters, and a gated
no-op launch of the sweep kernel is charged its own few bytes, not a setup sweep's gigabytes.

Per case: every role (kernel, grid, median ns, HBM bytes = (2*FETCH_SIZE + WRITE_SIZE) KiB per the
guide's correction, SQ shares), per kernel the sum over its roles in one call, and the whole call
(every role: ns summed, HBM bytes summed). Achieved rates are computed only against algorithmic bytes
the case defines: for the call, and for the case's dominant kernel (most time per call) when the case
names its algorithmic bytes per launch. A row whose achieved rate exceeds the 8 TB/s peak is refused:
the summary stops with an error instead of writing it. The scatter16 / scatter4 / scatter8 cases
calibrate FETCH_SIZE for scattered small reads ("fetch_per_line" against the 128 B a line holds)."""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PEAK_GBPS = 8000.0


def short_name(full: str) -> str | None:
    """The library kernel's short name ('crc32_sweep_kernel'), None for a runtime or torch kernel."""
    if "ambrycrc::" not in full:
        return None
    s = full.split("ambrycrc::", 1)[1]
    return s.split("(", 1)[0].split("<", 1)[0]


def trace_dispatches(path):
    """[(dispatch id, kernel, grid, ns)] of the library's kernels, in dispatch order."""
    out = []
    for r in csv.DictReader(open(path)):
        k = short_name(r["Kernel_Name"])
        if k:
            grid = int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0)
            out.append((int(r["Dispatch_Id"]), k, grid, int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    out.sort()
    return out


def pmc_dispatches(path):
    """[(dispatch id, kernel, grid, {counter: value})] of the library's kernels, in dispatch order."""
    per = {}
    for r in csv.DictReader(open(path)):
        k = short_name(r["Kernel_Name"])
        if not k:
            continue
        d = int(r["Dispatch_Id"])
        if d not in per:
            per[d] = (k, int(r["Grid_Size"]), {})
        c = per[d][2]
        c[r["Counter_Name"]] = c.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return [(d, k, g, c) for d, (k, g, c) in sorted(per.items())]


def call_period(seq, reps):
    """The smallest P such that the last reps * P entries of seq (kernel, grid) are reps copies of one call."""
    for p in range(1, len(seq) // reps + 1):
        tail = seq[len(seq) - reps * p:]
        if all(tail[i] == tail[i % p] for i in range(len(tail))):
            return p
    raise SystemExit("no periodic call sequence in %d dispatches (reps %d)" % (len(seq), reps))


def roles(disp, reps, key=lambda x: (x[1], x[2])):
    seq = [key(x) for x in disp]
    p = call_period(seq, reps)
    tail = disp[len(disp) - reps * p:]
    return p, [[tail[r * p + j] for r in range(reps)] for j in range(p)]


def summarize_case(cdir, reps_default):
    info = {}
    try:
        with open(os.path.join(cdir, "kt.log")) as f:
            for line in f:
                if line.startswith("{"):
                    info = json.loads(line)
    except OSError:
        pass
    reps = int(info.get("reps", reps_default))
    kt = os.path.join(cdir, "kt", "kt_kernel_trace.csv")
    if not os.path.exists(kt):
        return None
    p, troles = roles(trace_dispatches(kt), reps)
    rows = [{"kernel": t[0][1], "grid": t[0][2], "median_ns": statistics.median(x[3] for x in t),
             "min_ns": min(x[3] for x in t)} for t in troles]
    for name in ("fetch", "write", "sq"):
        f = os.path.join(cdir, name, "pmc_counter_collection.csv")
        if not os.path.exists(f):
            continue
        pp, proles = roles(pmc_dispatches(f), reps)
        if pp != p or any((pr[0][1], pr[0][2]) != (r["kernel"], r["grid"]) for pr, r in zip(proles, rows)):
            raise SystemExit("%s: the %s pass's call (%d dispatches) differs from the trace's (%d)" % (cdir, name, pp, p))
        for pr, r in zip(proles, rows):
            cs = collections.defaultdict(list)
            for x in pr:
                for c, v in x[3].items():
                    cs[c].append(v)
            r.setdefault("counters", {}).update({c: sum(v) / len(v) for c, v in cs.items()})
    for r in rows:
        c = r.get("counters", {})
        if "FETCH_SIZE" in c:
            r["hbm_bytes"] = (2 * c["FETCH_SIZE"] + c.get("WRITE_SIZE", 0.0)) * 1024
        wc = c.get("SQ_WAVE_CYCLES")
        if wc:
            r["wait_any_frac"] = round(c.get("SQ_WAIT_ANY", 0) / wc, 4)
            r["active_inst_frac"] = round(c.get("SQ_ACTIVE_INST_ANY", 0) / wc, 4)
    kern = {}
    for r in rows:
        k = kern.setdefault(r["kernel"], {"launches_per_call": 0, "ns": 0, "hbm_bytes": 0.0, "grids": []})
        k["launches_per_call"] += 1
        k["ns"] += r["median_ns"]
        k["grids"].append(r["grid"])
        k["hbm_bytes"] = k["hbm_bytes"] + r["hbm_bytes"] if "hbm_bytes" in r and k["hbm_bytes"] is not None else None
    call = {"launches": p, "ns": sum(r["median_ns"] for r in rows)}
    if all("hbm_bytes" in r for r in rows):
        call["hbm_bytes"] = sum(r["hbm_bytes"] for r in rows)
    alg = info.get("alg_bytes_per_launch")
    dominant = max(kern, key=lambda k: kern[k]["ns"])
    call["dominant_kernel"] = dominant
    call["dominant_share_of_time"] = round(kern[dominant]["ns"] / call["ns"], 4)
    if alg:
        call["alg_bytes"] = alg
        for where, ns, hb in (("call", call["ns"], call.get("hbm_bytes")),
                              ("dominant", kern[dominant]["ns"], kern[dominant]["hbm_bytes"])):
            gbps = alg / ns
            if gbps > PEAK_GBPS:
                raise SystemExit("%s: %s achieves %.0f GB/s > the %.0f GB/s peak: refusing the row"
                                 % (cdir, where, gbps, PEAK_GBPS))
            d = call if where == "call" else kern[dominant]
            d["achieved_GBps"] = round(gbps, 1)
            d["frac_of_8TBps"] = round(gbps / PEAK_GBPS, 4)
            if hb:
                d["traffic_over_alg"] = round(hb / alg, 4)
    return {"info": info, "mode_taken": info.get("mode_taken"), "roles": rows, "kernels": kern, "call": call}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--src", default=os.path.join(ROOT, "gpurun_out", "pmc_cases"))
    ap.add_argument("--tag", required=True)
    ap.add_argument("--reps", type=int, default=5, help="calls per case when kt.log does not say")
    ap.add_argument("--supersedes", default="", help="an earlier summary this one replaces, and why")
    ap.add_argument("--cases", default="", help="comma-separated case directories to summarise (default: all)")
    args = ap.parse_args()
    only = set(filter(None, args.cases.split(",")))
    res = {"what": __doc__.split("\n\n")[0], "pairing": __doc__.split("\n\n")[1], "cases": {}}
    if args.supersedes:
        res["supersedes"] = args.supersedes
    for cdir in sorted(glob.glob(os.path.join(args.src, "*", ""))):
        case = os.path.basename(os.path.dirname(cdir))
        if only and case not in only:
            continue
        v = summarize_case(cdir, args.reps)
        if v:
            res["cases"][case] = v
    # FETCH_SIZE calibration for scattered reads (MI355X_MICROARCH.md: the x2 correction is for wide streams)
    cal = []
    for c, v in res["cases"].items():
        lines = v["info"].get("lines")
        rb = [r for r in v["roles"] if r["kernel"] == "readbw_scatter_kernel" and "FETCH_SIZE" in r.get("counters", {})]
        if c.startswith("scatter") and lines and rb:
            v["call"]["fetch_per_line"] = round(rb[0]["counters"]["FETCH_SIZE"] * 1024 / lines, 2)
            cal.append(v["call"]["fetch_per_line"])
    if cal:
        res["scatter_fetch_factor"] = round(128.0 / (sum(cal) / len(cal)), 3)
    out = os.path.join(ROOT, "profiles", f"{args.tag}_small_cases.json")
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    for case, v in res["cases"].items():
        c = v["call"]
        print(case, v.get("mode_taken"), "launches", c["launches"], "us %.1f" % (c["ns"] / 1e3),
              "frac", c.get("frac_of_8TBps"), "traffic", c.get("traffic_over_alg"), "dominant", c["dominant_kernel"],
              {k: (round(x["ns"] / 1e3, 1), x.get("traffic_over_alg")) for k, x in v["kernels"].items()
               if k == c["dominant_kernel"]})
    return 0


if __name__ == "__main__":
    sys.exit(main())
