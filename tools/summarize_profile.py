#!/usr/bin/env python3
"""Condense rocprofv3 outputs (gpurun_out/prof_*) into committed profiles/ files.

  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (as emitted)
  profiles/<tag>_pmc_summary.json   per-dispatch averages of every PMC counter for the sweep kernel
  bench_data/pmc_traffic.json       HBM bytes per sweep-kernel launch per config, read by bench.py as
                                    roofline.traffic (bench_data/ travels to the GPU box; profiles/ does not)

Traffic correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE and WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE reads exactly half the bytes of a wide coalesced stream, so
hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024. Each counter comes from its own
--pmc pass.
"""
from __future__ import annotations

import argparse
import collections
import csv
import json
import os
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def pmc_avgs(path, kernel_substr, size_counter):
    """Per-counter averages over the kernel's C3-sized dispatches only.

    bench.py also launches the sweep kernel for its clock pre-warm (same size), the CPU-baseline
    parity check (64 chunks) and the host-path slabs; a dispatch counts when its size_counter
    value is at least half the largest one seen."""
    rows = [r for r in csv.DictReader(open(path)) if kernel_substr in r["Kernel_Name"]]
    per = collections.defaultdict(dict)
    for r in rows:
        per[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
    top = max((d.get(size_counter, 0.0) for d in per.values()), default=0.0)
    keep = [d for d in per.values() if d.get(size_counter, 0.0) >= 0.5 * top]
    agg = collections.defaultdict(list)
    for d in keep:
        for k, v in d.items():
            agg[k].append(v)
    return {k: sum(v) / len(v) for k, v in agg.items()}, {k: len(v) for k, v in agg.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--src", default=os.path.join(ROOT, "gpurun_out"))
    ap.add_argument("--tag", required=True)
    ap.add_argument("--kernel", default="crc32_sweep_kernel")
    ap.add_argument("--config", default="c3", help="bench.py config the PMC passes ran (key in pmc_traffic.json)")
    ap.add_argument("--alg-bytes", type=int, default=None,
                    help="algorithmic bytes per launch (default: from --config: chunk bytes + 4 B per chunk)")
    args = ap.parse_args()
    if args.alg_bytes is None:
        n, chunk = {"c3": (8192, 4 << 20), "c2": (65536, 64 << 10), "c5": (65536, 4 << 20)}[args.config]
        args.alg_bytes = n * chunk + 4 * n
    out = os.path.join(ROOT, "profiles")
    os.makedirs(out, exist_ok=True)
    shutil.copy(os.path.join(args.src, "prof_kt", "kt_kernel_stats.csv"),
                os.path.join(out, f"{args.tag}_kernel_stats.csv"))
    summary = {"kernel": args.kernel, "passes": {}}
    counters = {}
    for name, size_counter in (("prof_fetch", "FETCH_SIZE"), ("prof_write", "WRITE_SIZE"),
                               ("prof_sq", "GRBM_GUI_ACTIVE")):
        p = os.path.join(args.src, name, "pmc_counter_collection.csv")
        if os.path.exists(p):
            avg, cnt = pmc_avgs(p, args.kernel, size_counter)
            summary["passes"][name] = {"avg": avg, "dispatches": cnt}
            counters.update(avg)
    with open(os.path.join(args.src, "prof_kt", "kt_kernel_stats.csv")) as f:
        for r in csv.DictReader(f):
            if args.kernel in r["Name"]:
                summary["kernel_trace_all_dispatches"] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                                                          "min_ns": float(r["MinNs"]), "max_ns": float(r["MaxNs"])}
    # C3-sized dispatches (>= half the longest): pre-warm + warmup + timed steps
    trace = os.path.join(args.src, "prof_kt", "kt_kernel_trace.csv")
    if os.path.exists(trace):
        d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(open(trace))
             if args.kernel in r["Kernel_Name"]]
        big = sorted(x for x in d if x >= 0.5 * max(d))
        summary["kernel_trace"] = {"calls": len(big), "avg_ns": sum(big) / len(big), "median_ns": big[len(big) // 2],
                                   "min_ns": big[0], "max_ns": big[-1],
                                   "selection": "sweep dispatches >= 0.5 x the longest (C3-sized)"}

    if "FETCH_SIZE" in counters:
        hbm = (2 * counters["FETCH_SIZE"] + counters.get("WRITE_SIZE", 0.0)) * 1024
        summary["hbm_bytes_per_launch"] = hbm
        summary["algorithmic_bytes_per_launch"] = args.alg_bytes
        summary["traffic_over_algorithmic"] = hbm / args.alg_bytes
        tf = os.path.join(ROOT, "bench_data", "pmc_traffic.json")
        os.makedirs(os.path.dirname(tf), exist_ok=True)
        table = json.load(open(tf)) if os.path.exists(tf) else {}
        table[args.config] = {"hbm_bytes_per_launch": round(hbm), "algorithmic_bytes_per_launch": args.alg_bytes,
                              "traffic_over_algorithmic": round(hbm / args.alg_bytes, 6),
                              "source": f"profiles/{args.tag}_pmc_summary.json: (2*FETCH_SIZE + WRITE_SIZE) KiB, "
                                        f"separate rocprofv3 --pmc passes of bench.py --config {args.config}",
                              "kernel": args.kernel}
        with open(tf, "w") as f:
            json.dump(table, f, indent=1)
    if "GRBM_GUI_ACTIVE" in counters and "kernel_trace" in summary:
        summary["effective_clock_ghz_est"] = counters["GRBM_GUI_ACTIVE"] / 8 / (summary["kernel_trace"]["avg_ns"])
    with open(os.path.join(out, f"{args.tag}_pmc_summary.json"), "w") as f:
        json.dump(summary, f, indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
