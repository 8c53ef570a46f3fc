#!/usr/bin/env python3
"""Condense tools/pmc_cases.sh outputs (gpurun_out/pmc_cases/<case>/) into profiles/<tag>_small_cases.json:
per case and kernel, the kernel-trace duration and per-dispatch PMC averages, plus derived
figures: HBM bytes (2*FETCH_SIZE + WRITE_SIZE, KiB; MI355X_MICROARCH.md §HBM) against the
algorithmic bytes, achieved GB/s, VALU and LDS instructions per KiB of chunk data, the share
of wave-cycles parked (SQ_WAIT_ANY), stalled on LDS issue (SQ_WAIT_INST_LDS) and issuing
(SQ_ACTIVE_INST_ANY), and the effective clock (GRBM_GUI_ACTIVE / 8 / duration).

Per case also the whole call ("call": every kernel of one call, median durations summed, bytes
summed) -- the message verify's and the transform's figures are per call -- and the mode the call
took as the library reported it (ambrycrc_last_message_mode, "mode_taken"). The scatter16 / scatter4
/ scatter8 cases calibrate FETCH_SIZE for scattered small reads: measured FETCH bytes per read line
("fetch_per_line") against the 128 B each line holds."""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = ("crc32_sweep_kernel", "crc32_plan_scan_kernel", "crc32_plan_count_kernel", "msg_parse_kernel",
           "msg_reduce_kernel", "region_runs_kernel", "region_msg_kernel", "region_fused_kernel",
           "region_tail_kernel", "transform_place_kernel", "transform_jobs_kernel", "transform_finish_kernel",
           "transform_merge_kernel", "transform_desc_kernel", "props_fix_kernel", "put_layout_kernel",
           "put_seal_kernel", "gather_copy_kernel", "readbw_scatter_kernel")


def kname(full):
    for k in KERNELS:
        if k in full:
            return k
    return None


def trace(path):
    per = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        k = kname(r["Kernel_Name"])
        if k:
            per[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    out = {}
    for k, d in per.items():
        d.sort()
        # the repeated launches dominate; drop a first cold one if it is an outlier
        med = d[len(d) // 2]
        out[k] = {"calls": len(d), "median_ns": med, "avg_ns": sum(d) / len(d), "min_ns": d[0]}
    return out


def pmc(path, size_counter):
    per = collections.defaultdict(lambda: collections.defaultdict(dict))
    for r in csv.DictReader(open(path)):
        k = kname(r["Kernel_Name"])
        if k:
            per[k][r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
    out = {}
    for k, disp in per.items():
        vals = list(disp.values())
        key = size_counter if any(size_counter in v for v in vals) else None
        if key:
            top = max(v.get(key, 0.0) for v in vals)
            vals = [v for v in vals if v.get(key, 0.0) >= 0.5 * top]
        agg = collections.defaultdict(list)
        for v in vals:
            for c, x in v.items():
                agg[c].append(x)
        out[k] = {c: sum(x) / len(x) for c, x in agg.items()}
        out[k]["_dispatches"] = len(vals)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--src", default=os.path.join(ROOT, "gpurun_out", "pmc_cases"))
    ap.add_argument("--tag", required=True)
    ap.add_argument("--supersedes", default="", help="an earlier summary this one replaces, and why")
    args = ap.parse_args()
    res = {"what": __doc__.split("\n\n")[0], "cases": {}}
    if args.supersedes:
        res["supersedes"] = args.supersedes
    for cdir in sorted(glob.glob(os.path.join(args.src, "*", ""))):
        case = os.path.basename(os.path.dirname(cdir))
        info = {}
        try:
            with open(os.path.join(cdir, "kt.log")) as f:
                for line in f:
                    if line.startswith("{"):
                        info = json.loads(line)
        except OSError:
            pass
        kt = os.path.join(cdir, "kt", "kt_kernel_trace.csv")
        if not os.path.exists(kt):
            continue
        t = trace(kt)
        counters = collections.defaultdict(dict)
        for p, sc in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE"), ("sq", "SQ_WAVE_CYCLES")):
            f = os.path.join(cdir, p, "pmc_counter_collection.csv")
            if os.path.exists(f):
                for k, v in pmc(f, sc).items():
                    counters[k].update({c: x for c, x in v.items() if c != "_dispatches"})
        kern = {}
        alg = info.get("alg_bytes_per_launch")
        data_kib = (info["chunks"] * info["chunk_bytes"] / 1024) if "chunks" in info else (
            info.get("region_bytes", 0) / 1024)
        for k, tv in t.items():
            c = counters.get(k, {})
            row = {"trace": tv, "counters": c}
            ns = tv["median_ns"]
            if "FETCH_SIZE" in c:
                row["hbm_bytes"] = (2 * c["FETCH_SIZE"] + c.get("WRITE_SIZE", 0.0)) * 1024
            if k == "crc32_sweep_kernel" and alg:
                row["alg_bytes"] = alg
                row["achieved_GBps"] = round(alg / ns, 1)
                row["frac_of_8TBps"] = round(alg / ns / 8000, 4)
                if "hbm_bytes" in row:
                    row["traffic_over_alg"] = round(row["hbm_bytes"] / alg, 4)
            if "SQ_WAVE_CYCLES" in c and c["SQ_WAVE_CYCLES"]:
                wc = c["SQ_WAVE_CYCLES"]
                row["wait_any_frac"] = round(c.get("SQ_WAIT_ANY", 0) / wc, 4)
                row["wait_inst_lds_frac"] = round(c.get("SQ_WAIT_INST_LDS", 0) / wc, 4)
                row["active_inst_frac"] = round(c.get("SQ_ACTIVE_INST_ANY", 0) / wc, 4)
            if k == "crc32_sweep_kernel" and data_kib:
                for cn, nm in (("SQ_INSTS_VALU", "valu_per_kib"), ("SQ_INSTS_LDS", "lds_per_kib"),
                               ("SQ_INSTS_VMEM_RD", "vmem_rd_per_kib")):
                    if cn in c:
                        row[nm] = round(c[cn] / data_kib, 2)
            # no clock estimate: GRBM_GUI_ACTIVE counts over the counter window, which for dispatches
            # shorter than it (plan, reduce, single-call sweeps) exceeds the kernel time (round-2 review
            # found 4.0-7.6 "GHz" that way); GRBM_GUI_ACTIVE is kept raw only
            if "GRBM_GUI_ACTIVE" in c:
                row["grbm_gui_active"] = c["GRBM_GUI_ACTIVE"]
            kern[k] = row
        # the whole call: the calls are those of the kernel with the most total time; a kernel
        # launched at least half as often belongs to every call, `per_call` times (a transform runs
        # the plan kernels twice per call), medians summed
        heavy = max(t.values(), key=lambda tv: tv["median_ns"] * tv["calls"], default=None)
        reps = heavy["calls"] if heavy else 0
        per_call = {k: max(1, round(tv["calls"] / reps)) for k, tv in t.items() if reps and tv["calls"] >= max(1, reps // 2)}
        call = {"kernels": sorted(per_call), "launches_per_call": per_call,
                "ns": sum(t[k]["median_ns"] * n for k, n in per_call.items())}
        hb = [(kern[k].get("hbm_bytes"), n) for k, n in per_call.items()]
        if hb and all(x is not None for x, _ in hb):
            call["hbm_bytes"] = sum(x * n for x, n in hb)
        if alg and call["ns"]:
            call["alg_bytes"] = alg
            call["achieved_GBps"] = round(alg / call["ns"], 1)
            call["frac_of_8TBps"] = round(alg / call["ns"] / 8000, 4)
            if "hbm_bytes" in call:
                call["traffic_over_alg"] = round(call["hbm_bytes"] / alg, 4)
        if case.startswith("scatter") and "readbw_scatter_kernel" in counters:
            c = counters["readbw_scatter_kernel"]
            if "FETCH_SIZE" in c and info.get("lines"):
                call["fetch_per_line"] = round(c["FETCH_SIZE"] * 1024 / info["lines"], 2)
                call["fetch_over_bytes"] = round(c["FETCH_SIZE"] * 1024 / (info["lines"] * 128), 4)
        res["cases"][case] = {"info": info, "mode_taken": info.get("mode_taken"), "kernels": kern, "call": call}
    # FETCH_SIZE calibration for scattered reads (MI355X_MICROARCH.md: the x2 correction is for
    # wide streams): the scatter cases read a known number of 128-B lines; bytes per counted KiB
    # = 128 / fetch_per_line. Applied to the per-message kernels, whose reads are scattered lines.
    cal = [v["call"]["fetch_per_line"] for c, v in res["cases"].items()
           if c.startswith("scatter") and "fetch_per_line" in v["call"]]
    if cal:
        f = 128.0 / (sum(cal) / len(cal))
        res["scatter_fetch_factor"] = round(f, 3)
        for v in res["cases"].values():
            for k in ("region_msg_kernel", "region_tail_kernel", "msg_parse_kernel"):
                row = v["kernels"].get(k)
                if row and "FETCH_SIZE" in row["counters"]:
                    row["hbm_bytes_scatter_calibrated"] = (f * row["counters"]["FETCH_SIZE"] +
                                                           row["counters"].get("WRITE_SIZE", 0.0)) * 1024
    out = os.path.join(ROOT, "profiles", f"{args.tag}_small_cases.json")
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    for case, v in res["cases"].items():
        print(case, v.get("mode_taken"), v["call"])


if __name__ == "__main__":
    main()
