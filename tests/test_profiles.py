"""The evidence under profiles/: no tracked figure claims more than the HBM peak, and the PMC summariser
(tools/summarize_cases.py) pairs each timed dispatch's counters with that same dispatch's duration -- the
untimed setup never enters -- and refuses a rate above peak."""
import csv
import glob
import json
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

_PEAK_FRAC = re.compile(r'"(frac|frac_of_8TBps|frac_of_peak|value_frac_of_peak)":\s*(-?[0-9.]+(?:[eE][-+]?\d+)?)')


def test_no_tracked_profile_exceeds_peak():
    bad = []
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*.json*"))):
        with open(f) as fh:
            for m in _PEAK_FRAC.finditer(fh.read()):
                if float(m.group(2)) > 1.0:
                    bad.append((os.path.basename(f), m.group(1), m.group(2)))
    assert not bad, bad


def _write_case(d, reps, setup_bytes, call, fetch_of):
    """A fake pmc_cases/<case>/ directory: one setup sweep, then `reps` calls of `call` [(kernel, grid, ns)]."""
    disp = [("crc32_sweep_kernel", 4096, 900000)] + call * reps
    os.makedirs(os.path.join(d, "kt"))
    with open(os.path.join(d, "kt", "kt_kernel_trace.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Dispatch_Id", "Kernel_Name", "Start_Timestamp", "End_Timestamp", "Grid_Size_X"])
        w.writerow([0, "__amd_rocclr_fillBufferAligned", 0, 10, 256])
        for i, (k, g, ns) in enumerate(disp, 1):
            w.writerow([i, "void ambrycrc::%s<true>(ambrycrc::Args)" % k, 1000 * i, 1000 * i + ns, g])
    for p, counter in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        os.makedirs(os.path.join(d, p))
        with open(os.path.join(d, p, "pmc_counter_collection.csv"), "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Dispatch_Id", "Grid_Size", "Kernel_Name", "Counter_Name", "Counter_Value"])
            for i, (k, g, _) in enumerate(disp, 1):
                kib = setup_bytes / 1024 if i == 1 else fetch_of[k] / 1024
                w.writerow([i, g, "ambrycrc::%s(ambrycrc::Args)" % k, counter, kib / 2 if counter == "FETCH_SIZE" else 0])
    with open(os.path.join(d, "kt.log"), "w") as f:
        f.write(json.dumps({"reps": reps, "alg_bytes_per_launch": 2_000_000}) + "\n")


def test_summariser_pairs_timed_dispatches(tmp_path):
    from summarize_cases import summarize_case

    call = [("region_fused_kernel", 131072, 600_000), ("crc32_sweep_kernel", 4096, 4_700),
            ("crc32_plan_count_kernel", 32768, 4_000)]
    fetch_of = {"region_fused_kernel": 2_240_000, "crc32_sweep_kernel": 1_000, "crc32_plan_count_kernel": 500}
    d = str(tmp_path / "xform")
    _write_case(d, 4, 1.6e9, call, fetch_of)
    v = summarize_case(d, 5)
    assert v["call"]["launches"] == 3 and [r["kernel"] for r in v["roles"]] == [c[0] for c in call]
    sweep = v["kernels"]["crc32_sweep_kernel"]
    assert sweep["hbm_bytes"] == pytest.approx(1_000) and sweep["ns"] == 4_700  # the no-op's own bytes, not the setup's
    assert v["call"]["dominant_kernel"] == "region_fused_kernel"
    assert v["call"]["hbm_bytes"] == pytest.approx(2_241_500)
    assert v["call"]["traffic_over_alg"] == pytest.approx(2_241_500 / 2_000_000, rel=1e-3)
    assert "frac_of_8TBps" not in sweep  # no algorithmic rate for a kernel the case does not define it for


def test_summariser_refuses_a_rate_above_peak(tmp_path):
    from summarize_cases import summarize_case

    d = str(tmp_path / "fast")
    _write_case(d, 3, 1e9, [("crc32_sweep_kernel", 4096, 100)], {"crc32_sweep_kernel": 1000})
    with pytest.raises(SystemExit, match="peak"):
        summarize_case(d, 3)


def test_summariser_runs_on_a_tree(tmp_path):
    src = tmp_path / "cases"
    _write_case(str(src / "one"), 2, 1e9, [("region_runs_kernel", 8192, 300_000), ("region_msg_kernel", 1024, 100_000)],
                {"region_runs_kernel": 1_500_000, "region_msg_kernel": 400_000})
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "summarize_cases.py"), "--src", str(src),
                        "--tag", str(tmp_path / "t")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    out = json.load(open(str(tmp_path / "t") + "_small_cases.json"))
    assert out["cases"]["one"]["call"]["launches"] == 2
