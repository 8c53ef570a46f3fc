#!/usr/bin/env python3
"""bench.py -- device-resident CRC-32 over 4 MiB blob chunks (BASELINE.json metric, config C3).

One step = one pass of the hot path (ambrycrc_batch_dev: plan + sweep kernels)
over one batch of 8,192 x 4 MiB chunks (32 GiB) resident in HBM on every rank.
N>1: one process per GPU (torchrun), each rank owns its own 8,192-chunk shard
(weak scaling; C5 = 524,288 chunks = 8 such steps on 8 GPUs) and the 4-byte
CRCs are all-gathered over RCCL once per step.

Prints ONE JSON line (rank 0). Besides the driver contract it carries:
  roofline      sweep-kernel algorithmic bytes / its HIP-event-timed duration vs 8 TB/s
  cpu_baseline  the oracle's restatement of Crc32.java (kind "port") on host cores, bounded sample
  host_path     pinned-host -> HBM -> CRC rate (PCIe-inclusive; never `value`)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

METRIC = "GiB/s device-resident CRC32 over 4 MiB blob chunks; % of HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)

CONFIGS = {
    # name: (chunks per GPU, chunk bytes, description)
    "c3": (8192, 4 << 20, "C3: 8,192 x 4 MiB large-blob router chunks per GPU"),
    "c2": (65536, 64 << 10, "C2: 65,536 x 64 KiB small-object chunks per GPU"),
    # 524,288 x 4 MiB over 8 GPUs = 65,536 x 4 MiB = 256 GiB resident per
    # GPU (of 268 GiB HBM). Every chunk is distinct: a reused buffer let waves that run at
    # the same time read the same bytes, and the caches then served ~4 % of the reads.
    "c5": (65536, 4 << 20, "C5: 65,536 x 4 MiB chunks per GPU (256 GiB resident)"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS) + ["c4"])
    ap.add_argument("--variant", type=int, default=None)
    ap.add_argument("--grid", type=int, default=None, help="sweep-kernel workgroups (default: one per CU)")
    ap.add_argument("--window", type=int, default=None,
                    help="sweep rounds of at most this many bytes (default: the library's 32 GiB; 0 = one round)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-host-path", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--prewarm-s", type=float, default=0.3, help="untimed clock-ramp run before warmup")
    ap.add_argument("--quiet", action="store_true", help="no progress lines on stderr")
    ap.add_argument("--force-dist", action="store_true",
                    help="init the RCCL process group and all-gather even at WORLD_SIZE=1 (exercises the N>1 path)")
    return ap.parse_args()


def log(args, *msg):
    if not args.quiet:
        print("[bench]", *msg, file=sys.stderr, flush=True)


def build_workload(torch, dev, args, rank):
    from ambry_amd import device as D

    if args.config == "c4":
        from datagen import zipf_sizes

        sizes = zipf_sizes(32768)
        off = [0]
        for s in sizes[:-1]:
            off.append(off[-1] + ((int(s) + 15) // 16) * 16)
        total = off[-1] + int(sizes[-1])
        import numpy as np

        off_t = torch.tensor(np.asarray(off, dtype=np.int64), device=dev)
        len_t = torch.tensor(sizes.astype(np.int64), device=dev)
        desc = "C4: 32,768 Zipf(1.2) chunks 4 KiB-4 MiB (verify-on-read sizes)"
        n = len(sizes)
        chunk = None
    else:
        n, chunk, desc = CONFIGS[args.config]
        total = n * chunk
        off_t = torch.arange(n, dtype=torch.int64, device=dev) * chunk
        len_t = torch.full((n,), chunk, dtype=torch.int64, device=dev)
    buf = torch.empty(total, dtype=torch.uint8, device=dev)
    D.fill_random(buf, 0xA3B1C2D3 ^ (rank * 0x9E3779B97F4A7C15 & (2**64 - 1)), 0)
    torch.cuda.synchronize()
    return buf, off_t, len_t, n, total, chunk, desc


def cpu_baseline(buf, off_t, len_t, n, args):
    """Oracle (C restatement of Crc32.java slice-by-8) on host cores over a bounded sample."""
    import numpy as np

    from conftest import ORACLE_SO, Oracle

    if not os.path.exists(ORACLE_SO):
        return None
    orc = Oracle()
    sample_chunks = min(n, 64)
    off = off_t[:sample_chunks].cpu().numpy()
    ln = len_t[:sample_chunks].cpu().numpy()
    lo, hi = int(off[0]), int(off[-1] + ln[-1])
    host = buf[lo:hi].cpu().numpy()
    off = off - lo
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    res = {}
    for zl in (False, True):
        for th in (1, threads):
            t0 = time.perf_counter()
            passes = 0
            while True:
                out = orc.batch(host, off, ln, threads=th, zlib=zl)
                passes += 1
                el = time.perf_counter() - t0
                if el >= args.cpu_seconds / 4 or passes >= 1000:
                    break
            res[(zl, th)] = (passes * int(ln.sum()) / el / 2**30, passes, out)
    assert np.array_equal(res[(True, threads)][2], res[(False, threads)][2]), "zlib vs restatement"
    gibs, passes, out = res[(False, threads)]
    clmul = host_clmul_rate(host, off, ln, out, threads, args.cpu_seconds / 4)
    cpu_model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu_model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {
        "value": round(gibs, 3), "unit": "GiB/s", "cores": threads, "kind": "port",
        "cpu_model": cpu_model, "nproc": os.cpu_count(), "affinity_cpus": len(os.sched_getaffinity(0)),
        "sample": f"{sample_chunks} chunks x {int(ln[0]) if len(set(ln.tolist())) == 1 else 'mixed'} B "
                  f"(first chunks of the same workload, D2H-copied) x {passes} passes; oracle/crc32_ref.c "
                  f"slice-by-8 restating Crc32.java:55-98, {threads} pthreads",
        "single_thread_gibs": round(res[(False, 1)][0], 3),
        "zlib": {"gibs": round(res[(True, threads)][0], 3), "cores": threads,
                 "single_thread_gibs": round(res[(True, 1)][0], 3),
                 "what": "system zlib 1.2.11 crc32_z (the function java.util.zip.CRC32 wraps), same sample"},
        "host_clmul": clmul,
        "_out": out,
    }


def host_clmul_rate(host, off, ln, expect, threads, seconds):
    """The library's own CPU path (ambrycrc_update: carry-less-multiply fold, the class of
    HotSpot's CRC32 intrinsic) on the same sample, 1 thread and `threads` threads (ctypes
    releases the GIL for the call). Not the baseline: a check on what the JVM could do."""
    import ctypes
    import threading

    import numpy as np

    import ambry_amd

    lib = ambry_amd.lib()
    base = host.ctypes.data
    offs, lens = [int(o) for o in off], [int(x) for x in ln]
    got = np.array([lib.ambrycrc_update(0, base + o, n) for o, n in zip(offs, lens)], dtype=np.uint32)
    ok = bool(np.array_equal(got, np.asarray(expect, dtype=np.uint32)))

    def run(th):
        passes = [0] * th
        stop = time.perf_counter() + seconds

        def worker(t):
            idx = list(range(t, len(offs), th))
            while True:
                for i in idx:
                    lib.ambrycrc_update(0, ctypes.c_void_p(base + offs[i]), lens[i])
                passes[t] += 1
                if time.perf_counter() >= stop:
                    break

        t0 = time.perf_counter()
        ws = [threading.Thread(target=worker, args=(t,)) for t in range(th)]
        for w in ws:
            w.start()
        for w in ws:
            w.join()
        el = time.perf_counter() - t0
        return sum(passes[t] * sum(lens[t::th]) for t in range(th)) / el / 2**30

    return {"impl": lib.ambrycrc_host_impl().decode(), "single_thread_gibs": round(run(1), 3),
            "gibs": round(run(threads), 3), "cores": threads, "parity_vs_port": ok,
            "what": "libambrycrc ambrycrc_update on the host (CLMUL fold; HotSpot-intrinsic class), same sample"}


def measure_read_roof(torch, D, buf, total, device):
    """Read-only probe (ambrycrc_debug_readbw_dev variant 1: the sweep kernel's grid and access
    shape, nontemporal loads, no CRC arithmetic) over the same HBM buffer: best of 5 launches, GB/s."""
    from ambry_amd._lib import check, lib

    nbytes = total & ~((256 << 10) - 1)
    scratch = torch.empty(D.grid_size(device) * 1024, dtype=torch.int32, device=buf.device)
    best = None
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        check(lib().ambrycrc_debug_readbw_dev(buf.data_ptr(), nbytes, scratch.data_ptr(), 1,
                                              torch.cuda.current_stream().cuda_stream), "readbw")
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        best = ms if best is None else min(best, ms)
    return round(nbytes / (best / 1e3) / 1e9, 1)


def host_path_rate(torch, args):
    """Host buffers -> PCIe -> HBM -> CRC -> host (ambrycrc_batch_host); DESIGN.md only, never `value`.

    After one untimed full pass (first touch of the pinned pages by the DMA engine), the best
    of 3 synchronous calls for pinned and for pageable sources, beside the PCIe H2D roof: one
    2 GiB pinned->HBM hipMemcpyAsync (torch copy_) timed the same way.
    """
    from ambry_amd import device as D

    nchunks, chunk = 512, 4 << 20  # 2 GiB
    total = nchunks * chunk
    host = torch.empty(total, dtype=torch.uint8).pin_memory()
    host.view(torch.int64).random_()
    pageable = host.numpy().copy()

    def best_of(fn, reps=3):
        fn()
        best = None
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            best = el if best is None else min(best, el)
        return total / best / 2**30

    dev = torch.empty(total, dtype=torch.uint8, device="cuda")
    roof = best_of(lambda: dev.copy_(host, non_blocking=True))
    del dev
    res = {}
    for name, base in (("pinned", host.data_ptr()), ("pageable", pageable.ctypes.data)):
        chunks = [(base + i * chunk, chunk) for i in range(nchunks)]
        res[name] = best_of(lambda: D.crc32_batch_host(chunks, device=0, pinned=name == "pinned"))
    return {"value": round(res["pinned"], 2), "unit": "GiB/s",
            "pageable": round(res["pageable"], 2),
            "h2d_copy_roof": round(roof, 2),
            "frac_of_h2d_roof": round(res["pinned"] / roof, 4),
            "sample": f"{nchunks} x 4 MiB host chunks (2 GiB), synchronous ambrycrc_batch_host (H2D + kernels + "
                      "D2H of CRCs), best of 3 after one untimed pass; pinned = hipHostMalloc'd source, "
                      "pageable = malloc'd source staged by the library's copy threads"}


def main():
    args = parse()
    # stdout carries exactly one JSON line (rank 0). Native libraries print to fd 1 on their
    # own (RCCL's version banner at communicator init), so fd 1 is pointed at stderr for
    # the run and the result is written to a saved copy of the original stdout.
    sys.stdout.flush()
    result_fd = os.dup(1)
    os.dup2(2, 1)
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(args, f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    dist = None
    use_dist = world > 1 or args.force_dist
    if use_dist:
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    from ambry_amd import device as D

    D.init(dev.index)
    if args.variant is not None:
        D.set_variant(dev.index, args.variant)
    if args.grid is not None:
        D.set_grid(dev.index, args.grid)
    if args.window is not None:
        D.set_window(dev.index, args.window)

    log(args, f"rank {rank}/{world}: building workload {args.config}")
    buf, off_t, len_t, n, total, chunk, desc = build_workload(torch, dev, args, rank)
    gathered = torch.empty(world * n, dtype=torch.int32, device=dev) if use_dist else None

    verify = None
    if args.config == "c4":
        # C4 is the verify-on-read path: expected CRCs from a clean pass, then single-bit flips
        # in 1 % of the chunks (seeded); each step recomputes and compares (ambrycrc_verify_dev).
        import numpy as np

        expected = D.crc32_batch(buf, off_t, len_t).clone()
        rng = np.random.default_rng(20261016 + rank)
        bad = np.sort(rng.choice(n, size=n // 100, replace=False))
        lens_h = len_t.cpu().numpy()
        offs_h = off_t.cpu().numpy()
        pos = offs_h[bad] + (rng.random(len(bad)) * lens_h[bad]).astype(np.int64)
        bits = torch.tensor(1 << rng.integers(0, 8, size=len(bad)), dtype=torch.uint8, device=dev)
        pos_t = torch.tensor(pos, dtype=torch.int64, device=dev)
        buf[pos_t] ^= bits
        torch.cuda.synchronize()
        verify = {"expected": expected, "bad": bad, "out": torch.empty(n, dtype=torch.int32, device=dev),
                  "mism": torch.empty(n, dtype=torch.uint8, device=dev)}

    def step():
        if verify is not None:
            out, _, _ = D.crc32_verify(buf, off_t, len_t, verify["expected"], out=verify["out"],
                                       mismatch=verify["mism"], count=False)
        else:
            out = D.crc32_batch(buf, off_t, len_t)
        if use_dist:
            dist.all_gather_into_tensor(gathered, out)
        return out

    # Clock ramp: the MI355X takes tens of ms of sustained load to reach its steady clocks
    # (a 0.7 ms C2 step measured 13 % slower over the first 20 steps than over 100). Run the
    # step untimed for >= --prewarm-s before the contract's W warmup steps.
    t_pre = time.perf_counter()
    while True:
        out = step()
        torch.cuda.synchronize()
        if time.perf_counter() - t_pre >= args.prewarm_s:
            break
    for _ in range(args.warmup):
        out = step()
    torch.cuda.synchronize()
    D.timing_collect(dev.index)  # drop warmup events
    D.timing_enable(dev.index, True)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    ev0.record()
    for i in range(args.steps):
        out = step()
    ev1.record()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    wall = time.perf_counter() - t0
    D.timing_enable(dev.index, False)
    kern_each = D.timing_collect_each(dev.index)
    kern_ms, launches = sum(kern_each), len(kern_each)
    kern_median_ms = float(sorted(kern_each)[len(kern_each) // 2]) if kern_each else None
    ev_ms = ev0.elapsed_time(ev1)

    elapsed = wall
    if dist:
        t = torch.tensor([wall], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    allgather_ok = None
    if use_dist:  # this rank's CRCs must sit at its slot of the gathered vector
        allgather_ok = bool(torch.equal(gathered[rank * n:(rank + 1) * n], out))
        flag = torch.tensor([1 if allgather_ok else 0], dtype=torch.int32, device=dev)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        allgather_ok = bool(flag.item())
    read_roof = measure_read_roof(torch, D, buf, buf.numel(), dev.index) if args.config != "c4" else None
    crcs = out.cpu().numpy().view("uint32")
    verify_ok = None
    if verify is not None:  # the flags must name exactly the flipped chunks
        flagged = np.nonzero(verify["mism"].cpu().numpy())[0]
        _, _, cnt = D.crc32_verify(buf, off_t, len_t, verify["expected"])  # the counter form, once, untimed
        verify_ok = bool(np.array_equal(flagged, verify["bad"]) and int(cnt.item()) == len(verify["bad"]))
    step_bytes = total  # per rank
    value = world * step_bytes * args.steps / elapsed / 2**30
    kern_avg_s = kern_ms / max(1, launches) / 1e3
    alg_bytes = total + 4 * n  # chunk bytes read + 4 B CRC written per chunk (offset/len arrays excluded)
    achieved = alg_bytes / kern_avg_s / 1e9 if kern_avg_s > 0 else None

    result = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (device splitmix64 bytes; no dataset)",
        "config": {"workload": desc, "chunks_per_gpu": n, "chunk_bytes": chunk, "bytes_per_gpu_step": total,
                   "parallelism": f"shard{world}" + ("+rccl_allgather" if use_dist else ""),
                   "kernel_variant": D.get_variant(dev.index),
                   "grid_workgroups": D.grid_size(dev.index),
                   "sweep_window_bytes": args.window if args.window is not None else 32 << 30},
        "roofline": {
            "bound": "hbm",
            "kernel": "crc32_sweep_kernel",
            "achieved": round(achieved, 1) if achieved else None,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
            "traffic": None,
            "kernel_avg_ms": round(kern_avg_s * 1e3, 4),
            "kernel_median_ms": round(kern_median_ms, 4) if kern_median_ms else None,
            "algorithmic_bytes_per_launch": alg_bytes,
            "value_frac_of_peak": round(value * 2**30 / 1e9 / world / HBM_PEAK_GBS, 4),
            "measured_read_roof": read_roof,
            "frac_of_measured_read_roof": (round(achieved / read_roof, 4)
                                           if achieved and read_roof else None),
        },
        "timing": {"wall_s": round(elapsed, 4), "stream_event_ms": round(ev_ms, 3), "kernel_launches": launches},
        "allgather_ok": allgather_ok,
        "verify": (None if verify is None else
                   {"flipped_chunks": int(len(verify["bad"])), "flags_exact": verify_ok,
                    "what": "ambrycrc_verify_dev per step: CRCs recomputed and compared with the clean pass; "
                            "single-bit flips in 1 % of chunks (seeded)"}),
    }
    pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc) and args.config == "c3":
        try:
            with open(pmc) as f:
                p = json.load(f)
            result["roofline"]["traffic"] = p.get("hbm_bytes_per_launch")
            result["roofline"]["traffic_source"] = p.get("source")
        except Exception:
            pass

    if rank == 0 and world == 1:
        if not args.no_cpu_baseline:
            log(args, "cpu baseline")
            cb = cpu_baseline(buf, off_t, len_t, n, args)
            if cb is not None:
                ref = cb.pop("_out")
                cb["parity_vs_gpu"] = bool((ref == crcs[:len(ref)]).all())
                result["cpu_baseline"] = cb
        if not args.no_host_path and args.config == "c3":
            log(args, "host-resident path")
            del buf
            torch.cuda.empty_cache()
            result["host_path"] = host_path_rate(torch, args)
    if rank == 0:
        sys.stdout.flush()
        os.write(result_fd, (json.dumps(result) + "\n").encode())
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
