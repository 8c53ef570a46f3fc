#!/bin/bash
# Round 6: serialize streamed form -- is the 1000-B user-metadata case's extra time the blob's unaligned
# source loads? 4 KiB PUTs, blob source shifted 0 / 11 B (11: every blob load 16-B aligned).
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for sh in 0 11; do
    timeout -k 10 200 python tools/bench_put.py --cases 4k --copy-only --transform '' --reps 20 --blob-shift $sh > gpurun_out/r06n_sh${sh}_r$r.jsonl 2>&1 || { echo FAILED $sh; tail -3 gpurun_out/r06n_sh${sh}_r$r.jsonl; exit 1; }
    echo shift$sh r$r $(grep -o '"ms_median": [0-9.]*' gpurun_out/r06n_sh${sh}_r$r.jsonl)
  done
done
echo R06N_DONE
