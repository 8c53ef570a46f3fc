#!/bin/bash
# Round 6: the single-read segmented-scan verify probe (tools/probes/seg_verify, built in-tree on the CPU)
# and the two-pass product on the same box.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 180 tools/probes/seg_verify ambry_amd/libambrycrc.so > gpurun_out/r06g_seg.jsonl 2>&1 || { echo SEG_FAILED; tail -5 gpurun_out/r06g_seg.jsonl; exit 1; }
cat gpurun_out/r06g_seg.jsonl
timeout -k 10 300 python tools/bench_messages.py --cases 4k,1k,100 --modes region2 --reps 10 > gpurun_out/r06g_messages.jsonl 2>&1 || { echo MSG_FAILED; exit 1; }
grep -o '"config": "[^"]*"\|"ms_median": [0-9.]*' gpurun_out/r06g_messages.jsonl | paste - -
echo R06G_DONE
