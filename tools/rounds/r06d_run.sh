#!/bin/bash
# Round 6: message verify at every small size in both region forms (one pass / two passes) and the long-record
# mix, to pick the default form. Each step under its own limit.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python tools/bench_messages.py --cases 4k,3k,2k,1k,100 --modes region,region2 --reps 10 > gpurun_out/r06d_messages.jsonl 2>&1 || { echo MSG_FAILED; tail -5 gpurun_out/r06d_messages.jsonl; exit 1; }
grep -o '"mode_taken": "[^"]*"\|"config": "[^"]*"\|"ms_median": [0-9.]*' gpurun_out/r06d_messages.jsonl | paste - - -
timeout -k 10 300 python tools/probes/long_mix.py > gpurun_out/r06d_longmix.json 2>&1 || { echo LONGMIX_FAILED; tail -5 gpurun_out/r06d_longmix.json; exit 1; }
cat gpurun_out/r06d_longmix.json | tail -5
echo R06D_DONE
