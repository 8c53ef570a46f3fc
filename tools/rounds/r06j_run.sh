#!/bin/bash
# Round 6: put_stream_seal_kernel blocks per CU (2 / 3 / 4), interleaved A B C A B C, serialize 4 KiB PUTs.
set -o pipefail
mkdir -p gpurun_out
export AMBRYCRC_ALLOW_PROBE=1
for r in 1 2; do
  for b in 2 3 4; do
    AMBRYCRC_LIBRARY=$(realpath abtmp/seal$b/libambrycrc.so) timeout -k 10 200 python tools/bench_put.py --cases 4k --copy-only --transform '' --reps 20 > gpurun_out/r06j_seal${b}_r$r.jsonl 2>&1 || { echo FAILED $b; tail -3 gpurun_out/r06j_seal${b}_r$r.jsonl; exit 1; }
    echo seal$b r$r $(grep -o '"ms_median": [0-9.]*' gpurun_out/r06j_seal${b}_r$r.jsonl)
  done
done
echo R06J_DONE
