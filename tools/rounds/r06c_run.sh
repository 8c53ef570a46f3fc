#!/bin/bash
# Round 6, one GPU call: the copy roof at 1.39 / 5.56 / 22.2 GB, the transform at 1x / 4x / 16x the 4 KiB region
# (both verdicts), and Crc32Benchmark's ladder on the final tree. Each step under its own limit.
set -o pipefail
mkdir -p gpurun_out
for b in 1389101056 5556404224 22225616896; do
  timeout -k 10 120 ./tools/probes/copy_roof $b >> gpurun_out/r06c_copy_roof.jsonl 2>&1 || { echo COPY_ROOF_FAILED; exit 1; }
done
tail -3 gpurun_out/r06c_copy_roof.jsonl
timeout -k 10 400 python tools/bench_put.py --cases '' --transform 4k,4kx4,4kx16 --verdict device,host --reps 10 > gpurun_out/r06c_xform_sizes.jsonl 2>&1 || { echo XFORM_FAILED; tail -5 gpurun_out/r06c_xform_sizes.jsonl; exit 1; }
grep -o '"case": "[^"]*"\|"verdict": "[^"]*"\|"ms_median": [0-9.]*\|"GBps_hbm_min": [0-9.]*' gpurun_out/r06c_xform_sizes.jsonl | paste - - - -
timeout -k 10 400 python tools/bench_ladder.py > gpurun_out/r06c_ladder.jsonl 2> gpurun_out/r06c_ladder.err || { echo LADDER_FAILED; tail -5 gpurun_out/r06c_ladder.err; exit 1; }
wc -l gpurun_out/r06c_ladder.jsonl
echo R06C_DONE
