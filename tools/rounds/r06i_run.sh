#!/bin/bash
# Round 6: the 4 MiB-blob transform under the device and the host verdict, kernel traces.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in device host; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06i_kt_$v -o kt -- python3 tools/bench_put.py --cases '' --transform 4m --verdict $v --reps 5 > gpurun_out/r06i_$v.log 2>&1 || { echo FAILED $v; tail -5 gpurun_out/r06i_$v.log; exit 1; }
done
echo R06I_DONE
