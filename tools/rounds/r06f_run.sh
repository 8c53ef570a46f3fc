#!/bin/bash
# Round 6: the streamed serialize at a misaligned (1000-B user metadata: blob content 11 B off) and an
# aligned (1005 B) layout, both forms, with kernel traces.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for um in 1000 1005; do
  for form in stream jobs; do
    env_max=""; [ $form = jobs ] && env_max=0
    AMBRYCRC_STREAM_PUT_MAX=${env_max:-6144} timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06f_kt_${form}_${um} -o kt -- python3 tools/bench_put.py --cases 4k --copy-only --transform '' --reps 10 --um-len $um > gpurun_out/r06f_${form}_${um}.log 2>&1 || { echo FAILED $form $um; exit 1; }
  done
done
echo R06F_DONE
