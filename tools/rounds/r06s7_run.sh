#!/bin/bash
# r06s7: serialize stream kernel pipelined across messages (AMBRY_STREAM_PIPE=1, in-tree) vs the round's
# previous form (probe build with the knob at 0): put GPU tests on the in-tree build, then both builds
# timed on 262,144 x 4 KiB PUTs, interleaved, both user-metadata sizes, plus a kernel trace of each.
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_put.py tests/test_gpu_transform.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06s7_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r06s7_tests.log; exit 1; }
tail -n 2 gpurun_out/r06s7_tests.log
for r in 1 2; do for lib in pipe0 pipe1; do for um in 1000 1005; do
AMBRYCRC_ALLOW_PROBE=1 AMBRYCRC_LIBRARY=$PWD/abtmp/$lib/libambrycrc.so timeout -k 10 200 python3 tools/bench_put.py --cases 4k --copy-only --transform '' --um-len $um --reps 20 > gpurun_out/r06s7_${lib}_um${um}_r$r.jsonl 2>&1 || { echo BENCH_FAILED; tail -5 gpurun_out/r06s7_${lib}_um${um}_r$r.jsonl; exit 1; }
echo "$lib um$um r$r $(grep -o '"ms_median": [0-9.]*' gpurun_out/r06s7_${lib}_um${um}_r$r.jsonl)"
done; done; done
for lib in pipe0 pipe1; do
AMBRYCRC_ALLOW_PROBE=1 AMBRYCRC_LIBRARY=$PWD/abtmp/$lib/libambrycrc.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06s7_kt_$lib -o kt -- python3 tools/bench_put.py --cases 4k --copy-only --transform '' --reps 20 > gpurun_out/r06s7_kt_$lib.log 2>&1 || { echo KT_FAILED; exit 1; }
find gpurun_out/r06s7_kt_$lib -name '*kernel_stats.csv' -exec cp {} gpurun_out/r06s7_${lib}_kernel_stats.csv \;
grep -i "put_" gpurun_out/r06s7_${lib}_kernel_stats.csv | cut -d, -f1-5 | sed "s/^/$lib /"
done
