#!/bin/bash
# r06zz3: as r06zz2, with the streamed form's gated job path moved to the stream's side stream (ring slot word 2,
# done signal): put / transform GPU tests, HEAD vs the working tree (abtmp/new2) on 262,144 x 4 KiB PUTs,
# interleaved, plus a kernel trace of each.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_put.py tests/test_gpu_transform.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06zz3_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r06zz3_tests.log; exit 1; }
tail -n 2 gpurun_out/r06zz3_tests.log
for r in 1 2 3; do for lib in head new2; do
AMBRYCRC_ALLOW_PROBE=1 AMBRYCRC_LIBRARY=$PWD/abtmp/$lib/libambrycrc.so timeout -k 10 200 python3 tools/bench_put.py --cases 4k --copy-only --transform '' --reps 30 > gpurun_out/r06zz3_${lib}_r$r.jsonl 2>&1 || { echo BENCH_FAILED; tail -5 gpurun_out/r06zz3_${lib}_r$r.jsonl; exit 1; }
echo "$lib r$r $(grep -o '"ms_median": [0-9.]*' gpurun_out/r06zz3_${lib}_r$r.jsonl)"
done; done
for lib in head new2; do
AMBRYCRC_ALLOW_PROBE=1 AMBRYCRC_LIBRARY=$PWD/abtmp/$lib/libambrycrc.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06zz3_kt_$lib -o kt -- python3 tools/bench_put.py --cases 4k --copy-only --transform '' --reps 20 > gpurun_out/r06zz3_kt_$lib.log 2>&1 || { echo KT_FAILED; exit 1; }
find gpurun_out/r06zz3_kt_$lib -name '*kernel_stats.csv' -exec cp {} gpurun_out/r06zz3_${lib}_kernel_stats.csv \;
grep -i "put_" gpurun_out/r06zz3_${lib}_kernel_stats.csv | cut -d, -f1-5 | sed "s/^/$lib /"
done
echo R06ZZ3_DONE
