#!/bin/bash
# r06zz2: the layout kernel leaves streamed messages' job entries unwritten (a gated clear launch zeroes them
# when the job path runs) and stages its tables only in blocks that hash: put / transform GPU tests on the
# in-tree build, then HEAD (abtmp/head) vs the working tree (abtmp/new) on 262,144 x 4 KiB PUTs, interleaved,
# plus a kernel trace of each.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_put.py tests/test_gpu_transform.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06zz2_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r06zz2_tests.log; exit 1; }
tail -n 2 gpurun_out/r06zz2_tests.log
for r in 1 2 3; do for lib in head new; do
AMBRYCRC_ALLOW_PROBE=1 AMBRYCRC_LIBRARY=$PWD/abtmp/$lib/libambrycrc.so timeout -k 10 200 python3 tools/bench_put.py --cases 4k --copy-only --transform '' --reps 30 > gpurun_out/r06zz2_${lib}_r$r.jsonl 2>&1 || { echo BENCH_FAILED; tail -5 gpurun_out/r06zz2_${lib}_r$r.jsonl; exit 1; }
echo "$lib r$r $(grep -o '"ms_median": [0-9.]*' gpurun_out/r06zz2_${lib}_r$r.jsonl)"
done; done
for lib in head new; do
AMBRYCRC_ALLOW_PROBE=1 AMBRYCRC_LIBRARY=$PWD/abtmp/$lib/libambrycrc.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06zz2_kt_$lib -o kt -- python3 tools/bench_put.py --cases 4k --copy-only --transform '' --reps 20 > gpurun_out/r06zz2_kt_$lib.log 2>&1 || { echo KT_FAILED; exit 1; }
find gpurun_out/r06zz2_kt_$lib -name '*kernel_stats.csv' -exec cp {} gpurun_out/r06zz2_${lib}_kernel_stats.csv \;
grep -i "put_" gpurun_out/r06zz2_${lib}_kernel_stats.csv | cut -d, -f1-5 | sed "s/^/$lib /"
done
echo R06ZZ2_DONE
