#!/bin/bash
# r06s6: serialize stream kernel with the LDS segment table (no select chains, no flat loads):
# the put GPU tests, then bench_put 4k copy mode at both user-metadata sizes, twice, under a kernel trace.
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_put.py tests/test_gpu_transform.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06s6_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r06s6_tests.log; exit 1; }
tail -n 2 gpurun_out/r06s6_tests.log
for r in 1 2; do for um in 1000 1005; do
timeout -k 10 200 python3 tools/bench_put.py --cases 4k --copy-only --transform '' --um-len $um --reps 20 > gpurun_out/r06s6_put_um${um}_r$r.jsonl 2>&1 || { echo BENCH_FAILED; tail -5 gpurun_out/r06s6_put_um${um}_r$r.jsonl; exit 1; }
grep -o '"ms_median": [0-9.]*' gpurun_out/r06s6_put_um${um}_r$r.jsonl | sed "s/^/um$um r$r /"
done; done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06s6_kt -o kt -- python3 tools/bench_put.py --cases 4k --copy-only --transform '' --reps 20 > gpurun_out/r06s6_kt.log 2>&1 || { echo KT_FAILED; exit 1; }
find gpurun_out/r06s6_kt -name '*kernel_stats.csv' -exec cp {} gpurun_out/r06s6_kernel_stats.csv \;
grep -i "put_" gpurun_out/r06s6_kernel_stats.csv | cut -d, -f1-5
