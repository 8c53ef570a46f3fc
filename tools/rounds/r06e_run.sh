#!/bin/bash
# Round 6: the streamed serialize (put_stream_kernel) -- the PUT tests in both copy-mode forms, then the
# serialize bench in both forms; and a kernel trace of the 4x-size transform under the device verdict.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_put.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r06e_put_tests.log 2>&1 || { echo PUT_TESTS_FAILED; tail -40 gpurun_out/r06e_put_tests.log; exit 1; }
tail -2 gpurun_out/r06e_put_tests.log
timeout -k 10 300 python tools/bench_put.py --cases 4k,64k --copy-only --transform '' --reps 10 > gpurun_out/r06e_put_stream.jsonl 2>&1 || { echo PUT_BENCH_FAILED; tail -5 gpurun_out/r06e_put_stream.jsonl; exit 1; }
AMBRYCRC_STREAM_PUT_MAX=0 timeout -k 10 300 python tools/bench_put.py --cases 4k --copy-only --transform '' --reps 10 > gpurun_out/r06e_put_jobs.jsonl 2>&1 || { echo PUT_BENCH_JOBS_FAILED; tail -5 gpurun_out/r06e_put_jobs.jsonl; exit 1; }
grep -h -o '"case": "[^"]*"\|"ms_median": [0-9.]*' gpurun_out/r06e_put_stream.jsonl gpurun_out/r06e_put_jobs.jsonl | paste - -
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06e_kt_put -o kt -- python3 tools/bench_put.py --cases 4k --copy-only --transform '' --reps 5 > gpurun_out/r06e_kt_put.log 2>&1 || { echo KT_PUT_FAILED; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06e_kt_x4 -o kt -- python3 tools/bench_put.py --cases '' --transform 4kx4 --verdict device --reps 5 > gpurun_out/r06e_kt_x4.log 2>&1 || { echo KT_X4_FAILED; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06e_kt_x4h -o kt -- python3 tools/bench_put.py --cases '' --transform 4kx4 --verdict host --reps 5 > gpurun_out/r06e_kt_x4h.log 2>&1 || { echo KT_X4H_FAILED; exit 1; }
find gpurun_out/r06e_kt_put gpurun_out/r06e_kt_x4 -name '*kernel_stats.csv' | head
echo R06E_DONE
