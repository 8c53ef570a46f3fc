#!/bin/bash
# r06s9: final-tree check: the -m gpu suite, smoke(), the bench line, serialize / transform cases,
# and the read roof at the small-record regions' size (1.29 GiB) next to the C3 size.
set -o pipefail
export TMPDIR=/tmp
TAG=r06s9 NO_BENCH= bash tools/gpu_quick.sh || exit 1
timeout -k 10 300 python3 tools/bench_put.py --cases 4k --copy-only --transform 4k --reps 20 > gpurun_out/r06s9_put.jsonl 2>&1 || { echo PUT_FAILED; tail -5 gpurun_out/r06s9_put.jsonl; exit 1; }
grep -o '"case": "[^"]*"\|"verdict": "[a-z]*"\|"ms_median": [0-9.]*\|"ms_back_to_back": [0-9.]*' gpurun_out/r06s9_put.jsonl | paste -sd' ' | sed 's/"case"/\n"case"/g'
echo
timeout -k 10 120 tools/probes/readroof 1.289 > gpurun_out/r06s9_readroof_small.txt 2>&1 || { echo RR_FAILED; exit 1; }
tail -n 4 gpurun_out/r06s9_readroof_small.txt
timeout -k 10 300 python3 tools/bench_messages.py --cases 4k,1k,100 --reps 10 > gpurun_out/r06s9_messages.jsonl 2>&1 || { echo MSG_FAILED; tail -5 gpurun_out/r06s9_messages.jsonl; exit 1; }
grep -o '"case": "[^"]*"\|"ms_median": [0-9.]*' gpurun_out/r06s9_messages.jsonl | paste -sd' ' | sed 's/"case"/\n"case"/g'
echo FINAL_DONE
