#!/bin/bash
# r06t2: final-tree PMC passes (kernel trace, FETCH_SIZE, WRITE_SIZE, SQ) of the small-record cases,
# then the paired summary (tools/summarize_cases.py).
set -o pipefail
rm -rf gpurun_out/pmc_cases
CASES="msg4k msg1k msg100 xform4k put4k" REPS=5 timeout -k 10 900 bash tools/pmc_cases.sh > gpurun_out/r06t2_pmc.log 2>&1 || { echo PMC_FAILED; tail -5 gpurun_out/r06t2_pmc.log; exit 1; }
tail -n 6 gpurun_out/r06t2_pmc.log
python3 tools/summarize_cases.py --tag r06t2 > gpurun_out/r06t2_summary.txt 2>&1; tail -n 40 gpurun_out/r06t2_summary.txt
