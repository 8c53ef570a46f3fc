#!/bin/bash
# r06s5: the serialize seal's load cost: in-tree build vs probe builds without head/tail loads (3) or
# run-sum loads (2), put4k copy mode under a kernel trace, interleaved twice.
set -o pipefail
LIBS="abtmp/base/libambrycrc.so abtmp/prb3/libambrycrc.so abtmp/prb2/libambrycrc.so" CASES=put4k ROUNDS=2 REPS=10 timeout -k 10 600 bash tools/ab_cases.sh > gpurun_out/r06s5.log 2>&1 || { echo AB_FAILED; tail -5 gpurun_out/r06s5.log; exit 1; }
python3 tools/ab_summary.py > gpurun_out/r06s5_summary.txt 2>&1; cat gpurun_out/r06s5_summary.txt | head -60
