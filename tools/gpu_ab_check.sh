#!/bin/bash
# Full GPU suite on the in-tree build, then an interleaved kernel-trace A/B of $LIBS on $CASES.
set -euo pipefail
TAG=${TAG:-ab}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_gpu_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_gpu_tests.log
LIBS="$LIBS" CASES="$CASES" ROUNDS=${ROUNDS:-2} timeout -k 10 400 bash tools/ab_cases.sh > gpurun_out/${TAG}_ab.log 2>&1
echo AB_DONE
