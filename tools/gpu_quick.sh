#!/bin/bash
# One GPU call: the -m gpu suite (or the tests named in $TESTS), smoke(), then the default bench line.
# Each step under its own time limit, stopping at the first failure. Outputs under gpurun_out/${TAG}_*.
set -o pipefail
TAG=${TAG:-r06}
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/${TAG}_gpu_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo SMOKE_FAILED; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
if [ -z "$NO_BENCH" ]; then
  timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo BENCH_FAILED; tail -5 gpurun_out/${TAG}_bench.err; exit 1; }
  cat gpurun_out/${TAG}_bench.json
fi
echo QUICK_DONE
