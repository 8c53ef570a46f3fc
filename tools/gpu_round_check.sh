#!/bin/bash
# Round evidence on one GPU box: the full -m gpu suite, smoke(), the default bench line, then
# tools/profile.sh (kernel trace + PMC passes of the bench). Outputs under gpurun_out/${TAG}_*.
set -o pipefail
TAG=${TAG:-r02ap}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/${TAG}_gpu_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit 1
cat gpurun_out/${TAG}_bench.json
bash tools/profile.sh
echo ROUND_CHECK_DONE
