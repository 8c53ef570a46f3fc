#!/bin/bash
# One GPU call's worth of round evidence, each step under its own time limit, stopping at the first
# failure: the full -m gpu suite, smoke(), the message verify and PUT/transform benches, kernel
# traces of the small-record cases, and the default bench line. Outputs under gpurun_out/${TAG}_*.
set -o pipefail
TAG=${TAG:-r04}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/${TAG}_gpu_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo SMOKE_FAILED; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 300 python tools/bench_messages.py --cases ${MSG_CASES:-4k,1k,100,64k} --modes ${MSG_MODES:-region,region2,jobs} > gpurun_out/${TAG}_messages.jsonl 2>&1 || { echo MSG_BENCH_FAILED; tail -5 gpurun_out/${TAG}_messages.jsonl; exit 1; }
grep -o '"config": "[^"]*"\|"mode_taken": "[^"]*"\|"ms_median": [0-9.]*\|"GiBps": [0-9.]*' gpurun_out/${TAG}_messages.jsonl | paste - - - - | grep -v C1
timeout -k 10 400 python tools/bench_put.py --cases ${PUT_CASES:-4k,64k} --transform ${XFORM_CASES:-64k,4k,4m} --copy-only > gpurun_out/${TAG}_put.jsonl 2>&1 || { echo PUT_BENCH_FAILED; tail -5 gpurun_out/${TAG}_put.jsonl; exit 1; }
grep -o '"case": "[^"]*"\|"ms_median": [0-9.]*' gpurun_out/${TAG}_put.jsonl | paste - -
if [ -n "${KT_CASES-msg4k msg1k xform4k}" ]; then
  TAG=${TAG}_kt CASES="${KT_CASES-msg4k msg1k xform4k}" timeout -k 10 400 bash tools/kt_cases.sh > /dev/null 2>&1 || { echo KT_FAILED; exit 1; }
  python tools/kt_summary.py gpurun_out/kt/${TAG}_kt | grep -v "rocprim\|at::native\|rocclr\|fill_splitmix"
fi
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo BENCH_FAILED; tail -5 gpurun_out/${TAG}_bench.err; exit 1; }
cut -c1-400 gpurun_out/${TAG}_bench.json
echo ROUND_CHECK_DONE
