# Round-5 check of the copy form's ends-early change: GPU suite, transform timings, xform4k PMC
# traffic, bench line (the host-leg calibration). Outputs under gpurun_out/r05ar_*.
set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05ar_gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r05ar_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r05ar_gpu_tests.log
timeout -k 10 300 python tools/bench_put.py --cases 4k --transform 4k --copy-only > gpurun_out/r05ar_put.jsonl 2>&1 || { echo PUT_FAILED; tail -5 gpurun_out/r05ar_put.jsonl; exit 1; }
grep -o '"case": "[^"]*"\|"ms_median": [0-9.]*' gpurun_out/r05ar_put.jsonl | paste - -
rm -rf gpurun_out/pmc_cases
CASES="xform4k" REPS=5 timeout -k 10 400 bash tools/pmc_cases.sh > gpurun_out/r05ar_pmc.log 2>&1 || { echo PMC_FAILED; tail -5 gpurun_out/r05ar_pmc.log; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/r05ar_bench.json 2> gpurun_out/r05ar_bench.err || { echo BENCH_FAILED; exit 1; }
python -c "
import json;d=json.load(open('gpurun_out/r05ar_bench.json'));print(d['value'], d['host_path']['dispatch'])"
