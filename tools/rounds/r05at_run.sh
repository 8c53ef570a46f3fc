# Copy-mode serialize A/B: copy-through (default) vs gather copy + CRC in place (AMBRYCRC_PUT_GATHER=1).
set -o pipefail
AMBRYCRC_PUT_GATHER=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_put.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05at_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r05at_tests.log; exit 1; }
tail -1 gpurun_out/r05at_tests.log
for r in 1 2; do for g in 0 1; do
  AMBRYCRC_PUT_GATHER=$g timeout -k 10 200 python tools/bench_put.py --cases 4k,64k,4m --copy-only > gpurun_out/r05at_g${g}_r${r}.jsonl 2>&1 || { echo FAILED g$g; tail -5 gpurun_out/r05at_g${g}_r${r}.jsonl; exit 1; }
  echo "g$g r$r $(grep -o '"case": "[^"]*"\|"ms_median": [0-9.]*' gpurun_out/r05at_g${g}_r${r}.jsonl | paste - - | tr '\n' ' ')"
done; done
