#!/bin/bash
# Round 6: serialize streamed form, wave pieces past the message skipped, edge bytes merged through LDS:
# put tests on the product library, then old / new interleaved on 4 KiB PUTs (1000-B and 1005-B user metadata).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_put.py > gpurun_out/r06p_put_tests.log 2>&1 || { echo TESTS FAILED; tail -20 gpurun_out/r06p_put_tests.log; exit 1; }
tail -1 gpurun_out/r06p_put_tests.log
export AMBRYCRC_ALLOW_PROBE=1
for r in 1 2; do
  for v in old new; do
    for um in 1000 1005; do
      AMBRYCRC_LIBRARY=$(realpath abtmp/put_$v/libambrycrc.so) timeout -k 10 200 python tools/bench_put.py --cases 4k --copy-only --transform '' --reps 20 --um-len $um > gpurun_out/r06p_${v}_um${um}_r$r.jsonl 2>&1 || { echo FAILED $v; tail -3 gpurun_out/r06p_${v}_um${um}_r$r.jsonl; exit 1; }
      echo $v um$um r$r $(grep -o '"ms_median": [0-9.]*' gpurun_out/r06p_${v}_um${um}_r$r.jsonl)
    done
  done
done
echo R06P_DONE
