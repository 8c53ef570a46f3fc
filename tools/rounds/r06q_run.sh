#!/bin/bash
# Round 6: put_stream_kernel knobs one at a time (AMBRY_PS_SKIP, _DESC_VGPR, _PAIR_EDGES) against the
# round's first streamed form (old) and the LDS edge merge alone (ps_v1); 4 KiB PUTs, 1000 / 1005-B user metadata.
set -o pipefail
mkdir -p gpurun_out
export AMBRYCRC_ALLOW_PROBE=1
AMBRYCRC_LIBRARY=$(realpath abtmp/ps_all/libambrycrc.so) timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_put.py > gpurun_out/r06q_put_tests.log 2>&1 || { echo TESTS FAILED; tail -20 gpurun_out/r06q_put_tests.log; exit 1; }
tail -1 gpurun_out/r06q_put_tests.log
for r in 1 2; do
  for v in put_old ps_v1 ps_skip ps_desc ps_pair ps_all; do
    for um in 1000 1005; do
      AMBRYCRC_LIBRARY=$(realpath abtmp/$v/libambrycrc.so) timeout -k 10 200 python tools/bench_put.py --cases 4k --copy-only --transform '' --reps 20 --um-len $um > gpurun_out/r06q_${v}_um${um}_r$r.jsonl 2>&1 || { echo FAILED $v; tail -3 gpurun_out/r06q_${v}_um${um}_r$r.jsonl; exit 1; }
      echo $v um$um r$r $(grep -o '"ms_median": [0-9.]*' gpurun_out/r06q_${v}_um${um}_r$r.jsonl)
    done
  done
done
echo R06Q_DONE
