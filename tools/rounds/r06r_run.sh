#!/bin/bash
# Round 6: the transform's device verdict on a side stream: transform tests, then
# the side form against the inline gated chain (AMBRYCRC_XFORM_SIDE=0) and the host verdict, interleaved.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_transform.py > gpurun_out/r06r_xform_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r06r_xform_tests.log; exit 1; }
tail -1 gpurun_out/r06r_xform_tests.log
for r in 1 2; do
  for side in 1 0; do
    AMBRYCRC_XFORM_SIDE=$side timeout -k 10 300 python tools/bench_put.py --cases '' --transform 4k,4kx4 --verdict device,host --reps 20 > gpurun_out/r06r_side${side}_r$r.jsonl 2>&1 || { echo FAILED $side; tail -3 gpurun_out/r06r_side${side}_r$r.jsonl; exit 1; }
    echo side$side r$r; python -c "import json,sys; [print(d[\"case\"][:40], d[\"verdict\"], d[\"ms_median\"], d[\"ms_back_to_back\"], d.get(\"path_taken\")) for d in map(json.loads, open(sys.argv[1]))]" gpurun_out/r06r_side${side}_r$r.jsonl
  done
done
echo R06R_DONE
