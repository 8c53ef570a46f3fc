#!/bin/bash
# Round-mapping A/B (AMBRY_GRP_IL class bitmask): GPU parity of the builds in $BUILDS, then the
# interleaved kernel-time A/B (tools/ab_cases.sh) of base and them.
export AMBRYCRC_ALLOW_PROBE=1  # the A/B libraries are probe builds (tools/ab_build.sh)
set -euo pipefail
BUILDS=${BUILDS:-"il12 il4 il8 il15"}
for b in $BUILDS; do
  AMBRYCRC_LIBRARY=$PWD/build/ab/$b/libambrycrc.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 \
    --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_put.py tests/test_gpu_messages.py \
    tests/test_gpu_transform.py > gpurun_out/${b}_tests.log 2>&1
  echo "$b $(tail -1 gpurun_out/${b}_tests.log)"
done
LIBS="build/ab/base/libambrycrc.so $(for b in $BUILDS; do echo -n "build/ab/$b/libambrycrc.so "; done)" \
  ROUNDS=${ROUNDS:-3} CASES=${CASES:-"batch100 batch1k batch4k batch4109 msg4k put4k"} bash tools/ab_cases.sh
