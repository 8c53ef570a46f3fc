#!/bin/bash
# Kernel trace (rocprofv3 --kernel-trace --stats) of tools/probes/pmc_case.py cases, one directory
# per case and tag: gpurun_out/kt/<TAG>/<case>/. Environment passes through (AMBRYCRC_FUSED_PROC,
# AMBRYCRC_REGION, ...). Then: python tools/kt_summary.py gpurun_out/kt/<TAG>
set -euo pipefail
export TMPDIR=/tmp
TAG=${TAG:-kt}
CASES=${CASES:-"msg4k msg1k"}
REPS=${REPS:-5}
for c in $CASES; do
  d=gpurun_out/kt/$TAG/$c
  mkdir -p $d
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $d/raw -o kt -- python3 tools/probes/pmc_case.py $c --reps $REPS > $d/kt.log 2>&1
  find $d/raw -name '*.csv' -exec cp {} $d/ \;
  rm -rf $d/raw
  echo "case $c done"
done
