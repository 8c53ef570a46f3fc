#!/bin/bash
# Kernel time of one small-record case at several batch sizes (fixed vs per-byte cost):
# rocprofv3 kernel trace of tools/probes/pmc_case.py <case> --gib <g> for g in $GIBS.
set -euo pipefail
export TMPDIR=/tmp
CASE=${CASE:-batch4k}
GIBS=${GIBS:-"0.25 0.5 1 2"}
OUT=gpurun_out/size_scan/$CASE
mkdir -p $OUT
for g in $GIBS; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/g$g -o kt \
    -- python3 tools/probes/pmc_case.py $CASE --gib $g --reps 5 > $OUT/g$g.log 2>&1
  f=$(find $OUT/g$g -name 'kt_kernel_stats.csv' | head -1)
  us=$(python3 -c "import csv,sys; print(sum(float(r['AverageNs'])/1e3 for r in csv.DictReader(open('$f')) if 'sweep_kernel' in r['Name'] or 'plan' in r['Name']))")
  echo "$CASE gib=$g kernels_us=$us"
done
