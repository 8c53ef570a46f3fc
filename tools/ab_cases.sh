#!/bin/bash
# A/B kernel timing on one box: the small-record cases of tools/probes/pmc_case.py under a
# rocprofv3 kernel trace, once per library build in $LIBS (paths to libambrycrc.so builds, loaded
# through AMBRYCRC_LIBRARY), interleaved A B A B ... $ROUNDS times so box-to-box and drift
# variance cancels. Then `python tools/ab_summary.py`.
set -euo pipefail
export TMPDIR=/tmp
CASES=${CASES:-"batch100 batch1k batch4k batch4109 msg4k"}
ROUNDS=${ROUNDS:-2}
REPS=${REPS:-5}
OUT=gpurun_out/ab
mkdir -p $OUT
for r in $(seq 1 $ROUNDS); do
  for lib in $LIBS; do
    tag=$(basename $(dirname $lib))
    for c in $CASES; do
      d=$OUT/$tag/$c/r$r
      mkdir -p $d
      AMBRYCRC_LIBRARY=$(realpath $lib) timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv \
        -d $d/kt -o kt -- python3 tools/probes/pmc_case.py $c --reps $REPS > $d/kt.log 2>&1
      find $d/kt -name '*kernel_stats.csv' -exec cp {} $d/ \;
      rm -rf $d/kt
    done
    echo "round $r lib $tag done"
  done
done
