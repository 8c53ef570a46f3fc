#!/bin/bash
# A/B kernel timing on one box: the small-record cases of tools/probes/pmc_case.py under a
# rocprofv3 kernel trace, once per library build in $LIBS (paths to libambrycrc.so builds, loaded
# through AMBRYCRC_LIBRARY), interleaved A B A B ... $ROUNDS times so box-to-box and drift
# variance cancels. Then `python tools/ab_summary.py`.
export AMBRYCRC_ALLOW_PROBE=1  # the A/B libraries are probe builds (tools/ab_build.sh)
set -euo pipefail
export TMPDIR=/tmp
CASES=${CASES:-"batch100 batch1k batch4k batch4109 msg4k"}
ROUNDS=${ROUNDS:-2}
REPS=${REPS:-5}
OUT=gpurun_out/ab
mkdir -p $OUT
# VARIANTS (optional): run each library once per AMBRYCRC_VARIANT value, tagged <lib>_v<variant>.
VARIANTS=${VARIANTS:-"-"}
for r in $(seq 1 $ROUNDS); do
  for lib in $LIBS; do
    for v in $VARIANTS; do
      tag=$(basename $(dirname $lib))
      if [ "$v" != "-" ]; then tag=${tag}_v$v; export AMBRYCRC_VARIANT=$v; else unset AMBRYCRC_VARIANT; fi
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
done
