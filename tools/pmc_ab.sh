#!/bin/bash
# SQ counters of library builds side by side (A/B of kernel shapes): for each lib in $LIBS and
# case in $CASES (tools/probes/pmc_case.py), two rocprofv3 --pmc passes of <= 8 SQ counters each
# (no trace domain with --pmc), every pass its own run. Then `python tools/pmc_ab_summary.py`.
export AMBRYCRC_ALLOW_PROBE=1  # the A/B libraries are probe builds (tools/ab_build.sh)
set -euo pipefail
export TMPDIR=/tmp
CASES=${CASES:-"batch4k"}
REPS=${REPS:-3}
OUT=gpurun_out/pmc_ab
mkdir -p $OUT
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
pick() { local s=""; for k in "$@"; do if grep -qw "$k" $OUT/counters.txt; then s="$s $k"; fi; done; echo $s; }
P1=$(pick SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_WAVES)
P2=$(pick SQ_WAVE_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS)
echo "pass1:$P1"; echo "pass2:$P2"
for lib in $LIBS; do
  tag=$(basename $(dirname $lib))
  for c in $CASES; do
    d=$OUT/$tag/$c
    mkdir -p $d
    for p in 1 2; do
      cn=P$p
      AMBRYCRC_LIBRARY=$(realpath $lib) timeout -s KILL 120 rocprofv3 --pmc ${!cn} --output-format csv -d $d/p$p -o pmc \
        -- python3 tools/probes/pmc_case.py $c --reps $REPS > $d/p$p.log 2>&1
      find $d/p$p -name 'pmc_counter_collection.csv' -exec cp {} $d/ \; 2>/dev/null || true
      mv $d/pmc_counter_collection.csv $d/p$p.csv 2>/dev/null || true
      rm -rf $d/p$p
    done
    echo "$tag $c done"
  done
done
