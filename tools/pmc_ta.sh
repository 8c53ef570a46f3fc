#!/bin/bash
# Vector-memory front-end counters (TA / TD / TCP / TCC) of library builds side by side, for the
# small-record cases: is a CU's L1 path (addresses and cache lines per wave load) what bounds a
# group-phase round? One rocprofv3 --pmc pass per block limit (TA 2, TD 2, TCP 4, TCC 4).
export AMBRYCRC_ALLOW_PROBE=1  # the A/B libraries are probe builds (tools/ab_build.sh)
set -euo pipefail
export TMPDIR=/tmp
CASES=${CASES:-"batch100 batch4k"}
REPS=${REPS:-3}
OUT=gpurun_out/pmc_ta
mkdir -p $OUT
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
pick() { local s=""; for k in "$@"; do if grep -qw "$k" $OUT/counters.txt; then s="$s $k"; fi; done; echo $s; }
P1=$(pick SQ_WAVE_CYCLES SQ_BUSY_CYCLES TA_TA_BUSY TA_FLAT_READ_WAVEFRONTS TD_TD_BUSY TD_LOAD_WAVEFRONT GRBM_GUI_ACTIVE GRBM_COUNT)
P2=$(pick SQ_WAVE_CYCLES TCP_TOTAL_CACHE_ACCESSES TCP_TCC_READ_REQ TCP_PENDING_STALL_CYCLES TCP_TCP_TA_DATA_STALL_CYCLES TCC_HIT TCC_MISS TCC_REQ)
echo "pass1:$P1"; echo "pass2:$P2"
for lib in $LIBS; do
  tag=$(basename $(dirname $lib))
  for c in $CASES; do
    d=$OUT/$tag/$c
    mkdir -p $d
    for p in 1 2; do
      cn=P$p
      AMBRYCRC_LIBRARY=$(realpath $lib) timeout -s KILL 120 rocprofv3 --pmc ${!cn} --output-format csv -d $d/p$p -o pmc \
        -- python3 tools/probes/pmc_case.py $c --reps $REPS > $d/p$p.log 2>&1 || echo "pass $p failed"
      find $d/p$p -name 'pmc_counter_collection.csv' -exec cp {} $d/p$p.csv \; 2>/dev/null || true
      rm -rf $d/p$p
    done
    echo "$tag $c done"
  done
done
