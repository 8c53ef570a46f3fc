#!/bin/bash
# Cache-side counters of the message-verify kernels (region pass 1 / pass 2) for $CASES
# (tools/probes/pmc_case.py), one rocprofv3 --pmc pass per counter set (no trace domains), each its
# own run: L2 hits / misses / requests / HBM read requests, then the L1 (TCP) and address-unit
# view. `python tools/pmc_cache_summary.py` prints the per-kernel averages.
set -euo pipefail
export TMPDIR=/tmp
CASES=${CASES:-"msg4k msg100"}
REPS=${REPS:-3}
OUT=gpurun_out/pmc_cache
mkdir -p $OUT
P1="TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum TCC_EA0_RDREQ_sum"
P2="TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum"
for c in $CASES; do
  for p in 1 2; do
    cn=P$p
    d=$OUT/$c/p$p
    timeout -s KILL 120 rocprofv3 --pmc ${!cn} --output-format csv -d $d -o pmc -- python3 tools/probes/pmc_case.py $c --reps $REPS > $OUT/$c.p$p.log 2>&1
    find $d -name 'pmc_counter_collection.csv' -exec cp {} $OUT/$c.p$p.csv \;
    rm -rf $d
  done
  echo "$c done"
done
