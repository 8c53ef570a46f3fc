#!/bin/bash
# r06s8: region verify pass 2 (region_msg_kernel) load cost: product vs probe builds with no record CRCs
# (1), no run-sum loads (2), no head / tail run loads (3); msg4k / msg1k / msg100, interleaved twice.
set -o pipefail
export AMBRYCRC_PROBE=1  # timing-only probe builds: bench_messages skips its verdict checks
LIBS="abtmp/base/libambrycrc.so abtmp/prb1/libambrycrc.so abtmp/prb2/libambrycrc.so abtmp/prb3/libambrycrc.so" CASES="msg4k msg1k msg100" ROUNDS=2 REPS=10 timeout -k 10 800 bash tools/ab_cases.sh > gpurun_out/r06s8.log 2>&1 || { echo AB_FAILED; tail -5 gpurun_out/r06s8.log; exit 1; }
for d in gpurun_out/ab/*/msg*/r*; do
  python3 -c "
import csv,sys
d='$d'
for row in csv.DictReader(open(d+'/kt_kernel_stats.csv')):
    n=row['Name']
    if 'region_' in n: print(d.split('/ab/')[1], n.split('(')[0].replace('ambrycrc::','').split('<')[0], row['Calls'], round(float(row['AverageNs'])/1e3,1))
"
done
