#!/bin/bash
# r06t1: region pass 2 reading each record's head / tail runs by lane quads (one 64-B request per run)
# instead of four 16-B loads per lane: the message GPU tests on the in-tree build, then HEAD vs quad
# builds on msg4k / msg1k / msg100 (kernel traces, interleaved twice; bench_messages checks parity).
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_messages.py tests/test_gpu_transform.py tests/test_filestore.py tests/test_protocol.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06t1_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r06t1_tests.log; exit 1; }
tail -n 2 gpurun_out/r06t1_tests.log
rm -rf gpurun_out/ab
LIBS="abtmp/head/libambrycrc.so abtmp/quad/libambrycrc.so" CASES="msg4k msg1k msg100" ROUNDS=2 REPS=10 timeout -k 10 600 bash tools/ab_cases.sh > gpurun_out/r06t1.log 2>&1 || { echo AB_FAILED; tail -5 gpurun_out/r06t1.log; exit 1; }
for d in gpurun_out/ab/*/msg*/r*; do
  python3 -c "
import csv
d='$d'
for row in csv.DictReader(open(d+'/kt_kernel_stats.csv')):
    n=row['Name']
    if 'region_' in n: print(d.split('/ab/')[1], n.split('(')[0].replace('ambrycrc::','').split('<')[0], row['Calls'], round(float(row['AverageNs'])/1e3,1))
"
done
