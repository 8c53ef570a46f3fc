#!/bin/bash
# rocprofv3 evidence for the small-record paths, on the GPU box from the
# repo root: for each case of tools/probes/pmc_case.py, a kernel-trace pass and three counter
# passes (FETCH_SIZE; WRITE_SIZE; SQ issue/wait counters + GRBM_GUI_ACTIVE), each its own run,
# no trace domain combined with --pmc. Then `python tools/summarize_cases.py --tag <tag>`.
set -euo pipefail
export TMPDIR=/tmp
CASES=${CASES:-"scatter16 scatter4 scatter8 msg4k msg1k msg4k_1pass xform4k xform64k batch100 batch4k put4k"}
REPS=${REPS:-5}
mkdir -p gpurun_out/pmc_cases
# keep only the SQ counters this rocprofv3 lists for the device
timeout -s KILL 60 rocprofv3 -L > gpurun_out/pmc_cases/counters.txt 2>&1 || true
SQ=""
for k in SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD; do
  if grep -qw "$k" gpurun_out/pmc_cases/counters.txt; then SQ="$SQ $k"; fi
done
echo "SQ counters:$SQ"
for c in $CASES; do
  d=gpurun_out/pmc_cases/$c
  mkdir -p $d
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $d/kt -o kt -- python3 tools/probes/pmc_case.py $c --reps $REPS > $d/kt.log 2>&1
  if [ -n "${KT_ONLY:-}" ]; then
    find $d/kt -mindepth 2 -name '*.csv' -exec cp {} $d/kt/ \;
    echo "case $c done (kernel trace only)"
    continue
  fi
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $d/fetch -o pmc -- python3 tools/probes/pmc_case.py $c --reps $REPS > $d/fetch.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $d/write -o pmc -- python3 tools/probes/pmc_case.py $c --reps $REPS > $d/write.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc $SQ GRBM_GUI_ACTIVE --output-format csv -d $d/sq -o pmc -- python3 tools/probes/pmc_case.py $c --reps $REPS > $d/sq.log 2>&1
  for p in kt fetch write sq; do
    find $d/$p -mindepth 2 -name '*.csv' -exec cp {} $d/$p/ \;
  done
  echo "case $c done"
done
