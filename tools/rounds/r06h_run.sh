#!/bin/bash
# Round 6: counters of the segmented-scan verify probe's stream kernel (one --pmc pass each, no trace domains).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD --output-format csv -d gpurun_out/r06h_sq -o pmc -- tools/probes/seg_verify ambry_amd/libambrycrc.so > gpurun_out/r06h_sq.log 2>&1 || { echo SQ_FAILED; tail -5 gpurun_out/r06h_sq.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/r06h_sq2 -o pmc -- tools/probes/seg_verify ambry_amd/libambrycrc.so > gpurun_out/r06h_sq2.log 2>&1 || { echo SQ2_FAILED; tail -5 gpurun_out/r06h_sq2.log; exit 1; }
find gpurun_out/r06h_sq gpurun_out/r06h_sq2 -name '*counter_collection.csv'
echo R06H_DONE
