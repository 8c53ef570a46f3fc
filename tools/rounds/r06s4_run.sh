#!/bin/bash
# r06s4: copy forms over 17.2 GB into 5 fresh destinations (placement sensitivity of share vs window
# forms), then the 4 MiB transform into fresh outputs at several sweep windows.
set -o pipefail
timeout -k 10 300 tools/probes/copy_roof 17184796672 5 > gpurun_out/r06s4_copy.jsonl 2>&1 || { echo FAILED; tail -5 gpurun_out/r06s4_copy.jsonl; exit 1; }
cat gpurun_out/r06s4_copy.jsonl
timeout -k 10 400 python -u tools/probes/xform_offset.py --fresh 5 --offsets 0 --windows 0,4294967296,1073741824,268435456 > gpurun_out/r06s4_win.jsonl 2> gpurun_out/r06s4_win.err || { echo WIN_FAILED; tail -5 gpurun_out/r06s4_win.err; exit 1; }
cat gpurun_out/r06s4_win.jsonl
