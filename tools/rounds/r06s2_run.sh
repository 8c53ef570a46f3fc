#!/bin/bash
# r06s2: the large-blob transform's output-placement probe, then a kernel trace of the 4 MiB transform.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u tools/probes/xform_offset.py > gpurun_out/r06s2_offset.jsonl 2> gpurun_out/r06s2_offset.err || { echo PROBE_FAILED; tail -5 gpurun_out/r06s2_offset.err; exit 1; }
cat gpurun_out/r06s2_offset.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06s2_kt -o kt -- python3 tools/bench_put.py --cases '' --transform 4m --verdict device --reps 5 > gpurun_out/r06s2_kt.log 2>&1 || { echo KT_FAILED; tail -5 gpurun_out/r06s2_kt.log; exit 1; }
echo DONE
