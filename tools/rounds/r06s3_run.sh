#!/bin/bash
# r06s3: the output-placement probe, fresh outputs first and rounded sizes.
set -o pipefail
timeout -k 10 300 python -u tools/probes/xform_offset.py --fresh-first --fresh 3 --offsets 0,1073741824 --round-to 2097152,1073741824 > gpurun_out/r06s3_a.jsonl 2> gpurun_out/r06s3_a.err || { echo A_FAILED; tail -5 gpurun_out/r06s3_a.err; exit 1; }
cat gpurun_out/r06s3_a.jsonl
timeout -k 10 300 python -u tools/probes/xform_offset.py --fresh 3 --offsets 0 --round-to 2097152,1073741824,4294967296 > gpurun_out/r06s3_b.jsonl 2> gpurun_out/r06s3_b.err || { echo B_FAILED; tail -5 gpurun_out/r06s3_b.err; exit 1; }
cat gpurun_out/r06s3_b.jsonl
echo DONE
