#!/bin/bash
# Round 6 final check on the committed tree: the full -m gpu suite, smoke, message / PUT / transform
# benches, the default bench line; then the probe's counters (r06h).
set -o pipefail
mkdir -p gpurun_out
TAG=r06z KT_CASES="" bash tools/round_check.sh || exit 1
bash tools/rounds/r06h_run.sh || exit 1
echo R06Z_DONE
