#!/bin/bash
# Round 6, last session: the rebuilt tree (fresh container) checked end to end -- the full -m gpu
# suite, smoke, message / PUT / transform benches, the default bench line -- then bench.py's
# rocprofv3 kernel trace and HBM counter passes (tools/profile.sh).
set -o pipefail
mkdir -p gpurun_out
TAG=r06zz KT_CASES="" bash tools/round_check.sh || exit 1
bash tools/profile.sh || { echo PROFILE_FAILED; exit 1; }
echo R06ZZ_DONE
