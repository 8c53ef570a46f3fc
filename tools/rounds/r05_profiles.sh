#!/bin/bash
# Round-5 profile evidence on one GPU box: tools/profile.sh (C3 kernel trace + FETCH / WRITE / SQ
# passes of bench.py), then a kernel trace of the C2, C4 and C5 (world size 1) bench lines. Each
# step under its own limit; outputs under gpurun_out/ (summarize with tools/summarize_profile.py).
set -euo pipefail
export TMPDIR=/tmp
TAG=${TAG:-r05k}
bash tools/profile.sh
echo PROFILE_DONE
A="--no-cpu-baseline --no-host-path --steps 10 --warmup 2"
for c in c2 c4 c5; do
  X=""; if [ $c = c5 ]; then X="--inproc --gpus 1"; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_${c}_kt -o kt -- \
    python3 bench.py --config $c $A $X > gpurun_out/${TAG}_${c}.json 2> gpurun_out/${TAG}_${c}.err
  find gpurun_out/${TAG}_${c}_kt -name '*kernel_stats.csv' -exec cp {} gpurun_out/${TAG}_${c}_kernel_stats.csv \;
  rm -rf gpurun_out/${TAG}_${c}_kt
  echo "$c: $(cut -c1-120 gpurun_out/${TAG}_${c}.json)"
done
echo PROFILES_DONE
