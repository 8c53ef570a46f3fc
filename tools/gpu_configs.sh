#!/bin/bash
# Every BASELINE config's bench line on the current build (one GPU box): C1 (CPU), C2, C4
# verify-on-read, C5's per-GPU shard through the one-process-per-GPU RCCL gather (torchrun,
# world size 1) and through the one-process multi entry. Lines go to gpurun_out/<tag>_<config>.json.
set -euo pipefail
TAG=${TAG:-cfg}
mkdir -p gpurun_out
A="--no-cpu-baseline --no-host-path --steps 10 --warmup 2"
timeout -k 10 120 python bench.py --config c1 > gpurun_out/${TAG}_c1.json 2> gpurun_out/${TAG}_c1.err
timeout -k 10 180 python bench.py --config c2 $A > gpurun_out/${TAG}_c2.json 2> gpurun_out/${TAG}_c2.err
timeout -k 10 180 python bench.py --config c4 $A > gpurun_out/${TAG}_c4.json 2> gpurun_out/${TAG}_c4.err
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29561 bench.py --gpus 1 --config c5 $A > gpurun_out/${TAG}_c5_procs.json 2> gpurun_out/${TAG}_c5_procs.err
timeout -k 10 300 python bench.py --gpus 1 --inproc --config c5 $A > gpurun_out/${TAG}_c5_inproc.json 2> gpurun_out/${TAG}_c5_inproc.err
echo CONFIGS_DONE
