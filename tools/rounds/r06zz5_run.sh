#!/bin/bash
# r06zz5: the driver's multi-GPU launch form on the final tree, at the one rank this box has:
# torch.distributed.run with one process (procs mode: gloo control plane, RCCL communicator of one
# rank, ambrycrc_batch_dev_gather), default config (C3 at world size 1) and C5's 256 GiB shard.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 1 --steps 10 --warmup 2 > gpurun_out/r06zz5_procs_c3.json 2> gpurun_out/r06zz5_procs_c3.err || { echo C3_PROCS_FAILED; tail -5 gpurun_out/r06zz5_procs_c3.err; exit 1; }
cut -c1-300 gpurun_out/r06zz5_procs_c3.json
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 1 --config c5 --steps 5 --warmup 1 --no-cpu-baseline --no-host-path > gpurun_out/r06zz5_procs_c5.json 2> gpurun_out/r06zz5_procs_c5.err || { echo C5_PROCS_FAILED; tail -5 gpurun_out/r06zz5_procs_c5.err; exit 1; }
cut -c1-300 gpurun_out/r06zz5_procs_c5.json
echo R06ZZ5_DONE
