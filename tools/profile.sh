#!/bin/bash
# rocprofv3 evidence for bench.py's roofline (run on the GPU box from the repo root):
#   prof_kt     --kernel-trace --stats      per-kernel durations (sweep kernel average)
#   prof_fetch  --pmc FETCH_SIZE            HBM read KiB (gfx950: half the bytes of a wide stream)
#   prof_write  --pmc WRITE_SIZE            HBM write KiB
#   prof_sq     --pmc SQ_* GRBM_GUI_ACTIVE  LDS / VALU issue and bank conflicts
# Each counter set in its own pass, no trace domains combined with --pmc. Then
#   python tools/summarize_profile.py --tag <round tag> --config <c3|c2|c5>
# copies the summaries into profiles/ and the traffic into bench_data/pmc_traffic.json.
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
# the kernel-trace pass profiles the bench command itself (default arguments unless
# BENCH_ARGS is set); the counter passes skip the CPU baseline and host path to stay short
ARGS=${BENCH_ARGS:-""}
PMC_ARGS=${PMC_BENCH_ARGS:-"--steps 5 --warmup 2 --no-cpu-baseline --no-host-path"}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_kt -o kt -- python3 bench.py $ARGS > gpurun_out/prof_kt.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch -o pmc -- python3 bench.py $PMC_ARGS > gpurun_out/prof_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write -o pmc -- python3 bench.py $PMC_ARGS > gpurun_out/prof_write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/prof_sq -o pmc -- python3 bench.py $PMC_ARGS > gpurun_out/prof_sq.log 2>&1
# rocprofv3 nests outputs under a host/pid directory: flatten the files summarize_profile.py reads
for d in prof_kt prof_fetch prof_write prof_sq; do
  find gpurun_out/$d -mindepth 2 -name '*.csv' -exec cp {} gpurun_out/$d/ \;
done
