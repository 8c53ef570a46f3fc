#!/bin/bash
# r06zz8: the share ticket's window, continued: C5 at 2 / 4 / 8 GiB windows, and C3 (32 GiB, one round at
# the 32 GiB default) at 4 / 8 / 32 GiB windows, interleaved twice.
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
for w in 2 4 8; do
timeout -k 10 300 python bench.py --config c5 --steps 5 --warmup 1 --no-cpu-baseline --no-host-path --window $((w << 30)) > gpurun_out/r06zz8_c5_w${w}_r$r.json 2> gpurun_out/r06zz8_c5_w${w}_r$r.err || { echo C5_FAILED; tail -5 gpurun_out/r06zz8_c5_w${w}_r$r.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print('c5 window=${w}GiB r$r', d['value'], d['ms_per_step'], r['kernel_avg_ms'], r['achieved'], r['measured_read_roof'])" gpurun_out/r06zz8_c5_w${w}_r$r.json
done
for w in 4 8 32; do
timeout -k 10 300 python bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline --no-host-path --window $((w << 30)) > gpurun_out/r06zz8_c3_w${w}_r$r.json 2> gpurun_out/r06zz8_c3_w${w}_r$r.err || { echo C3_FAILED; tail -5 gpurun_out/r06zz8_c3_w${w}_r$r.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print('c3 window=${w}GiB r$r', d['value'], d['ms_per_step'], r['kernel_avg_ms'], r['achieved'], r['measured_read_roof'])" gpurun_out/r06zz8_c3_w${w}_r$r.json
done
done
echo R06ZZ8_DONE
