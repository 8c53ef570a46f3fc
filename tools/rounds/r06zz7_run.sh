#!/bin/bash
# r06zz7: C5 at N = 1 with the share ticket (r06zz6) at sweep windows of 8, 16 and 32 GiB (bench.py
# --window), interleaved twice.
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do for w in 8 16 32; do
timeout -k 10 300 python bench.py --config c5 --steps 5 --warmup 1 --no-cpu-baseline --no-host-path --window $((w << 30)) > gpurun_out/r06zz7_c5_w${w}_r$r.json 2> gpurun_out/r06zz7_c5_w${w}_r$r.err || { echo C5_FAILED; tail -5 gpurun_out/r06zz7_c5_w${w}_r$r.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print('window=${w}GiB r$r', d['value'], d['ms_per_step'], r['kernel_avg_ms'], r['achieved'], r['measured_read_roof'])" gpurun_out/r06zz7_c5_w${w}_r$r.json
done; done
echo R06ZZ7_DONE
