#!/bin/bash
# r06zz9: the share ticket's window, last sweep: C3 at 1 / 2 / 4 GiB, C2 (4 GiB total) at 1 / 2 / 4 GiB
# (4: one round), C5 at 4 / 8 GiB, interleaved twice.
set -o pipefail
mkdir -p gpurun_out
run() {  # config window_gib steps warmup round
  timeout -k 10 300 python bench.py --config $1 --steps $3 --warmup $4 --no-cpu-baseline --no-host-path --window $(($2 << 30)) > gpurun_out/r06zz9_$1_w$2_r$5.json 2> gpurun_out/r06zz9_$1_w$2_r$5.err || { echo FAILED $1 $2; tail -5 gpurun_out/r06zz9_$1_w$2_r$5.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print('$1 window=$2GiB r$5', d['value'], d['ms_per_step'], r['kernel_avg_ms'], r['achieved'], r['measured_read_roof'])" gpurun_out/r06zz9_$1_w$2_r$5.json
}
for r in 1 2; do
for w in 1 2 4; do run c3 $w 20 3 $r || exit 1; done
for w in 1 2 4; do run c2 $w 50 5 $r || exit 1; done
for w in 4 8; do run c5 $w 5 1 $r || exit 1; done
done
echo R06ZZ9_DONE
