#!/bin/bash
# r06zzA: the auto sweep window (4 GiB, shares >= 1 MiB, ticket) on the working tree: the whole -m gpu suite,
# smoke, then the default bench line (C3) and C5 / C2 at N = 1, each against HEAD's build (abtmp/head: one
# round at C3, 32 GiB static rounds at C5), interleaved.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06zzA_gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r06zzA_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r06zzA_gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06zzA_smoke.log 2>&1 || { echo SMOKE_FAILED; exit 1; }
tail -1 gpurun_out/r06zzA_smoke.log
run() {  # lib config steps warmup round
  AMBRYCRC_ALLOW_PROBE=1 AMBRYCRC_LIBRARY=$PWD/abtmp/$1/libambrycrc.so timeout -k 10 300 python bench.py --config $2 --steps $3 --warmup $4 --no-cpu-baseline --no-host-path > gpurun_out/r06zzA_$1_$2_r$5.json 2> gpurun_out/r06zzA_$1_$2_r$5.err || { echo FAILED $1 $2; tail -5 gpurun_out/r06zzA_$1_$2_r$5.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print('$1 $2 r$5', d['value'], d['ms_per_step'], r['kernel_avg_ms'], r['achieved'], r['measured_read_roof'])" gpurun_out/r06zzA_$1_$2_r$5.json
}
for r in 1 2; do for cfg in "c3 20 3" "c5 5 1" "c2 50 5"; do for lib in head win; do run $lib $cfg $r || exit 1; done; done; done
echo R06ZZA_DONE
