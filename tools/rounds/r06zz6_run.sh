#!/bin/bash
# r06zz6: sweep rounds with a share ticket (rounds past the first take the next unclaimed share in
# batch order) vs the static round-robin (AMBRYCRC_WINDOW_TICKET=0): window / rounds / past-4-GiB parity
# tests and the multi-GPU tests (C5's 256 GiB shard), then C5 at N = 1 with each form, interleaved.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multi.py -m gpu -x -q --timeout 300 --timeout-method thread -k "window or rounds or 4gib or multi or gather or c5" > gpurun_out/r06zz6_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r06zz6_tests.log; exit 1; }
tail -n 2 gpurun_out/r06zz6_tests.log
for r in 1 2; do for tk in 0 1; do
AMBRYCRC_WINDOW_TICKET=$tk timeout -k 10 300 python bench.py --config c5 --steps 5 --warmup 1 --no-cpu-baseline --no-host-path > gpurun_out/r06zz6_c5_t${tk}_r$r.json 2> gpurun_out/r06zz6_c5_t${tk}_r$r.err || { echo C5_FAILED; tail -5 gpurun_out/r06zz6_c5_t${tk}_r$r.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print('ticket=$tk r$r', d['value'], d['ms_per_step'], r['kernel_avg_ms'], r['achieved'], r['measured_read_roof'])" gpurun_out/r06zz6_c5_t${tk}_r$r.json
done; done
echo R06ZZ6_DONE
