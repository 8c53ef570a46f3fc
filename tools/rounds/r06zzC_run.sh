#!/bin/bash
# r06zzC: the last check of the round on the tree as committed (product sources of 2bdf13f, rebuilt after the
# ticket experiment was reverted): the whole -m gpu suite, smoke, the default bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06zzC_gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r06zzC_gpu_tests.log; exit 1; }
tail -1 gpurun_out/r06zzC_gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06zzC_smoke.log 2>&1 || { echo SMOKE_FAILED; exit 1; }
tail -1 gpurun_out/r06zzC_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/r06zzC_bench.json 2> gpurun_out/r06zzC_bench.err || { echo BENCH_FAILED; tail -5 gpurun_out/r06zzC_bench.err; exit 1; }
cut -c1-300 gpurun_out/r06zzC_bench.json
echo R06ZZC_DONE
