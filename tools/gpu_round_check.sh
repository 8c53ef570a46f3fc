set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02ap_gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r02ap_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r02ap_gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02ap_smoke.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/r02ap_bench.json 2> gpurun_out/r02ap_bench.err || exit 1
cat gpurun_out/r02ap_bench.json
LIBS="build/ab/base/libambrycrc.so build/ab/new/libambrycrc.so" CASES="batch100 batch1k msg4k" ROUNDS=2 REPS=5 timeout -k 10 400 bash tools/ab_cases.sh > gpurun_out/r02ap_ab.log 2>&1 || exit 1
echo AB_DONE
