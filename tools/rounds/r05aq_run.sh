set -o pipefail
AMBRYCRC_LIBRARY=abl/fe1/libambrycrc.so AMBRYCRC_ALLOW_PROBE=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_messages.py tests/test_gpu_transform.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05aq_fe1_tests.log 2>&1 || { echo FE1_TESTS_FAILED; tail -30 gpurun_out/r05aq_fe1_tests.log; exit 1; }
tail -1 gpurun_out/r05aq_fe1_tests.log
rm -rf gpurun_out/ab
LIBS="abl/fe0/libambrycrc.so abl/fe1/libambrycrc.so" CASES="xform4k msg4k_1pass msg1k_1pass msg100_1pass" ROUNDS=3 REPS=5 timeout -k 10 500 bash tools/ab_cases.sh > gpurun_out/r05aq_ab.log 2>&1 || { echo AB_FAILED; tail -5 gpurun_out/r05aq_ab.log; exit 1; }
AB_MATCH=region_ python tools/ab_summary.py gpurun_out/ab
timeout -k 10 200 python -u -m pytest tests/test_gpu_host_policy.py tests/test_host_policy.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05aq_tests.log 2>&1 || { echo HOST_TESTS_FAILED; tail -20 gpurun_out/r05aq_tests.log; exit 1; }
tail -1 gpurun_out/r05aq_tests.log
timeout -k 10 300 python bench.py > gpurun_out/r05aq_bench.json 2> gpurun_out/r05aq_bench.err || { echo BENCH_FAILED; exit 1; }
python -c "
import json;d=json.load(open('gpurun_out/r05aq_bench.json'));print(d['value'], d['host_path']['dispatch'])"
