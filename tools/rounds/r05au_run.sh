# Copy form A/B: transform_fast's shape checks after the wait (fp0, the committed tree) vs right after
# the parse (fp1); fp1's library first through the transform GPU tests.
set -o pipefail
AMBRYCRC_LIBRARY=abl/fp1/libambrycrc.so AMBRYCRC_ALLOW_PROBE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_transform.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05au_fp1_tests.log 2>&1 || { echo FP1_TESTS_FAILED; tail -30 gpurun_out/r05au_fp1_tests.log; exit 1; }
tail -1 gpurun_out/r05au_fp1_tests.log
rm -rf gpurun_out/ab
LIBS="abl/fp0/libambrycrc.so abl/fp1/libambrycrc.so" CASES="xform4k" ROUNDS=4 REPS=5 timeout -k 10 400 bash tools/ab_cases.sh > gpurun_out/r05au_ab.log 2>&1 || { echo AB_FAILED; tail -5 gpurun_out/r05au_ab.log; exit 1; }
AB_MATCH=region_ python tools/ab_summary.py gpurun_out/ab
