# One-pass A/B: processors parse a batch at once (ld0) or only once the stream is within LEAD bytes of it.
set -o pipefail
rm -rf gpurun_out/ab
LIBS="abl/ld0/libambrycrc.so abl/ld65536/libambrycrc.so abl/ld262144/libambrycrc.so abl/ld1048576/libambrycrc.so" CASES="xform4k msg4k_1pass" ROUNDS=3 REPS=5 timeout -k 10 700 bash tools/ab_cases.sh > gpurun_out/r05av_ab.log 2>&1 || { echo AB_FAILED; tail -5 gpurun_out/r05av_ab.log; exit 1; }
AB_MATCH=region_ python tools/ab_summary.py gpurun_out/ab
