# Copy-form processor count with the record ends hashed after the parse (AMBRY_FUSED_ENDS 1):
# 262,144 x 4 KiB PUTs at 3 / 4 / 5 processor waves, twice each, then the larger transforms.
set -o pipefail
for r in 1 2; do for p in 3 4 5; do
  AMBRYCRC_FUSED_PROC=$p timeout -k 10 200 python tools/bench_put.py --transform 4k --copy-only > gpurun_out/r05as_p${p}_r${r}.jsonl 2>&1 || { echo FAILED p$p; tail -5 gpurun_out/r05as_p${p}_r${r}.jsonl; exit 1; }
  echo "p$p r$r $(grep -o '"ms_median": [0-9.]*' gpurun_out/r05as_p${p}_r${r}.jsonl | tr '\n' ' ')"
done; done
timeout -k 10 300 python tools/bench_put.py --transform 64k,4m --copy-only > gpurun_out/r05as_big.jsonl 2>&1 || { echo BIG_FAILED; exit 1; }
grep -o '"case": "[^"]*"\|"ms_median": [0-9.]*' gpurun_out/r05as_big.jsonl | paste - -
