#!/bin/bash
# Round-5 evidence on one GPU box, each step under its own limit, stopping at the first failure:
# the long-record mix (tools/probes/long_mix.py), message verify per case and mode in separate
# processes, the 4 KiB transform (both verdicts), then every config's bench line (gpu_configs.sh).
set -o pipefail
TAG=${TAG:-r05f}
timeout -k 10 240 python tools/probes/long_mix.py > gpurun_out/${TAG}_longmix.json 2>&1 || { echo LONGMIX_FAILED; tail -5 gpurun_out/${TAG}_longmix.json; exit 1; }
tail -1 gpurun_out/${TAG}_longmix.json | cut -c1-400
for c in ${MSG_CASES:-4k 1k 100}; do
  for m in region2 region jobs; do
    timeout -k 10 150 python tools/bench_messages.py --cases $c --modes $m --reps 20 | grep -v '"C1' >> gpurun_out/${TAG}_messages.jsonl || { echo MSG_FAILED $c $m; exit 1; }
  done
done
grep -o '"config": "[^"]*"\|"mode_taken": "[^"]*"\|"ms_median": [0-9.]*' gpurun_out/${TAG}_messages.jsonl | paste - - -
timeout -k 10 200 python tools/bench_put.py --cases "" --transform 4k --reps 20 > gpurun_out/${TAG}_put.jsonl 2>&1 || { echo PUT_FAILED; exit 1; }
grep -o '"verdict": "[^"]*"\|"ms_median": [0-9.]*' gpurun_out/${TAG}_put.jsonl | paste - -
if [ -z "${NO_CONFIGS:-}" ]; then
  TAG=$TAG bash tools/gpu_configs.sh || { echo CONFIGS_FAILED; exit 1; }
  for f in gpurun_out/${TAG}_c*.json; do echo "$f: $(cut -c1-160 $f)"; done
fi
echo EVIDENCE_DONE
