# A/B of the one-pass region kernel's workgroup size (builds with -DAMBRY_FUSED_WAVES_VERIFY=W
# -DAMBRY_FUSED_WAVES_COPY=W under abtmp/fw<W>)
# and processor count: transform of 4 KiB PUTs (fast path) and one-pass verify of 4 KiB / 1 KiB /
# 100-B blob messages. Usage: bash tools/probes/fw_ab.sh <tag> "<W>:<P>[:<verify region mode>] ..." [rounds]
export AMBRYCRC_ALLOW_PROBE=1
tag=$1; cfgs=$2; rounds=${3:-2}
run() { # name lib proc [verify region mode]
  AMBRYCRC_LIBRARY=$PWD/abtmp/$2/libambrycrc.so AMBRYCRC_FUSED_PROC=$3 timeout -k 10 120 python tools/bench_put.py --cases "" --transform 4k --reps 10 > gpurun_out/${tag}_$1_x.jsonl 2>&1 &&
  AMBRYCRC_LIBRARY=$PWD/abtmp/$2/libambrycrc.so AMBRYCRC_FUSED_PROC=$3 timeout -k 10 120 python tools/bench_messages.py --cases 4k,1k,100 --modes $([ "${4:-1}" = 2 ] && echo region2 || echo region) > gpurun_out/${tag}_$1_v.jsonl 2>&1 &&
  echo "$1 x=$(grep -o '"ms_median": [0-9.]*' gpurun_out/${tag}_$1_x.jsonl | cut -d' ' -f2 | tr '\n' ' ') v=$(grep -o '"ms_median": [0-9.]*' gpurun_out/${tag}_$1_v.jsonl | cut -d' ' -f2 | tr '\n' ' ')"
}
for r in $(seq 1 $rounds); do
  for c in $cfgs; do
    IFS=: read -r w p m <<< "$c"
    run w${w}p${p}m${m:-1}_$r fw$w $p ${m:-1} || exit 1
  done
done
