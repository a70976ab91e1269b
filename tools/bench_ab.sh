#!/bin/bash
# A/B of one environment switch on the end-to-end bench (GPU box, from the repo root):
#   tools/bench_ab.sh VAR value1 value2 ...   (e.g. VASR_SCAN_NPL 4 0 4 0: interleaved repeats)
# Prints "VAR=value RTFx ms_per_step scan_us gemm_us" per run; logs in gpurun_out/ab_*.log.
set -euo pipefail
VAR=$1; shift
mkdir -p gpurun_out
i=0
for v in "$@"; do
  log=gpurun_out/ab_${VAR}_${v}_$i.log
  env "$VAR=$v" timeout -k 10 200 python bench.py --no-cpu-baseline > "$log" 2>&1
  tail -n 1 "$log" | python3 -c "
import sys, json
d = json.loads(sys.stdin.read())
k = d['kernels']
print('$VAR=$v', d['value'], d['ms_per_step'], k['scan']['avg_launch_us'], k['gemm']['avg_launch_us'])"
  i=$((i+1))
done
