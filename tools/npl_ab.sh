#!/bin/bash
# Lane-layout A/B on one box (VASR_SCAN_NPL=2|4): scan alone at 16 / 32 clips and the bench.
set -euo pipefail
TAG=${1:-npl}; R=${2:-2}
OUT=gpurun_out/$TAG; mkdir -p $OUT
for r in $(seq 1 $R); do
  for npl in 4 2; do
    for b in 16 32; do
      VASR_SCAN_NPL=$npl timeout -k 10 60 python tools/scan_bench.py $b 501 384 64 2 200 2>/dev/null | sed "s/^/npl$npl /" >> $OUT/scan.txt
    done
    VASR_SCAN_NPL=$npl timeout -k 10 200 python bench.py --inproc --no-cpu-baseline > $OUT/bench.npl$npl.$r.json 2>/dev/null
    python -c "import json;d=json.load(open('$OUT/bench.npl$npl.$r.json'));print('npl$npl',$r,d['value'],d['roofline']['avg_launch_us'])" >> $OUT/summary.txt
  done
done
