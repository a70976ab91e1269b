#!/bin/bash
# Utterance-group streams A/B on one box: 1 graph (32-clip launches) vs 2 concurrent 16-clip
# groups, interleaved, for C2 / C4 / C3.  Usage: tools/streams_ab.sh <tag> <rounds>
set -euo pipefail
TAG=${1:-streams}; R=${2:-3}
OUT=gpurun_out/$TAG; mkdir -p $OUT
for r in $(seq 1 $R); do
  for cfg in "c2:" "c4:--seconds 30" "c3:--bf16"; do
    name=${cfg%%:*}; args=${cfg#*:}
    for s in 1 2; do
      timeout -k 10 200 python bench.py --inproc --no-cpu-baseline --streams $s $args > $OUT/$name.s$s.$r.json 2>/dev/null
      python -c "import json;d=json.load(open('$OUT/$name.s$s.$r.json'));r=d['roofline'];print('$name s$s r$r',d['value'],d['ms_per_step'],r['frac'],r['avg_launch_us'])" >> $OUT/summary.txt
    done
  done
done
