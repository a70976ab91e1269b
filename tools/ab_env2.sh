#!/bin/bash
# Env A/B of bench.py on one box (diagnostic): tools/ab_env2.sh <tag> <rounds> "<ENV=..>" "<ENV=..>" ...
set -euo pipefail
TAG=$1; R=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
for r in $(seq 1 $R); do
  i=0
  for e in "$@"; do
    i=$((i+1))
    env $e timeout -k 10 200 python bench.py --no-cpu-baseline --no-scatter > $OUT/bench.$i.$r.json 2> $OUT/bench.$i.$r.err
    python -c "import json;d=json.load(open('$OUT/bench.$i.$r.json'));print('$e',$r,d['value'],d['ms_per_step'],d['rank0_tokens_match_reference'])" >> $OUT/summary.txt
  done
done
