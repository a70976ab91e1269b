#!/bin/bash
# A/B of whole-library variants on one box (diagnostic): for each round, for each variant
# .so (VASR_LIB), the scan alone at 16 and 32 clips (mode 2) and one bench line.
#   tools/lib_ab.sh <tag> <rounds> <lib.so>...
set -euo pipefail
TAG=$1; R=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
for r in $(seq 1 $R); do
  for lib in "$@"; do
    n=$(basename $lib .so)
    for b in 16 32; do
      VASR_LIB=$lib timeout -k 10 60 python tools/scan_bench.py $b 501 384 64 2 200 2>/dev/null | sed "s/^/$n /" >> $OUT/scan.txt
    done
    VASR_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-scatter > $OUT/bench.$n.$r.json 2>/dev/null
    python -c "import json,sys;d=json.load(open('$OUT/bench.$n.$r.json'));print('$n',$r,d['value'],d['roofline']['avg_launch_us'])" >> $OUT/summary.txt
  done
done
