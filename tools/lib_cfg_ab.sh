#!/bin/bash
# A/B of whole-library variants (VASR_LIB) on one box over bench configs, interleaved.
#   tools/lib_cfg_ab.sh <tag> <rounds> <lib.so>...     (configs: C2, C4 30 s, C3 bf16)
set -euo pipefail
TAG=$1; R=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
for r in $(seq 1 $R); do
  for cfg in "c2:" "c4:--seconds 30" "c3:--bf16"; do
    name=${cfg%%:*}; args=${cfg#*:}
    for lib in "$@"; do
      n=$(basename $lib .so)
      VASR_LIB=$lib timeout -k 10 200 python bench.py --inproc --no-cpu-baseline --no-scatter $args > $OUT/$name.$n.$r.json 2>/dev/null
      python -c "import json;d=json.load(open('$OUT/$name.$n.$r.json'));print('$name $n r$r',d['value'],d['ms_per_step'],d['roofline']['avg_launch_us'],d.get('rank0_tokens_match_reference'))" >> $OUT/summary.txt
    done
  done
done
