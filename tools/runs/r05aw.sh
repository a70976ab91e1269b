#!/bin/bash
# C2 interleaved A/B: ln_dwconv tile height forced to 16 rows (round-start behaviour) vs the automatic choice.
set -euo pipefail
OUT=gpurun_out/r05aw; mkdir -p $OUT
for r in 1 2 3 4; do
  for rows in 16 0; do
    VASR_DW_ROWS=$rows timeout -k 10 200 python bench.py --no-cpu-baseline --no-scatter > $OUT/c2.$rows.$r.json 2>/dev/null
    python -c "import json;d=json.load(open('$OUT/c2.$rows.$r.json'));s=d['config']['schedule'];print('c2 rows=$rows r$r', d['value'], d['ms_per_step'], s['chosen_streams'], s['ms_per_replay_by_streams'])" >> $OUT/summary.txt
  done
done
cat $OUT/summary.txt
