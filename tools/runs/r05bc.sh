#!/bin/bash
# Tile-shape threshold of the split-bf16 tile GEMMs (VASR_X3_MIN_TILES: tiles a launch needs before
# the larger tile shape is taken; 0 = the built-in 1.9 / 1.4 per CU) at C2, interleaved.
set -uo pipefail
OUT=gpurun_out/r05bc; mkdir -p $OUT
for r in 1 2 3; do
  for mt in 0 1000 600; do
    VASR_X3_MIN_TILES=$mt timeout -k 10 200 python bench.py --no-cpu-baseline --no-scatter > $OUT/c2.$mt.$r.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('$OUT/c2.$mt.$r.json'));s=d['config']['schedule'];print('c2 mt=$mt r$r', d['value'], d['ms_per_step'], s['chosen_streams'], s['ms_per_replay_by_streams'])" >> $OUT/summary.txt
  done
done
cat $OUT/summary.txt
