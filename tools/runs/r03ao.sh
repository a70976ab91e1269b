#!/bin/bash
# r03ao: concurrent-group replay mismatch after the chained first replays; one 32-clip graph vs two
# 16-clip groups (stress and end-to-end C2, interleaved).
set -uo pipefail
O=gpurun_out/r03ao
mkdir -p $O
timeout -k 10 250 python tools/diag/graph_stress.py caller 32 > $O/caller32.txt 2>&1
timeout -k 10 250 python tools/diag/graph_stress.py single 32 > $O/single32.txt 2>&1
grep -h MODE $O/caller32.txt $O/single32.txt
for i in 0 1; do
  for s in 2 1; do
    timeout -k 10 240 python bench.py --no-cpu-baseline --streams $s > $O/c2_s${s}_$i.json 2> $O/c2_s${s}_$i.err
    python3 -c "import json; d=json.loads(open('$O/c2_s${s}_$i.json').read().strip().splitlines()[-1]); t=d.get('tokens_vs_reference') or {}; print('streams', $s, round(d['value']), d['ms_per_step'], 'tokens', t.get('clips_identical'))" | tee -a $O/ab.txt
  done
done
