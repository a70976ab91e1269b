#!/bin/bash
# r06v: the scan's chunk length in the two-group (two-stream) schedules: 16-step chunks forced
# (VASR_SCAN_T=16: 3 waves per SIMD, so the two groups' scans can share the SIMDs) vs the default
# (32-step chunks at <= 2 waves per SIMD for 16-clip launches), C4 (30 s) and C2, interleaved.
set -uo pipefail
O=gpurun_out/r06v; mkdir -p $O
export TMPDIR=/tmp
summ() { python3 -c "import json,sys; d=json.load(open('$1')); s=d['config']['schedule'] or {}; print('$2', d['value'], d['ms_per_step'], s.get('chosen_streams'), s.get('ms_per_replay_by_streams'), (d['tokens_vs_reference'] or {}).get('all_ranks_pass'), d['machine']['clock_ghz'])"; }
run() { local name=$1; shift; timeout -k 10 300 python bench.py --inproc --no-cpu-baseline "$@" > $O/$name.json 2> $O/$name.err || { echo "$name rc $?"; tail -5 $O/$name.err; exit 1; }; summ $O/$name.json $name; }
for r in 1 2; do
run c4_def_$r --seconds 30
VASR_SCAN_T=16 run c4_t16_$r --seconds 30
run c2_def_$r
VASR_SCAN_T=16 run c2_t16_$r
done
