#!/bin/bash
# r06aj: the tile engine's shape choice at the one-graph C2 shapes (M = 16032): default picker vs always
# 128 x 128 where it divides (VASR_X3_MIN_TILES=1) vs always 64 x 64 (=100000), interleaved C2 lines.
set -uo pipefail
O=gpurun_out/r06aj; mkdir -p $O
export TMPDIR=/tmp
summ() { python3 -c "import json,sys; d=json.load(open('$1')); t=d['tokens_vs_reference'] or {}; s=d['config']['schedule'] or {}; print('$2', d['value'], d['ms_per_step'], s.get('ms_per_replay_by_streams'), t.get('all_ranks_pass'), d['machine']['clock_ghz'])"; }
run() { local name=$1; shift; timeout -k 10 300 python bench.py --inproc --no-cpu-baseline "$@" > $O/$name.json 2> $O/$name.err || { echo "$name rc $?"; tail -5 $O/$name.err; exit 1; }; summ $O/$name.json $name; }
for r in 1 2; do
run c2_def_$r
VASR_X3_MIN_TILES=1 run c2_big_$r
VASR_X3_MIN_TILES=100000 run c2_small_$r
done
