#!/bin/bash
# r06aq: one bench line per BASELINE config at the final HEAD on one box (C2, C3 bf16, C4 30 s, C5 INT8,
# one 10-s and one 30-s utterance).
set -uo pipefail
O=gpurun_out/r06aq; mkdir -p $O
export TMPDIR=/tmp
summ() { python3 -c "import json,sys; d=json.load(open('$1')); r=d['roofline']; s=d['config']['schedule'] or {}; t=d['tokens_vs_reference'] or {}; print('$2', d['value'], d['ms_per_step'], s.get('chosen_streams'), r['avg_launch_us'], r['frac'], t.get('all_ranks_pass'), t.get('token_edit_rate'), d['machine']['clock_ghz'])"; }
run() { local name=$1; shift; timeout -k 10 300 python bench.py --inproc --no-cpu-baseline "$@" > $O/$name.json 2> $O/$name.err || { echo "$name rc $?"; tail -5 $O/$name.err; exit 1; }; summ $O/$name.json $name; }
run c2
run c3_bf16 --bf16
run c4_30s --seconds 30
run c5_int8 --int8
run b1_10s --batch 1 --steps 50 --warmup 10
run b1_30s --batch 1 --seconds 30 --steps 50 --warmup 10
