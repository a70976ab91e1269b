#!/bin/bash
# r06i: one bench line per BASELINE config at HEAD (C2, C3 bf16, C4 30 s, C5 INT8, one utterance), then
# z-in-tail on / off interleaved for C2 and C4.
set -uo pipefail
O=gpurun_out/r06i; mkdir -p $O
export TMPDIR=/tmp
summ() { python3 -c "import json,sys; d=json.load(open('$1')); r=d['roofline']; s=d['config']['schedule'] or {}; print('$2', d['value'], d['ms_per_step'], s.get('chosen_streams'), s.get('ms_per_replay_by_streams'), r['avg_launch_us'], r['frac'], d['kernels'].get('z_in_tail'), (d['tokens_vs_reference'] or {}).get('all_ranks_pass'), (d['tokens_vs_reference'] or {}).get('token_edit_rate'), d['machine']['clock_ghz'])"; }
run() { local name=$1; shift; timeout -k 10 300 python bench.py --inproc --no-cpu-baseline "$@" > $O/$name.json 2> $O/$name.err || { echo "$name rc $?"; tail -5 $O/$name.err; exit 1; }; summ $O/$name.json $name; }
run c2
run c3_bf16 --bf16
run c4_30s --seconds 30
run c5_int8 --int8
run b1_10s --batch 1 --steps 50 --warmup 10
run b1_30s --batch 1 --seconds 30 --steps 50 --warmup 10
for r in 1 2; do
for z in 0 1; do
VASR_Z_IN_TAIL=$z run c2_z${z}_$r
VASR_Z_IN_TAIL=$z run c4_z${z}_$r --seconds 30
done
done
