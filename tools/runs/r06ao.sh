#!/bin/bash
# r06ao: z-in-tail also for the global SSM blocks (M = 2048 at C2: VASR_Z_IN_TAIL_MIN=1025) vs the
# default threshold (4097 rows): bitwise block check at M = 2048, interleaved C2 lines.
set -uo pipefail
O=gpurun_out/r06ao; mkdir -p $O
export TMPDIR=/tmp
summ() { python3 -c "import json,sys; d=json.load(open('$1')); t=d['tokens_vs_reference'] or {}; s=d['config']['schedule'] or {}; print('$2', d['value'], d['ms_per_step'], s.get('ms_per_replay_by_streams'), t.get('all_ranks_pass'), d['machine']['clock_ghz'])"; }
run() { local name=$1; shift; timeout -k 10 300 python bench.py --inproc --no-cpu-baseline "$@" > $O/$name.json 2> $O/$name.err || { echo "$name rc $?"; tail -5 $O/$name.err; exit 1; }; summ $O/$name.json $name; }
for r in 1 2 3; do
run c2_def_$r
VASR_Z_IN_TAIL_MIN=1025 run c2_glob_$r
done
