#!/bin/bash
# r06ar: the tile picker taking 64 x 64 tiles for N <= 192 at any M: GEMM A/B (bitwise) at C2 / C4 shapes,
# then interleaved C2 and C4 lines.
set -uo pipefail
O=gpurun_out/r06ar; mkdir -p $O
export TMPDIR=/tmp
V=tools/_variants
timeout -k 10 300 python -u tools/gemm_ab_libs.py 5 16032:192:0:240,16032:192:0:192,48032:192:0:240,48032:192:0:192,8016:192:0:192 $V/pick_old.so $V/pick_new.so > $O/pick_ab.txt 2>&1 || { echo "ab rc $?"; tail -5 $O/pick_ab.txt; exit 1; }
cat $O/pick_ab.txt
summ() { python3 -c "import json,sys; d=json.load(open('$1')); t=d['tokens_vs_reference'] or {}; s=d['config']['schedule'] or {}; print('$2', d['value'], d['ms_per_step'], s.get('ms_per_replay_by_streams'), t.get('all_ranks_pass'), d['machine']['clock_ghz'])"; }
run() { local name=$1; shift; timeout -k 10 300 python bench.py --inproc --no-cpu-baseline "$@" > $O/$name.json 2> $O/$name.err || { echo "$name rc $?"; tail -5 $O/$name.err; exit 1; }; summ $O/$name.json $name; }
for r in 1 2; do
VASR_LIB=$PWD/$V/pick_old.so run c2_old_$r
VASR_LIB=$PWD/$V/pick_new.so run c2_new_$r
VASR_LIB=$PWD/$V/pick_old.so run c4_old_$r --seconds 30
VASR_LIB=$PWD/$V/pick_new.so run c4_new_$r --seconds 30
done
