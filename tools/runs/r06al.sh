#!/bin/bash
# r06al: XCD-aware tile order in ln_dwconv (each XCD writes the u rows the projection's workgroups on it
# read) vs blockIdx order: bitwise + isolated A/B, then interleaved C2 lines.
set -uo pipefail
O=gpurun_out/r06al; mkdir -p $O
export TMPDIR=/tmp
V=tools/_variants
timeout -k 10 300 python -u tools/dw_ab_libs.py 6 32:501,32:1501,1:501 $V/dwx0.so $V/dwx1.so > $O/dw_ab.txt 2>&1 || { echo "ab rc $?"; tail -5 $O/dw_ab.txt; exit 1; }
cat $O/dw_ab.txt
summ() { python3 -c "import json,sys; d=json.load(open('$1')); t=d['tokens_vs_reference'] or {}; s=d['config']['schedule'] or {}; print('$2', d['value'], d['ms_per_step'], s.get('ms_per_replay_by_streams'), t.get('all_ranks_pass'), d['machine']['clock_ghz'])"; }
run() { local name=$1; shift; timeout -k 10 300 python bench.py --inproc --no-cpu-baseline "$@" > $O/$name.json 2> $O/$name.err || { echo "$name rc $?"; tail -5 $O/$name.err; exit 1; }; summ $O/$name.json $name; }
for r in 1 2 3; do
VASR_LIB=$PWD/$V/dwx0.so run c2_d0_$r
VASR_LIB=$PWD/$V/dwx1.so run c2_d1_$r
done
