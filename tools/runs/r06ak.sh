#!/bin/bash
# r06ak: XCD-aware tile order in the gated tail (each XCD a run of consecutive row tiles, as the scan's
# utterances) vs blockIdx order: bitwise + isolated A/B, then interleaved C2 lines (the L2 effect needs
# the scan's writes just before).
set -uo pipefail
O=gpurun_out/r06ak; mkdir -p $O
export TMPDIR=/tmp
V=tools/_variants
timeout -k 10 300 python -u tools/tail_ab_libs.py 6 16032,8016 f32 $V/tailg_xcd0.so $V/tailg_xcd1.so > $O/xcd_ab.txt 2>&1 || { echo "ab rc $?"; tail -5 $O/xcd_ab.txt; exit 1; }
cat $O/xcd_ab.txt
summ() { python3 -c "import json,sys; d=json.load(open('$1')); t=d['tokens_vs_reference'] or {}; s=d['config']['schedule'] or {}; print('$2', d['value'], d['ms_per_step'], s.get('ms_per_replay_by_streams'), t.get('all_ranks_pass'), d['machine']['clock_ghz'])"; }
run() { local name=$1; shift; timeout -k 10 300 python bench.py --inproc --no-cpu-baseline "$@" > $O/$name.json 2> $O/$name.err || { echo "$name rc $?"; tail -5 $O/$name.err; exit 1; }; summ $O/$name.json $name; }
for r in 1 2 3; do
VASR_LIB=$PWD/$V/tailg_xcd0.so run c2_x0_$r
VASR_LIB=$PWD/$V/tailg_xcd1.so run c2_x1_$r
done
