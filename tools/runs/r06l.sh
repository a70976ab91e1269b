#!/bin/bash
# r06l: z-in-tail for the bf16 model (C3): the tail tests (fp32 + bf16 bitwise), then C3 with
# z-in-tail on / off interleaved (plus one C2 line as the box's clock reference).
set -uo pipefail
O=gpurun_out/r06l; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_ssm_tail.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/tail_tests.txt 2>&1; rc=$?
tail -3 $O/tail_tests.txt; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/tail_tests.txt | head -20; exit $rc; }
summ() { python3 -c "import json,sys; d=json.load(open('$1')); r=d['roofline']; s=d['config']['schedule'] or {}; k=d['kernels']; print('$2', d['value'], d['ms_per_step'], s.get('chosen_streams'), r['avg_launch_us'], r['frac'], k.get('z_in_tail'), k.get('ssm_tail_isolated_us'), (d['tokens_vs_reference'] or {}).get('all_ranks_pass'), (d['tokens_vs_reference'] or {}).get('token_edit_rate'), d['machine']['clock_ghz'])"; }
run() { local name=$1; shift; timeout -k 10 300 python bench.py --inproc --no-cpu-baseline "$@" > $O/$name.json 2> $O/$name.err || { echo "$name rc $?"; tail -5 $O/$name.err; exit 1; }; summ $O/$name.json $name; }
run c2
for r in 1 2 3; do
for z in 0 1; do
VASR_Z_IN_TAIL=$z run c3_z${z}_$r --bf16
done
done
