#!/bin/bash
# r06af: the attention's out_proj folded into the gated fusion's global-branch product (default) vs separate:
# parity tests (stage goldens, logits, bf16, INT8, distributed), then interleaved C2 / C3 lines.
set -uo pipefail
O=gpurun_out/r06af; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1; rc=$?
tail -2 $O/tests.txt; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/tests.txt | head -20; exit $rc; }
summ() { python3 -c "import json,sys; d=json.load(open('$1')); t=d['tokens_vs_reference'] or {}; print('$2', d['value'], d['ms_per_step'], t.get('token_edit_rate'), t.get('all_ranks_pass'), d['machine']['clock_ghz'])"; }
run() { local name=$1; shift; timeout -k 10 300 python bench.py --inproc --no-cpu-baseline "$@" > $O/$name.json 2> $O/$name.err || { echo "$name rc $?"; tail -5 $O/$name.err; exit 1; }; summ $O/$name.json $name; }
for r in 1 2 3; do
VASR_ATTN_COMPOSE=0 run c2_sep_$r
VASR_ATTN_COMPOSE=1 run c2_comp_$r
done
