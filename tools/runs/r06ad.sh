#!/bin/bash
# r06ad: the bf16 model (C3) with the composed projection ([W_in,x; W_xdt W_in,x] as one bf16 GEMM,
# VASR_BF16_COMPOSE=1) vs the two GEMMs: interleaved C3 lines with the token edit rate vs the reference.
set -uo pipefail
O=gpurun_out/r06ad; mkdir -p $O
export TMPDIR=/tmp
summ() { python3 -c "import json,sys; d=json.load(open('$1')); t=d['tokens_vs_reference'] or {}; print('$2', d['value'], d['ms_per_step'], d['kernels'].get('z_in_tail'), t.get('token_edit_rate'), t.get('all_ranks_pass'), d['machine']['clock_ghz'])"; }
run() { local name=$1; shift; timeout -k 10 300 python bench.py --inproc --no-cpu-baseline "$@" > $O/$name.json 2> $O/$name.err || { echo "$name rc $?"; tail -5 $O/$name.err; exit 1; }; summ $O/$name.json $name; }
for r in 1 2 3; do
VASR_BF16_COMPOSE=0 run c3_two_$r --bf16
VASR_BF16_COMPOSE=1 run c3_comp_$r --bf16
done
