#!/bin/bash
# r06ai: the global context's local-only work (query LayerNorm, q projection, the fusion's local product)
# on a side stream inside the graph (VASR_HGC_FORK=1) vs in line: composed-fusion tests with the fork,
# then interleaved C2 lines.
set -uo pipefail
O=gpurun_out/r06ai; mkdir -p $O
export TMPDIR=/tmp
VASR_HGC_FORK=1 timeout -k 10 300 python -u -m pytest tests/test_attention_compose.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1; rc=$?
tail -2 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
summ() { python3 -c "import json,sys; d=json.load(open('$1')); t=d['tokens_vs_reference'] or {}; s=d['config']['schedule'] or {}; print('$2', d['value'], d['ms_per_step'], s.get('ms_per_replay_by_streams'), t.get('all_ranks_pass'), d['machine']['clock_ghz'])"; }
run() { local name=$1; shift; timeout -k 10 300 python bench.py --inproc --no-cpu-baseline "$@" > $O/$name.json 2> $O/$name.err || { echo "$name rc $?"; tail -5 $O/$name.err; exit 1; }; summ $O/$name.json $name; }
for r in 1 2 3; do
VASR_HGC_FORK=0 run c2_line_$r
VASR_HGC_FORK=1 run c2_fork_$r
done
