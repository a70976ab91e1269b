#!/bin/bash
# r06ae: the composed bf16 projection as the default: bf16 tests, z-in-tail tests, C3 bench-shape edit
# rates, and the C3 / C2 bench lines.
set -uo pipefail
O=gpurun_out/r06ae; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_bf16.py tests/test_ssm_tail.py tests/test_bench_workloads.py tests/test_fused_argmax.py -m gpu -x -q --timeout 300 --timeout-method thread -s > $O/tests.txt 2>&1; rc=$?
tail -2 $O/tests.txt; grep "bf16 edit rate" $O/tests.txt | head -8; [ $rc -eq 0 ] || exit $rc
summ() { python3 -c "import json,sys; d=json.load(open('$1')); t=d['tokens_vs_reference'] or {}; print('$2', d['value'], d['ms_per_step'], d['kernels'].get('z_in_tail'), t.get('token_edit_rate'), t.get('all_ranks_pass'), d['machine']['clock_ghz'])"; }
timeout -k 10 300 python bench.py --inproc --no-cpu-baseline --bf16 > $O/c3.json 2> $O/c3.err || { echo "c3 rc $?"; tail -5 $O/c3.err; exit 1; }
summ $O/c3.json c3
