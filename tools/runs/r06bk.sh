#!/bin/bash
# r06bk: closing HEAD check (the library build() leaves): GPU suite, smoke, the default bench line, C3 line.
set -uo pipefail
O=gpurun_out/r06bk; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.txt 2>&1; rc=$?
tail -2 $O/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke rc $?"; tail -5 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench rc $?"; tail -5 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; print('c2', d['value'], d['ms_per_step'], r['avg_launch_us'], r['frac'], r['traffic'], d['cpu_baseline']['value'], d['tokens_vs_reference']['all_ranks_pass'], d['machine']['clock_ghz'])"
timeout -k 10 300 python -u bench.py --inproc --no-cpu-baseline --bf16 > $O/bench_c3.json 2> $O/bench_c3.err || { echo "c3 rc $?"; tail -5 $O/bench_c3.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_c3.json')); print('c3', d['value'], d['ms_per_step'], d['kernels'].get('z_in_tail'), d['tokens_vs_reference'].get('token_edit_rate'))"
