#!/bin/bash
# r06a: round-6 start on a fresh box: GPU suite, smoke, default bench line, scan micro-bench (C2 / C4 shapes).
set -uo pipefail
O=gpurun_out/r06a; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1; rc=$?
tail -2 $O/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke rc $?"; tail -5 $O/smoke.txt; exit 1; }
echo smoke ok
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench rc $?"; tail -5 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; print('c2', d['value'], d['ms_per_step'], d['config']['schedule']['chosen_streams'], r['avg_launch_us'], r['frac'], d['cpu_baseline']['value'], d['tokens_vs_reference']['all_ranks_pass'], d['machine']['clock_ghz'])"
for r in 1 2 3; do
timeout -k 10 120 python tools/scan_bench.py 32 501 384 64 2 50 >> $O/scan.txt 2>&1 || exit 1
timeout -k 10 120 python tools/scan_bench.py 32 1501 384 64 2 20 >> $O/scan.txt 2>&1 || exit 1
done
cat $O/scan.txt
