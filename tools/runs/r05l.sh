#!/bin/bash
# r05l: HEAD check in a fresh container (library rebuilt here): GPU suite, one default bench line.
set -uo pipefail
O=gpurun_out/r05l
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1; rc=$?
tail -2 $O/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench1.json 2> $O/bench1.err || { echo "bench rc $?"; tail -5 $O/bench1.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench1.json')); print(d['value'], d['ms_per_step'], d['machine'], d['roofline']['avg_launch_us'], d['config']['schedule']['ms_per_replay_by_streams'])"
