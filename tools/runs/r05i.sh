#!/bin/bash
# r05i: autotune rounds until settled, losing schedules freed after the timed steps: the
# concurrency tests and three default bench lines (per-step device times).
set -uo pipefail
O=gpurun_out/r05i
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_concurrent_gpu.py tests/test_fused_argmax.py -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1; rc=$?
tail -2 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench$i.json 2> $O/bench$i.err || { echo "bench rc $?"; tail -5 $O/bench$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench$i.json')); s=d['step_ms_device']; print(d['value'], d['ms_per_step'], d['machine']['clock_ghz'], s['device_ms'][:6], s['median'], d['config']['schedule']['rounds'])"
done
