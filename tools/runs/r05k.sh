#!/bin/bash
# r05k: the warm-up reference check moved after the timed steps (no idle device between warm-up and timing):
# concurrency tests and three default bench lines (per-step device times).
set -uo pipefail
O=gpurun_out/r05k
mkdir -p $O
export TMPDIR=/tmp
true
true
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench$i.json 2> $O/bench$i.err || { echo "bench rc $?"; tail -5 $O/bench$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench$i.json')); s=d['step_ms_device']; print(d['value'], d['ms_per_step'], d['machine']['clock_ghz'], s['device_ms'][:6], s['median'], d['config']['schedule']['rounds'])"
done
