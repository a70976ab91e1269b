#!/bin/bash
# r05h: host- vs device-paced steps (tools/diag/host_bound.py) and a default bench line with the
# per-step device and host times.
set -uo pipefail
O=gpurun_out/r05h
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/diag/host_bound.py > $O/host_bound.txt 2>&1 || { echo "host_bound rc $?"; tail -5 $O/host_bound.txt; exit 1; }
cat $O/host_bound.txt
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo "bench rc $?"; tail -5 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['machine'], d['step_ms_device'], d['config']['schedule']['ms_per_replay_by_streams'])"
