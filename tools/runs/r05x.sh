#!/bin/bash
# r05x: one line per BASELINE config at HEAD (scan wave priority), smoke, and the two-group stress test.
set -uo pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r05x.log 2>&1 || { echo "smoke rc $?"; tail -5 gpurun_out/smoke_r05x.log; exit 1; }
echo smoke ok
timeout -k 10 1500 bash tools/config_benches.sh r05x || { echo "configs rc $?"; exit 1; }
for f in gpurun_out/cfg_r05x/*.json; do python3 -c "import json; d=json.load(open('$f')); s=d['config'].get('schedule') or {}; print('$(basename $f .json)', d['value'], d['ms_per_step'], s.get('chosen_streams'), s.get('ms_per_replay_by_streams'), d['roofline']['avg_launch_us'], d['roofline']['frac'], d['tokens_vs_reference']['all_ranks_pass'] if d.get('tokens_vs_reference') else None)"; done
