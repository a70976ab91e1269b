#!/bin/bash
# r04ad: is the autotuned default slower under the RCCL process group (the torchrun child at
# N = 1) than in-process?  Interleaved: default, --inproc, default, --inproc, --streams 1.
set -uo pipefail
O=gpurun_out/r04ad
mkdir -p $O
i=0
for form in "" "--inproc" "" "--inproc" "--streams 1" ""; do
  i=$((i+1))
  timeout -k 10 300 python -u bench.py --no-cpu-baseline $form > $O/b$i.json 2> $O/b$i.err || { echo "b$i rc $?"; exit 1; }
  python -c "import json; d=json.load(open('$O/b$i.json')); s=d['config'].get('schedule') or {}; print('b$i', '$form', d['value'], d['ms_per_step'], s.get('chosen_streams'), s.get('ms_per_replay_by_streams'))"
done
