#!/bin/bash
# r04ae: the N = 1 bench with the RCCL join deferred past the timed leg, interleaved with
# --inproc; the distributed GPU tests (launcher at N = 1 still joins RCCL for the serving leg).
set -uo pipefail
O=gpurun_out/r04ae
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_distributed_gpu.py -x -q --timeout 300 --timeout-method thread > $O/dist.txt 2>&1 || { echo "dist tests failed"; tail -20 $O/dist.txt; exit 1; }
tail -1 $O/dist.txt
i=0
for form in "" "--inproc" "" "--inproc" ""; do
  i=$((i+1))
  timeout -k 10 300 python -u bench.py --no-cpu-baseline $form > $O/b$i.json 2> $O/b$i.err || { echo "b$i rc $?"; exit 1; }
  python -c "import json; d=json.load(open('$O/b$i.json')); s=d['config'].get('schedule') or {}; w=d.get('with_scatter') or {}; print('b$i', '$form', d['value'], d['ms_per_step'], s.get('chosen_streams'), s.get('ms_per_replay_by_streams'), w.get('value'))"
done
