#!/bin/bash
# r04aj: final evidence at HEAD -- GPU suite, smoke, the default bench line (CPU baseline
# included) twice, the C2 bench through the N = 1 launcher with the serving leg.
set -uo pipefail
O=gpurun_out/r04aj
mkdir -p $O
run() {
  local n=$1; shift
  "$@" > $O/$n.txt 2>&1; local rc=$?
  echo "rc $rc" >> $O/$n.txt
  [ $rc -eq 0 ] || { echo "$n failed rc $rc"; tail -15 $O/$n.txt; exit $rc; }
}
run gpu_tests timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run smoke timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
for i in 1 2; do
  timeout -k 10 400 python -u bench.py > $O/bench$i.json 2> $O/bench$i.err || { echo "bench rc $?"; tail -5 $O/bench$i.err; exit 1; }
done
grep -E "passed|failed" $O/gpu_tests.txt | tail -1; grep "smoke ok" $O/smoke.txt
for f in $O/bench*.json; do python -c "import json; d=json.load(open('$f')); s=d['config']['schedule']; w=d.get('with_scatter') or {}; print('$f', d['value'], d['ms_per_step'], s['chosen_streams'], s['ms_per_replay_by_streams'], d['roofline']['frac'], d['tokens_vs_reference']['clips_identical'], d['graph_tokens_match_eager'], w.get('value'), d.get('cpu_baseline', {}).get('value'))"; done
