#!/bin/bash
# r04as: round-end evidence at HEAD (pipelined tail) -- full GPU suite, smoke, the default bench line (autotuned
# schedule, CPU baseline included), both fixed schedules, BASELINE config lines, and the rocprofv3
# kernel-trace + HBM passes of the default bench command.
set -uo pipefail
O=gpurun_out/r04as
mkdir -p $O
export TMPDIR=/tmp
run() {
  local n=$1; shift
  "$@" > $O/$n.txt 2>&1; local rc=$?
  echo "rc $rc" >> $O/$n.txt
  [ $rc -eq 0 ] || { echo "$n failed rc $rc"; tail -15 $O/$n.txt; exit $rc; }
}
run gpu_tests timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run smoke timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
timeout -k 10 400 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo "bench rc $?"; tail -5 $O/bench_default.err; exit 1; }
timeout -k 10 300 python -u bench.py --streams 1 --no-cpu-baseline > $O/bench_s1.json 2> $O/bench_s1.err || { echo "s1 rc $?"; exit 1; }
timeout -k 10 300 python -u bench.py --streams 2 --no-cpu-baseline > $O/bench_s2.json 2> $O/bench_s2.err || { echo "s2 rc $?"; exit 1; }
bash tools/config_benches.sh r04as || { echo "config benches failed"; exit 1; }
bash tools/profile.sh r04as --steps 10 --warmup 3 --no-cpu-baseline || { echo "profile failed"; exit 1; }
grep -E "passed|failed" $O/gpu_tests.txt | tail -1; tail -2 $O/smoke.txt | head -1
for f in $O/bench_*.json gpurun_out/cfg_r04as/*.json; do python -c "import json; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], d['config'].get('schedule') and d['config']['schedule']['chosen_streams'], d['roofline']['avg_launch_us'], d['roofline']['frac'], (d['tokens_vs_reference'] or {}).get('clips_identical'), d['graph_tokens_match_eager'])"; done
