#!/bin/bash
# r05av: final-HEAD evidence after the ln_dwconv tile-height change.
# GPU suite, smoke, default bench lines, config lines, rocprofv3 of the default command and of the one-utterance line.
set -uo pipefail
O=gpurun_out/r05av
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1; rc=$?
tail -2 $O/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke rc $?"; tail -5 $O/smoke.txt; exit 1; }
echo smoke ok
for i in 1 2; do
timeout -k 10 300 python -u bench.py > $O/bench$i.json 2> $O/bench$i.err || { echo "bench rc $?"; tail -5 $O/bench$i.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench$i.json')); s=d['config']['schedule']; r=d['roofline']; print('c2', d['value'], d['ms_per_step'], s['chosen_streams'], s['ms_per_replay_by_streams'], r['avg_launch_us'], r['frac'], r.get('whole_batch_launch', {}).get('frac'), d['cpu_baseline']['value'] if d.get('cpu_baseline') else None, d['machine']['clock_ghz'])"
done
timeout -k 10 1500 bash tools/config_benches.sh r05av || { echo "configs rc $?"; exit 1; }
for f in gpurun_out/cfg_r05av/*.json; do python3 -c "import json; d=json.load(open('$f')); s=d['config'].get('schedule') or {}; print('$(basename $f .json)', d['value'], d['ms_per_step'], s.get('chosen_streams'), s.get('ms_per_replay_by_streams'), d['roofline']['avg_launch_us'], d['tokens_vs_reference']['all_ranks_pass'] if d.get('tokens_vs_reference') else None, d['machine']['clock_ghz'])"; done
timeout -k 10 1000 bash tools/profile.sh r05av || { echo "profile rc $?"; exit 1; }
mkdir -p gpurun_out/prof_r05av_b1 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r05av_b1/trace -o run --output-format csv -- python3 bench.py --inproc --batch 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_r05av_b1/b1.json 2> gpurun_out/prof_r05av_b1/b1.err || { echo "b1 prof rc $?"; exit 1; }
echo profile done
