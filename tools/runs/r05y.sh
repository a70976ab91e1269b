#!/bin/bash
# r05y: interleaved A/B of the round-start library (no scan wave priority) vs HEAD on C3 (bf16) and C4 (30 s),
# whose lines came out below round 4's in r05x.
set -uo pipefail
O=gpurun_out/r05y
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
for lib in base_r05m head_r05; do
for cfg in "c3:--bf16" "c4:--seconds 30"; do
n=${cfg%%:*}; a=${cfg#*:}
VASR_LIB=tools/_variants/$lib.so timeout -k 10 300 python -u bench.py --no-cpu-baseline $a > $O/${n}_${lib}_$r.json 2> $O/${n}_${lib}_$r.err || { echo "$n $lib rc $?"; tail -3 $O/${n}_${lib}_$r.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/${n}_${lib}_$r.json')); s=d['config']['schedule']; print('$n $lib $r', d['value'], d['ms_per_step'], s['chosen_streams'], s['ms_per_replay_by_streams'], d['roofline']['avg_launch_us'], d['machine']['clock_ghz'])"
done
done
done
