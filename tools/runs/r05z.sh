#!/bin/bash
# r05z: interleaved A/B of the round-start library vs HEAD (scan wave priority) on C2, the default bench line.
set -uo pipefail
O=gpurun_out/r05z
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do
for lib in base_r05m head_r05; do
VASR_LIB=tools/_variants/$lib.so timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/c2_${lib}_$r.json 2> $O/c2_${lib}_$r.err || { echo "$lib rc $?"; tail -3 $O/c2_${lib}_$r.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/c2_${lib}_$r.json')); s=d['config']['schedule']; print('c2 $lib $r', d['value'], d['ms_per_step'], s['chosen_streams'], s['ms_per_replay_by_streams'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['machine']['clock_ghz'])"
done
done
