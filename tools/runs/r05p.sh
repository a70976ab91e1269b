#!/bin/bash
# r05p: the scan's in-kernel clock across process states: stamped scan build
# (VASR_SCAN_STAMPS) between rounds of C2 graph steps, before and after default bench lines.
set -uo pipefail
O=gpurun_out/r05p
mkdir -p $O
export TMPDIR=/tmp
VASR_LIB=tools/_variants/scan_stamps.so timeout -k 10 200 python -u tools/diag/scan_clock.py 15 200 20 > $O/clock1.txt 2>&1 || { echo "clock1 rc $?"; tail -5 $O/clock1.txt; exit 1; }
cat $O/clock1.txt
for i in 1 2; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench$i.json 2> $O/bench$i.err || { echo "bench rc $?"; tail -5 $O/bench$i.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench$i.json')); print(d['value'], d['ms_per_step'], d['machine'], d['roofline']['avg_launch_us'], d['config']['schedule']['ms_per_replay_by_streams'])"
done
VASR_LIB=tools/_variants/scan_stamps.so timeout -k 10 200 python -u tools/diag/scan_clock.py 40 200 20 > $O/clock2.txt 2>&1 || { echo "clock2 rc $?"; tail -5 $O/clock2.txt; exit 1; }
cat $O/clock2.txt
