#!/bin/bash
# r05aa: the two-group schedule with the 2-states-per-lane scan (16-clip launch = 768 blocks, three per CU, so
# the scan's "fewer chunks first" priority applies) vs the default 4-per-lane layout; C2 and C4, interleaved.
set -uo pipefail
O=gpurun_out/r05aa
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
for npl in 4 2; do
for cfg in "c2:" "c4:--seconds 30"; do
n=${cfg%%:*}; a=${cfg#*:}
VASR_SCAN_NPL=$npl timeout -k 10 300 python -u bench.py --no-cpu-baseline --streams 2 $a > $O/${n}_npl${npl}_$r.json 2> $O/${n}_npl${npl}_$r.err || { echo "$n $npl rc $?"; tail -3 $O/${n}_npl${npl}_$r.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/${n}_npl${npl}_$r.json')); print('$n npl$npl $r', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['machine']['clock_ghz'])"
done
done
done
