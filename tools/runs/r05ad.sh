#!/bin/bash
# r05ad: GEMM / tail kernels at wave priority 3 (above the scan's 0..3) in the two-group schedule: C4 and C2 with
# two groups forced, interleaved with HEAD.
set -uo pipefail
O=gpurun_out/r05ad
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
for lib in head_up mmaprio3; do
for cfg in "c4:--seconds 30" "c2:"; do
n=${cfg%%:*}; a=${cfg#*:}
VASR_LIB=tools/_variants/$lib.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --streams 2 $a > $O/${n}_${lib}_$r.json 2> $O/${n}_${lib}_$r.err || { echo "$n $lib rc $?"; tail -3 $O/${n}_${lib}_$r.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/${n}_${lib}_$r.json')); print('$n $lib $r', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['machine']['clock_ghz'])"
done
done
done
