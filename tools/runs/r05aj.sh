#!/bin/bash
# r05aj: two-group schedule with the B=16 scans' rotating priority in 0..1 instead of 0..2 (less VALU taken
# from the other group's co-resident GEMM / tail blocks): C2, C3, C4 with two groups forced, interleaved.
set -uo pipefail
O=gpurun_out/r05aj
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
for lib in head_p5 rot2; do
for cfg in "c2:" "c3:--bf16" "c4:--seconds 30"; do
n=${cfg%%:*}; a=${cfg#*:}
VASR_LIB=tools/_variants/$lib.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --streams 2 $a > $O/${n}_${lib}_$r.json 2> $O/${n}_${lib}_$r.err || { echo "$n $lib rc $?"; tail -3 $O/${n}_${lib}_$r.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/${n}_${lib}_$r.json')); print('$n $lib $r', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['machine']['clock_ghz'])"
done
done
done
