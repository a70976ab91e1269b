#!/bin/bash
# r05v: falling wave priority in the fused tail (per product) and in the tile GEMM (per k-stage): tail launch
# times, then interleaved one-graph bench lines (--streams 1) of HEAD vs the variants.
set -uo pipefail
O=gpurun_out/r05v
mkdir -p $O
export TMPDIR=/tmp
for lib in head_r05 tailprio; do
VASR_LIB=tools/_variants/$lib.so timeout -k 10 120 python -u tools/diag/tail_time.py 501 8016 16032 >> $O/tail.txt 2>&1 || { echo "tail rc $?"; tail -3 $O/tail.txt; exit 1; }
done
grep "M=" $O/tail.txt
for r in 1 2 3; do
for lib in head_r05 tailprio x3prio both_prio; do
VASR_LIB=tools/_variants/$lib.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --streams 1 --steps 60 > $O/b_${lib}_$r.json 2> $O/b_${lib}_$r.err || { echo "bench $lib rc $?"; tail -3 $O/b_${lib}_$r.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/b_${lib}_$r.json')); print('$lib', $r, d['value'], d['ms_per_step'], d['step_ms_device']['median'], d['machine']['clock_ghz'])"
done
done
