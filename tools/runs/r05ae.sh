#!/bin/bash
# r05ae: rows-engine column groups by a rounds x chunks cost model (M = 24048 / 48096 of the 30-s clips):
# C4 both schedules and C2, interleaved with the previous HEAD; the GPU GEMM tests.
set -uo pipefail
O=gpurun_out/r05ae
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_bench_workloads.py -m gpu -x -q --timeout 300 --timeout-method thread -k "gemm or rows or c4 or 30" > $O/tests.txt 2>&1; rc=$?
tail -2 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
for lib in head_up head_grp; do
for cfg in "c4:--seconds 30" "c2:"; do
n=${cfg%%:*}; a=${cfg#*:}
VASR_LIB=tools/_variants/$lib.so timeout -k 10 300 python -u bench.py --no-cpu-baseline $a > $O/${n}_${lib}_$r.json 2> $O/${n}_${lib}_$r.err || { echo "$n $lib rc $?"; tail -3 $O/${n}_${lib}_$r.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/${n}_${lib}_$r.json')); s=d['config']['schedule']; print('$n $lib $r', d['value'], d['ms_per_step'], s['chosen_streams'], s['ms_per_replay_by_streams'], d['roofline'].get('gemm_avg_launch_us'), d['machine']['clock_ghz'])"
done
done
done
